// Band backend plugin API (stand-in; signatures of band/interface/backend.h:6-26).
#pragma once
#include <set>

#include "band/common.h"

namespace band {
namespace interface {
class IBackendSpecific {
 public:
  virtual BackendType GetBackendType() const = 0;
  bool IsCompatible(const IBackendSpecific& rhs) const { return IsCompatible(&rhs); }
  bool IsCompatible(const IBackendSpecific* rhs) const { return GetBackendType() == rhs->GetBackendType(); }
};

class IBackendUtil {
 public:
  virtual ~IBackendUtil() = default;
  virtual std::set<DeviceFlag> GetAvailableDevices() const = 0;
};
}  // namespace interface
}  // namespace band
