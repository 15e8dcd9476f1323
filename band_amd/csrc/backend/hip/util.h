// HipUtil: IBackendUtil of the HIP backend (replaces TfLiteUtil,
// band/backend/tfl/util.cc:35-49).  kCPU is always available (Band needs a
// CPU worker to host every model: band/engine.cc:248-252); kGPU when a
// gfx950 device is visible.
#pragma once
#include <set>

#include "band/common.h"
#include "band/interface/backend.h"

namespace band {
namespace hip {
class HipUtil : public interface::IBackendUtil {
 public:
  std::set<DeviceFlag> GetAvailableDevices() const override;
};
}  // namespace hip
}  // namespace band
