// Band backend plugin API (stand-in; signatures of band/interface/model.h:17-38).
#pragma once
#include <string>

#include "absl/status/status.h"
#include "band/common.h"
#include "band/interface/backend.h"

namespace band {
namespace interface {
struct IModel : public IBackendSpecific {
 public:
  IModel(ModelId id) : id_(id) {}
  virtual ~IModel() = default;
  virtual absl::Status FromPath(const char* filename) = 0;
  virtual absl::Status FromBuffer(const char* buffer, size_t buffer_size) = 0;
  virtual bool IsInitialized() const = 0;
  ModelId GetId() const { return id_; }
  const std::string& GetPath() const { return path_; }

 protected:
  std::string path_;
  const ModelId id_;
};
}  // namespace interface
}  // namespace band
