// band::Model: one logical model with a backend model per BackendType
// (band/model.h/.cc).  Ids come from a process-wide counter.
#pragma once
#include <map>
#include <memory>
#include <set>

#include "absl/status/status.h"
#include "band/interface/model.h"

namespace band {

class Model {
 public:
  Model();
  ModelId GetId() const { return model_id_; }
  absl::Status FromPath(BackendType backend_type, const char* filename);
  absl::Status FromBuffer(BackendType backend_type, const char* buffer, size_t buffer_size);
  interface::IModel* GetBackendModel(BackendType backend_type);
  std::set<BackendType> GetSupportedBackends() const;

 private:
  const ModelId model_id_;
  std::map<BackendType, std::shared_ptr<interface::IModel>> backend_models_;
};

}  // namespace band
