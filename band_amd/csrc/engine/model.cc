#include "engine/model.h"

#include <atomic>

#include "band/backend_factory.h"

namespace band {

namespace {
std::atomic<int> g_next_id{0};
}

Model::Model() : model_id_(g_next_id++) {}

absl::Status Model::FromPath(BackendType backend_type, const char* filename) {
  if (GetBackendModel(backend_type))
    return absl::InternalError(std::string("Tried to create ") + ToString(backend_type) + " model again for model id " +
                               std::to_string(model_id_));
  std::shared_ptr<interface::IModel> m(BackendFactory::CreateModel(backend_type, model_id_));
  if (!m || !m->FromPath(filename).ok())
    return absl::InternalError(std::string("Failed to create ") + ToString(backend_type) + " model from " + filename);
  backend_models_[backend_type] = m;
  return absl::OkStatus();
}

absl::Status Model::FromBuffer(BackendType backend_type, const char* buffer, size_t buffer_size) {
  if (GetBackendModel(backend_type))
    return absl::InternalError(std::string("Tried to create ") + ToString(backend_type) + " model again for model id " +
                               std::to_string(model_id_));
  std::shared_ptr<interface::IModel> m(BackendFactory::CreateModel(backend_type, model_id_));
  if (!m || !m->FromBuffer(buffer, buffer_size).ok())
    return absl::InternalError(std::string("Failed to create ") + ToString(backend_type) + " model from buffer");
  backend_models_[backend_type] = m;
  return absl::OkStatus();
}

interface::IModel* Model::GetBackendModel(BackendType backend_type) {
  auto it = backend_models_.find(backend_type);
  return it == backend_models_.end() ? nullptr : it->second.get();
}

std::set<BackendType> Model::GetSupportedBackends() const {
  std::set<BackendType> s;
  for (const auto& kv : backend_models_) s.insert(kv.first);
  return s;
}

}  // namespace band
