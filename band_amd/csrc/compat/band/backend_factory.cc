// Stand-in registry (band/backend_factory.cc:19-98 semantics): backends
// register once through a registration function reached via a weak symbol;
// Create* hand out raw `new` objects owned by the caller.
#include "band/backend_factory.h"

#include <mutex>

namespace band {
// Band resolves this weak symbol to the backend linked into the binary; the
// HIP backend provides the strong definition (backend/hip/backend.cc).
bool TfLiteRegisterCreators() __attribute__((weak));

namespace {
using ExecCreator = Creator<interface::IModelExecutor, ModelId, WorkerId, DeviceFlag, CpuSet, int>;
using ModelCreator = Creator<interface::IModel, ModelId>;
using UtilCreator = Creator<interface::IBackendUtil>;
std::map<BackendType, std::shared_ptr<ExecCreator>>& Execs() { static std::map<BackendType, std::shared_ptr<ExecCreator>> m; return m; }
std::map<BackendType, std::shared_ptr<ModelCreator>>& Models() { static std::map<BackendType, std::shared_ptr<ModelCreator>> m; return m; }
std::map<BackendType, std::shared_ptr<UtilCreator>>& Utils() { static std::map<BackendType, std::shared_ptr<UtilCreator>> m; return m; }
std::once_flag g_once;
void RegisterAll() {
  std::call_once(g_once, [] {
    if (TfLiteRegisterCreators) TfLiteRegisterCreators();
  });
}
}  // namespace

interface::IModelExecutor* BackendFactory::CreateModelExecutor(BackendType backend, ModelId model_id,
                                                               WorkerId worker_id, DeviceFlag device_flag,
                                                               CpuSet mask, int num_threads) {
  RegisterAll();
  auto it = Execs().find(backend);
  return it == Execs().end() ? nullptr : it->second->Create(model_id, worker_id, device_flag, mask, num_threads);
}
interface::IModel* BackendFactory::CreateModel(BackendType backend, ModelId id) {
  RegisterAll();
  auto it = Models().find(backend);
  return it == Models().end() ? nullptr : it->second->Create(id);
}
interface::IBackendUtil* BackendFactory::GetBackendUtil(BackendType backend) {
  RegisterAll();
  auto it = Utils().find(backend);
  return it == Utils().end() ? nullptr : it->second->Create();
}
std::vector<BackendType> BackendFactory::GetAvailableBackends() {
  RegisterAll();
  std::vector<BackendType> v;
  for (auto& kv : Execs()) v.push_back(kv.first);
  return v;
}
void BackendFactory::RegisterBackendCreators(BackendType backend, ExecCreator* e, ModelCreator* m, UtilCreator* u) {
  Execs()[backend] = std::shared_ptr<ExecCreator>(e);
  Models()[backend] = std::shared_ptr<ModelCreator>(m);
  Utils()[backend] = std::shared_ptr<UtilCreator>(u);
}
}  // namespace band
