// Stand-in for band/backend_factory.h (band/backend_factory.h:22-70): the
// static creator registry through which Band instantiates backends.
#pragma once
#include <map>
#include <memory>
#include <vector>

#include "band/common.h"
#include "band/device/cpu.h"
#include "band/interface/backend.h"
#include "band/interface/model.h"
#include "band/interface/model_executor.h"

namespace band {
template <typename Base, class... Args>
struct Creator {
 public:
  virtual ~Creator() = default;
  virtual Base* Create(Args...) const { return nullptr; }
};

class BackendFactory {
 public:
  static interface::IModelExecutor* CreateModelExecutor(
      BackendType backend, ModelId model_id, WorkerId worker_id, DeviceFlag device_flag,
      CpuSet thread_affinity_mask = BandCPUMaskGetSet(CPUMaskFlag::kAll), int num_threads = -1);
  static interface::IModel* CreateModel(BackendType backend, ModelId id);
  static interface::IBackendUtil* GetBackendUtil(BackendType backend);
  static std::vector<BackendType> GetAvailableBackends();
  static void RegisterBackendCreators(
      BackendType backend,
      Creator<interface::IModelExecutor, ModelId, WorkerId, DeviceFlag, CpuSet, int>* model_executor_creator,
      Creator<interface::IModel, ModelId>* model_creator,
      Creator<interface::IBackendUtil>* util_creator);
};
}  // namespace band
