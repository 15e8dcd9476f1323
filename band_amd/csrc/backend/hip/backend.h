// Creators + registration of the HIP backend (replaces band/backend/tfl/backend.{h,cc}).
//
// Drop-in choice: the HIP backend registers itself under BackendType::kTfLite
// by providing the strong definition of `band::TfLiteRegisterCreators()`,
// the weak symbol Band's BackendFactory calls (band/backend_factory.cc:10-33).
// Linking band/backend/hip instead of band/backend/tfl therefore swaps the
// backend with no change to Band's engine, configs or C API (kBandTfLite).
#pragma once

#include "backend/hip/model.h"
#include "backend/hip/model_executor.h"
#include "backend/hip/util.h"
#include "band/backend_factory.h"

namespace band {
namespace hip {

class ModelExecutorCreator
    : public Creator<interface::IModelExecutor, ModelId, WorkerId, DeviceFlag, CpuSet, int> {
 public:
  interface::IModelExecutor* Create(ModelId model_id, WorkerId worker_id, DeviceFlag device_flag,
                                    CpuSet mask, int num_threads) const override {
    return new HipModelExecutor(model_id, worker_id, device_flag, mask, num_threads);
  }
};

class ModelCreator : public Creator<interface::IModel, ModelId> {
 public:
  interface::IModel* Create(ModelId id) const override { return new HipModel(id); }
};

class UtilCreator : public Creator<interface::IBackendUtil> {
 public:
  interface::IBackendUtil* Create() const override { return new HipUtil(); }
};

// page-locked request-ring memory per NUMA node (bhx_ring_page_nodes):
// CountRingPages samples a new ring block, RingPageNodes reads the totals
void CountRingPages(const void* p, size_t bytes);
int RingPageNodes(long long* bytes_per_node, int cap);

}  // namespace hip

bool TfLiteRegisterCreators();
bool HipRegisterCreators();

}  // namespace band
