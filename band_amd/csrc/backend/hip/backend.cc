#include "backend/hip/backend.h"

#include <cstdlib>

#include "band_hip_kernels.h"
#include "engine/tensor.h"

namespace band {

namespace {
// request-ring slots in page-locked memory when a GPU is present, so batched
// passes DMA them directly (HipModelExecutor::ExecuteJobBatchDirect);
// BAND_HIP_PINNED_RINGS=0 keeps them on the heap
void* RingAlloc(size_t bytes) {
  static const bool on = [] {
    const char* e = std::getenv("BAND_HIP_PINNED_RINGS");
    int n = 0;
    return !(e && e[0] == '0') && bh_device_count(&n) == 0 && n > 0;
  }();
  void* p = nullptr;
  if (!on || bh_host_alloc(&p, bytes) != 0) return nullptr;
  return p;
}
void RingFree(void* p) { bh_host_free(p); }
}  // namespace

bool HipRegisterCreators() {
  BackendFactory::RegisterBackendCreators(BackendType::kTfLite, new hip::ModelExecutorCreator,
                                          new hip::ModelCreator, new hip::UtilCreator);
  RingHostAllocator a;
  a.alloc = RingAlloc;
  a.free = RingFree;
  SetRingHostAllocator(a);
  return true;
}

// Strong definition of the symbol Band's factory references weakly.
bool TfLiteRegisterCreators() { return HipRegisterCreators(); }

}  // namespace band
