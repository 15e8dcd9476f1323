#include "backend/hip/backend.h"

#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
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
  hip::CountRingPages(p, bytes);
  return p;
}
void RingFree(void* p) { bh_host_free(p); }
}  // namespace

namespace hip {
namespace {
constexpr int kMaxNodes = 64;
std::atomic<long long> g_ring_node_bytes[kMaxNodes + 1];  // [kMaxNodes]: node unknown
}  // namespace

void CountRingPages(const void* p, size_t bytes) {
  // NUMA node of every 16th page (get_mempolicy MPOL_F_NODE | MPOL_F_ADDR);
  // page-locked memory is resident, so the node is settled
  const size_t page = 4096, step = 16 * page;
  for (size_t off = 0; off < bytes; off += step) {
    int node = -1;
    const long rc = syscall(SYS_get_mempolicy, &node, nullptr, 0UL,
                            const_cast<char*>(static_cast<const char*>(p)) + off, 3UL);
    const int slot = (rc == 0 && node >= 0 && node < kMaxNodes) ? node : kMaxNodes;
    g_ring_node_bytes[slot] += static_cast<long long>(std::min(step, bytes - off));
  }
}

int RingPageNodes(long long* bytes_per_node, int cap) {
  int n = 0;
  for (int i = 0; i <= kMaxNodes; ++i)
    if (g_ring_node_bytes[i].load()) n = i + 1;
  for (int i = 0; i < cap && i < n; ++i) bytes_per_node[i] = g_ring_node_bytes[i].load();
  return n;
}
}  // namespace hip

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
