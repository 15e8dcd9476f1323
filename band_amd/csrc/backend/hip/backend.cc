#include "backend/hip/backend.h"

#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <mutex>
#include <unordered_map>

#include "band_hip_backend.h"
#include "band_hip_kernels.h"

namespace band {
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
  return true;
}

// Strong definition of the symbol Band's factory references weakly.
bool TfLiteRegisterCreators() { return HipRegisterCreators(); }

}  // namespace band

namespace {
std::mutex g_ring_mu;
long long g_ring_pinned_bytes = 0;
std::unordered_map<void*, long long> g_ring_blocks;
}  // namespace

// request-ring slots in page-locked memory (include/band_hip_backend.h):
// the engine asks only for models a GPU worker runs whole, so batched and
// one-job passes DMA them directly (HipModelExecutor::ExecuteJobBatchDirect)
extern "C" void* bhx_ring_host_alloc(size_t bytes) {
  static const bool on = [] {
    const char* e = std::getenv("BAND_HIP_PINNED_RINGS");
    int n = 0;
    return !(e && e[0] == '0') && bh_device_count(&n) == 0 && n > 0;
  }();
  static const long long cap = [] {
    const char* e = std::getenv("BAND_HIP_PINNED_RING_MB");
    const long long mb = e ? std::atoll(e) : 8192;
    return (mb > 0 ? mb : 0) << 20;
  }();
  if (!on || bytes == 0) return nullptr;
  const long long b = static_cast<long long>(bytes);
  {
    std::lock_guard<std::mutex> lk(g_ring_mu);
    if (g_ring_pinned_bytes + b > cap) return nullptr;
    g_ring_pinned_bytes += b;
  }
  void* p = nullptr;
  if (bh_host_alloc(&p, bytes) != 0 || !p) {
    std::lock_guard<std::mutex> lk(g_ring_mu);
    g_ring_pinned_bytes -= b;
    return nullptr;
  }
  {
    std::lock_guard<std::mutex> lk(g_ring_mu);
    g_ring_blocks[p] = b;
  }
  band::hip::CountRingPages(p, bytes);
  return p;
}

extern "C" void bhx_ring_host_free(void* p) {
  if (!p) return;
  {
    std::lock_guard<std::mutex> lk(g_ring_mu);
    auto it = g_ring_blocks.find(p);
    if (it != g_ring_blocks.end()) {
      g_ring_pinned_bytes -= it->second;
      g_ring_blocks.erase(it);
    }
  }
  bh_host_free(p);
}
