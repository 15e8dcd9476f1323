// Where a CU-masked stream's workgroups run on MI355X
// (hipExtStreamCreateWithCUMask): for several 256-bit masks, launches
// 2048 one-wave workgroups that spin ~20 us each, records every
// workgroup's XCC_ID and HW_ID (s_getreg, register reads only), and prints
// the workgroups per XCD, the distinct CUs used and the elapsed time.
// Question answered: does mask bit k select CU k of XCD k / 32, or of
// XCD k % 8 - i.e. can a stream be confined to whole XCDs.
// build: hipcc -O2 --offload-arch=gfx950 tools/cumask_probe.hip -o tools/cumask_probe
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cstdio>
#include <set>
#include <vector>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));         \
      return 1;                                                            \
    }                                                                      \
  } while (0)

__global__ void where_kernel(unsigned* out, long long spin) {
  if (threadIdx.x == 0) {
    const unsigned xcc = __builtin_amdgcn_s_getreg((3 << 11) | 20);  // HW_REG_XCC_ID [3:0]
    const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_REG_HW_ID
    out[2 * blockIdx.x] = xcc;
    out[2 * blockIdx.x + 1] = hw;
  }
  const long long t0 = clock64();
  while (clock64() - t0 < spin) {
  }
}

int main() {
  const int nwg = 2048;
  unsigned* d = nullptr;
  CK(hipMalloc(&d, nwg * 2 * sizeof(unsigned)));
  struct M {
    const char* name;
    std::vector<uint32_t> m;
  };
  std::vector<M> masks = {
      {"all 256", std::vector<uint32_t>(8, 0xffffffffu)},
      {"bits 0-31", {0xffffffffu, 0, 0, 0, 0, 0, 0, 0}},
      {"bits 0-63", {0xffffffffu, 0xffffffffu, 0, 0, 0, 0, 0, 0}},
      {"every 8th bit (0, 8, ..)", std::vector<uint32_t>(8, 0x01010101u)},
      {"bits 0-127", {0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0, 0, 0, 0}},
  };
  std::vector<unsigned> h(nwg * 2);
  for (auto& mk : masks) {
    hipStream_t s;
    CK(hipExtStreamCreateWithCUMask(&s, (uint32_t)mk.m.size(), mk.m.data()));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    hipLaunchKernelGGL(where_kernel, dim3(nwg), dim3(64), 0, s, d, 40000LL);  // warm
    CK(hipStreamSynchronize(s));
    CK(hipEventRecord(e0, s));
    hipLaunchKernelGGL(where_kernel, dim3(nwg), dim3(64), 0, s, d, 40000LL);
    CK(hipEventRecord(e1, s));
    CK(hipStreamSynchronize(s));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    CK(hipMemcpy(h.data(), d, h.size() * sizeof(unsigned), hipMemcpyDeviceToHost));
    int per_xcc[16] = {0};
    std::set<unsigned> cus[16];
    for (int i = 0; i < nwg; ++i) {
      const unsigned x = h[2 * i] & 15, hw = h[2 * i + 1];
      per_xcc[x]++;
      cus[x].insert((hw >> 8) & 0xff);  // cu_id | sh_id | se_id
    }
    std::printf("%-26s %8.1f us  WGs per XCC:", mk.name, ms * 1e3);
    for (int x = 0; x < 8; ++x) std::printf(" %4d", per_xcc[x]);
    std::printf("  | CUs per XCC:");
    for (int x = 0; x < 8; ++x) std::printf(" %2zu", cus[x].size());
    std::printf("\n");
    CK(hipStreamDestroy(s));
  }
  CK(hipFree(d));
  return 0;
}
