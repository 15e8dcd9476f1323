// Diagnostic: cost of a dependent kernel launch on this device, to separate
// launch/graph overhead from in-kernel latency (not part of the product).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { std::printf("%s -> %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__global__ void k_empty() {}

// each workgroup reads `bytes_per_wg` written by the previous launch and
// writes the same amount for the next one
__global__ void k_chain(const int* __restrict__ in, int* __restrict__ out, int words_per_wg) {
  const int base = blockIdx.x * words_per_wg;
  int s = 0;
  for (int i = threadIdx.x; i < words_per_wg; i += blockDim.x) s += in[base + i];
  for (int i = threadIdx.x; i < words_per_wg; i += blockDim.x) out[base + i] = s + i;
}

int main() {
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  int *a, *b;
  CK(hipMalloc(&a, 64 << 20));
  CK(hipMalloc(&b, 64 << 20));
  CK(hipMemset(a, 0, 64 << 20));
  CK(hipMemset(b, 0, 64 << 20));
  const int N = 200;
  struct Cfg { const char* name; int grid, block, words; };
  std::vector<Cfg> cfgs = {{"empty 1x64", 1, 64, 0}, {"empty 256x256", 256, 256, 0},
                           {"chain 1x64 256B", 1, 64, 64}, {"chain 256x256 4KB/wg", 256, 256, 1024},
                           {"chain 64x256 4KB/wg", 64, 256, 1024}, {"chain 1024x256 4KB/wg", 1024, 256, 1024},
                           {"chain 256x256 64KB/wg", 256, 256, 16384}};
  for (const Cfg& c : cfgs) {
    for (int graph = 0; graph < 2; ++graph) {
      auto issue = [&]() {
        for (int i = 0; i < N; ++i) {
          if (c.words == 0) hipLaunchKernelGGL(k_empty, dim3(c.grid), dim3(c.block), 0, st);
          else hipLaunchKernelGGL(k_chain, dim3(c.grid), dim3(c.block), 0, st, (i & 1) ? b : a, (i & 1) ? a : b, c.words);
        }
      };
      hipGraphExec_t ge = nullptr;
      if (graph) {
        hipGraph_t g;
        CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
        issue();
        CK(hipStreamEndCapture(st, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        CK(hipGraphDestroy(g));
      }
      float best = 1e30f;
      for (int rep = 0; rep < 5; ++rep) {
        CK(hipEventRecord(e0, st));
        if (graph) CK(hipGraphLaunch(ge, st)); else issue();
        CK(hipEventRecord(e1, st));
        CK(hipStreamSynchronize(st));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (ms < best) best = ms;
      }
      std::printf("%-26s %-6s %7.2f us/launch\n", c.name, graph ? "graph" : "stream", best * 1e3f / N);
      if (ge) CK(hipGraphExecDestroy(ge));
    }
  }
  return 0;
}
