// Diagnostic: does a large by-value kernel argument (the chain kernels pass
// bh_chain_params, ~0.7 KB) cost dispatch time in a dependent hipGraph
// chain?  N dependent launches of a 1-workgroup kernel that reads one word
// of its argument, kernarg sizes 16 B .. 2 KB, eager and graph.
#include <hip/hip_runtime.h>
#include <cstdio>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { std::printf("%s -> %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

template <int B>
struct Arg {
  int v[B / 4];
};

template <int B>
__global__ void k_arg(Arg<B> a, int* out) {
  if (threadIdx.x == 0) out[0] += a.v[(B / 4) - 1];
}

template <int B>
static int run(hipStream_t st, int* out, hipEvent_t e0, hipEvent_t e1) {
  const int N = 400;
  Arg<B> a{};
  a.v[B / 4 - 1] = 1;
  for (int graph = 0; graph < 2; ++graph) {
    hipGraphExec_t ex = nullptr;
    if (graph) {
      hipGraph_t g;
      CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
      for (int i = 0; i < N; ++i) k_arg<B><<<1, 64, 0, st>>>(a, out);
      CK(hipStreamEndCapture(st, &g));
      CK(hipGraphInstantiate(&ex, g, nullptr, nullptr, 0));
      CK(hipGraphLaunch(ex, st));
    }
    for (int rep = 0; rep < 3; ++rep) {
      CK(hipStreamSynchronize(st));
      CK(hipEventRecord(e0, st));
      if (graph) CK(hipGraphLaunch(ex, st));
      else
        for (int i = 0; i < N; ++i) k_arg<B><<<1, 64, 0, st>>>(a, out);
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (rep == 2) std::printf("kernarg %5d B  %s  %.2f us per launch\n", B + 8, graph ? "graph" : "eager", 1e3 * ms / N);
    }
  }
  return 0;
}

int main() {
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  int* out;
  CK(hipMalloc(&out, 256));
  CK(hipMemset(out, 0, 256));
  if (run<16>(st, out, e0, e1) || run<256>(st, out, e0, e1) || run<768>(st, out, e0, e1) ||
      run<2048>(st, out, e0, e1))
    return 1;
  return 0;
}
