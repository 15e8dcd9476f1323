// Diagnostic (not part of the product): how dependent kernel streams scale
// when S of them run at once, with no host work in between.  Each stream
// runs N back-to-back launches of one synthetic kernel; the aggregate
// launches/s for S = 1, 2, 4, 8 shows whether concurrent passes interfere
// through the queues / dispatcher (an empty kernel), through the CUs'
// latency hiding (a sleep kernel that only waits), or through VALU issue (a
// kernel that only computes).
// build: hipcc --offload-arch=gfx950 -O2 tools/queue_probe.hip -o tools/queue_probe
// usage: queue_probe <empty|sleep|valu> [workgroups=300] [threads=256] [launches=2000]
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#define CK(x)                                                                            \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) {                                                              \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(2);                                                                      \
    }                                                                                    \
  } while (0)

__global__ void k_empty(int* out) {}

// ~8 us of waiting per wave (s_sleep 127 ~ 8k cycles at 64 cycles per unit)
__global__ void k_sleep(int* out) {
  for (int i = 0; i < 1; ++i) __builtin_amdgcn_s_sleep(127);
  if (threadIdx.x == 0 && blockIdx.x == 0 && out) out[0] = 1;
}

// ~4k dependent VALU ops per lane
__global__ void k_valu(int* out) {
  unsigned v = threadIdx.x * 2654435761u + blockIdx.x;
#pragma unroll 8
  for (int i = 0; i < 4096; ++i) v = v * 1664525u + 1013904223u;
  if (v == 0x12345678u && out) out[blockIdx.x] = (int)v;  // keeps the loop
}

int main(int argc, char** argv) {
  const char* mode = argc > 1 ? argv[1] : "empty";
  const int wgs = argc > 2 ? std::atoi(argv[2]) : 300;
  const int threads = argc > 3 ? std::atoi(argv[3]) : 256;
  const int n = argc > 4 ? std::atoi(argv[4]) : 2000;
  void (*k)(int*) = std::strcmp(mode, "sleep") == 0 ? k_sleep : std::strcmp(mode, "valu") == 0 ? k_valu : k_empty;
  int* buf = nullptr;
  CK(hipMalloc(&buf, 1 << 20));
  std::vector<hipStream_t> st(8);
  for (auto& s : st) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  // warm up every stream
  for (auto& s : st) {
    hipLaunchKernelGGL(k, dim3(wgs), dim3(threads), 0, s, buf);
    CK(hipStreamSynchronize(s));
  }
  double base = 0;
  for (int S : {1, 2, 4, 8}) {
    auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> th;
    for (int i = 0; i < S; ++i)
      th.emplace_back([&, i] {
        for (int j = 0; j < n; ++j) hipLaunchKernelGGL(k, dim3(wgs), dim3(threads), 0, st[i], buf);
        (void)hipStreamSynchronize(st[i]);
      });
    for (auto& t : th) t.join();
    const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    const double rate = S * n / s;
    if (S == 1) base = rate;
    std::printf("%s wgs %d x %d: streams %d  %9.0f launches/s  %6.2f us/launch/stream  x%.2f\n", mode, wgs, threads,
                S, rate, 1e6 * s / n, rate / base);
    std::fflush(stdout);
  }
  CK(hipFree(buf));
  return 0;
}
