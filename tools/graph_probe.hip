// Minimal reproducer for the rocprofv3 crashes seen while profiling bench.py
// ("Profiler crashes"): captures a stream into a hipGraph
// the way HipModelExecutor does and replays it, with one variable changed per
// mode, so the tool's failure can be pinned to one graph feature.
//   mode 0: graph of kernels only
//   mode 1: kernels + an H2D memcpy node from pinned (hipHostMalloc) memory
//   mode 2: kernels + a D2H memcpy node into pinned memory
//   mode 3: H2D + kernels + D2H (the executor's shape)
//   mode 4: no graph; T host threads launching kernels eagerly on own streams
//   mode 5: mode 3 with hipMemcpyWithStream-free capture of pageable memory
//   mode 7: mode 3 run on a std::thread instead of the main thread
//   mode 6: mode 3 on S streams (one graph each, more streams than HW queues), replayed in turn
// usage: graph_probe <mode> [threads (mode 4) | kernels per graph (modes 0-3, default 8)]
// build: hipcc --offload-arch=gfx950 -O2 tools/graph_probe.hip -o tools/graph_probe -lpthread
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <thread>
#include <vector>

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(2);                                                                \
    }                                                                         \
  } while (0)

struct Args {
  const int* in;
  int* out;
  int n;
  int pad[29];  // a by-value parameter block of the size the executor's kernels take
};

__global__ void add_one(Args a) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < a.n) a.out[i] = a.in[i] + 1;
}

static int run_graph(int mode, int nk) {
  const char* ne = getenv("PROBE_ELEMS");  // copy / kernel size in ints (default 64 Ki)
  const int n = ne ? atoi(ne) : (1 << 16);
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  int *d0, *d1, *h;
  CK(hipMalloc(&d0, n * 4));
  CK(hipMalloc(&d1, n * 4));
  if (mode == 5) {
    h = (int*)malloc(n * 4);
  } else {
    CK(hipHostMalloc(&h, n * 4, hipHostMallocPortable));
  }
  for (int i = 0; i < n; ++i) h[i] = i;
  CK(hipMemcpy(d0, h, n * 4, hipMemcpyHostToDevice));
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  if (mode == 1 || mode == 3 || mode == 5) CK(hipMemcpyAsync(d0, h, n * 4, hipMemcpyHostToDevice, s));
  for (int k = 0; k < nk; ++k) {
    Args a{};
    a.in = (k & 1) ? d1 : d0;
    a.out = (k & 1) ? d0 : d1;
    a.n = n;
    hipLaunchKernelGGL(add_one, dim3((n + 255) / 256), dim3(256), 0, s, a);
    CK(hipGetLastError());
  }
  if (mode == 2 || mode == 3 || mode == 5) CK(hipMemcpyAsync(h, d0, n * 4, hipMemcpyDeviceToHost, s));
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamEndCapture(s, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  for (int it = 0; it < 20; ++it) CK(hipGraphLaunch(ge, s));
  CK(hipStreamSynchronize(s));
  printf("mode %d: graph of %d kernels replayed, h[1] = %d\n", mode, nk, h[1]);
  CK(hipGraphExecDestroy(ge));
  CK(hipGraphDestroy(g));
  CK(hipFree(d0));
  CK(hipFree(d1));
  if (mode == 5) free(h); else CK(hipHostFree(h));
  CK(hipStreamDestroy(s));
  return 0;
}

static int run_streams(int ns) {
  const int n = 1 << 16;
  std::vector<hipStream_t> ss(ns);
  std::vector<hipGraphExec_t> ge(ns);
  std::vector<int*> d0(ns), d1(ns), h(ns);
  for (int i = 0; i < ns; ++i) {
    CK(hipStreamCreateWithFlags(&ss[i], hipStreamNonBlocking));
    CK(hipMalloc(&d0[i], n * 4));
    CK(hipMalloc(&d1[i], n * 4));
    CK(hipHostMalloc(&h[i], n * 4, hipHostMallocPortable));
    for (int j = 0; j < n; ++j) h[i][j] = j;
  }
  for (int i = 0; i < ns; ++i) {
    // one eager pass first, as the executor does before capturing
    for (int cap = 0; cap < 2; ++cap) {
      if (cap) CK(hipStreamBeginCapture(ss[i], hipStreamCaptureModeThreadLocal));
      CK(hipMemcpyAsync(d0[i], h[i], n * 4, hipMemcpyHostToDevice, ss[i]));
      for (int k = 0; k < 60; ++k) {
        Args a{};
        a.in = (k & 1) ? d1[i] : d0[i];
        a.out = (k & 1) ? d0[i] : d1[i];
        a.n = n;
        hipLaunchKernelGGL(add_one, dim3(n / 256), dim3(256), 0, ss[i], a);
        CK(hipGetLastError());
      }
      CK(hipMemcpyAsync(h[i], d0[i], n * 4, hipMemcpyDeviceToHost, ss[i]));
      if (cap) {
        hipGraph_t g;
        CK(hipStreamEndCapture(ss[i], &g));
        CK(hipGraphInstantiate(&ge[i], g, nullptr, nullptr, 0));
        CK(hipGraphDestroy(g));
      } else {
        CK(hipStreamSynchronize(ss[i]));
      }
    }
  }
  for (int it = 0; it < 8; ++it)
    for (int i = 0; i < ns; ++i) {
      CK(hipGraphLaunch(ge[i], ss[i]));
      CK(hipStreamSynchronize(ss[i]));
    }
  printf("mode 6: %d streams x 8 graph replays done, h[0][1] = %d\n", ns, h[0][1]);
  return 0;
}

static int run_threads(int threads) {
  const int n = 1 << 16;
  std::vector<std::thread> ts;
  for (int t = 0; t < threads; ++t) {
    ts.emplace_back([=] {
      hipStream_t s;
      CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
      int *d0, *d1;
      CK(hipMalloc(&d0, n * 4));
      CK(hipMalloc(&d1, n * 4));
      for (int it = 0; it < 200; ++it) {
        Args a{};
        a.in = d0;
        a.out = d1;
        a.n = n;
        hipLaunchKernelGGL(add_one, dim3(n / 256), dim3(256), 0, s, a);
        CK(hipGetLastError());
      }
      CK(hipStreamSynchronize(s));
      CK(hipFree(d0));
      CK(hipFree(d1));
      CK(hipStreamDestroy(s));
    });
  }
  for (auto& t : ts) t.join();
  printf("mode 4: %d threads x 200 eager launches done\n", threads);
  return 0;
}

int main(int argc, char** argv) {
  int mode = argc > 1 ? atoi(argv[1]) : 0;
  int threads = argc > 2 ? atoi(argv[2]) : 8;
  if (mode == 4) return run_threads(threads);
  if (mode == 6) return run_streams(threads);
  if (mode == 7) {
    int rc = 0;
    std::thread t([&] { rc = run_graph(3, 60); });
    t.join();
    return rc;
  }
  return run_graph(mode, argc > 2 ? atoi(argv[2]) : 8);
}
