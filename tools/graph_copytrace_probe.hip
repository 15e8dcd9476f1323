// Reproducer for the rocprofv3 7.2 SIGSEGV under --memory-copy-trace
// (verdict item 7), with no code of this repository:
// ONE captured graph holding an H2D copy node, a kernel node and a D2H copy
// node, launched 20000 times, faults inside the tool's hipGraphLaunch
// interception (a memcpy reading past the end of a mapping, the same stack
// as the bench's records profiles/r04q_tr2_copytrace_crash.txt and
// r04r_copytrace_step25_crash.txt).  1 graph x 1 launch, kernel-only graphs
// and copy-only graphs (1000 graphs x 20 launches) trace cleanly, and the
// kernel's argument size makes no difference (small / padded):
// profiles/r04v_graph_copytrace_probe.txt.
//   usage: graph_copytrace_probe small|padded [graphs=1000] [launches=20] [k|mk|m]
//   nodes: k = the kernel node alone, mk = H2D copy + kernel + D2H copy,
//   m = the two copies alone
//   build: hipcc --offload-arch=gfx950 -O2 tools/graph_copytrace_probe.hip -o tools/graph_copytrace_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

struct Small {
  const int* table;
  int n;
};
struct Padded {
  const int* table;
  int n;
  int pad[61];  // 256 bytes in all
};

__global__ void small_kernel(const int* table, int n, int* out) {
  if (threadIdx.x == 0 && blockIdx.x < (unsigned)n) out[blockIdx.x] = table[blockIdx.x] + 1;
}
__global__ void padded_kernel(Padded a, int* out) {
  if (threadIdx.x == 0 && blockIdx.x < (unsigned)a.n) out[blockIdx.x] = a.table[blockIdx.x] + 1;
}

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));             \
      return 1;                                                                \
    }                                                                          \
  } while (0)

int main(int argc, char** argv) {
  const bool padded = argc > 1 && std::strcmp(argv[1], "padded") == 0;
  const int graphs = argc > 2 ? std::atoi(argv[2]) : 1000;
  const int launches = argc > 3 ? std::atoi(argv[3]) : 20;
  const char* nodes = argc > 4 ? argv[4] : "mk";
  const bool copies = std::strchr(nodes, 'm') != nullptr, kernel = std::strchr(nodes, 'k') != nullptr;
  int *table = nullptr, *out = nullptr, *host = nullptr;
  CK(hipMalloc(&table, 64 * sizeof(int)));
  CK(hipMalloc(&out, 64 * sizeof(int)));
  CK(hipMemset(table, 0, 64 * sizeof(int)));
  CK(hipHostMalloc(&host, 64 * sizeof(int)));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  std::vector<hipGraphExec_t> execs(graphs);
  for (int g = 0; g < graphs; ++g) {
    hipGraph_t graph;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    if (copies) CK(hipMemcpyAsync(table, host, 64 * sizeof(int), hipMemcpyHostToDevice, s));
    if (!kernel) {
    } else if (padded) {
      Padded a{};
      a.table = table;
      a.n = 16;
      hipLaunchKernelGGL(padded_kernel, dim3(16), dim3(64), 0, s, a, out);
    } else {
      hipLaunchKernelGGL(small_kernel, dim3(16), dim3(64), 0, s, (const int*)table, 16, out);
    }
    CK(hipGetLastError());
    if (copies) CK(hipMemcpyAsync(host, out, 64 * sizeof(int), hipMemcpyDeviceToHost, s));
    CK(hipStreamEndCapture(s, &graph));
    CK(hipGraphInstantiate(&execs[g], graph, nullptr, nullptr, 0));
    CK(hipGraphDestroy(graph));
  }
  for (int l = 0; l < launches; ++l)
    for (int g = 0; g < graphs; ++g) CK(hipGraphLaunch(execs[g], s));
  CK(hipStreamSynchronize(s));
  for (auto& e : execs) CK(hipGraphExecDestroy(e));
  std::printf("graph_copytrace_probe %s %s: %d graphs x %d launches OK\n", padded ? "padded" : "small", nodes, graphs,
              launches);
  return 0;
}
