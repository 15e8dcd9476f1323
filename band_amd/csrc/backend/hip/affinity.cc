#include "backend/hip/affinity.h"

#include <dirent.h>
#include <sched.h>
#include <unistd.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <mutex>
#include <sstream>

#include "band/device/cpu.h"
#include "band_hip_kernels.h"

namespace band {
namespace hip {

std::vector<int> ParseCpuList(const std::string& s) {
  std::vector<int> out;
  std::stringstream ss(s);
  std::string piece;
  while (std::getline(ss, piece, ',')) {
    const size_t dash = piece.find('-');
    char* end = nullptr;
    if (dash == std::string::npos) {
      const long v = std::strtol(piece.c_str(), &end, 10);
      if (end != piece.c_str() && v >= 0 && v < CPU_SETSIZE) out.push_back(static_cast<int>(v));
      continue;
    }
    const long a = std::strtol(piece.substr(0, dash).c_str(), &end, 10);
    const long b = std::strtol(piece.substr(dash + 1).c_str(), nullptr, 10);
    if (a < 0 || b < a || b >= CPU_SETSIZE) continue;
    for (long v = a; v <= b; ++v) out.push_back(static_cast<int>(v));
  }
  std::sort(out.begin(), out.end());
  out.erase(std::unique(out.begin(), out.end()), out.end());
  return out;
}

namespace {
std::vector<int> MaskCpus(const cpu_set_t& m) {
  std::vector<int> out;
  for (int c = 0; c < CPU_SETSIZE; ++c)
    if (CPU_ISSET(c, &m)) out.push_back(c);
  return out;
}
}  // namespace

const std::vector<int>& ProcessCpus() {
  static const std::vector<int> cpus = [] {
    cpu_set_t m;
    CPU_ZERO(&m);
    if (sched_getaffinity(getpid(), sizeof(m), &m) != 0) return std::vector<int>();
    return MaskCpus(m);
  }();
  return cpus;
}

std::vector<int> PinnableCpus(const CpuSet& set) {
  std::vector<int> cpus;
  const int n = static_cast<int>(std::min<size_t>(GetCPUCount(), CPU_SETSIZE));
  for (int i = 0; i < n; ++i)
    if (set.IsEnabled(i)) cpus.push_back(i);
  const std::vector<int>& allowed = ProcessCpus();
  if (cpus.empty() || std::includes(cpus.begin(), cpus.end(), allowed.begin(), allowed.end())) return {};
  return cpus;
}

bool PinThread(pthread_t t, const std::vector<int>& cpus) {
  if (cpus.empty()) return false;
  cpu_set_t m;
  CPU_ZERO(&m);
  for (int c : cpus)
    if (c >= 0 && c < CPU_SETSIZE) CPU_SET(c, &m);
  return pthread_setaffinity_np(t, sizeof(m), &m) == 0;
}

std::vector<int> CallingThreadCpus() {
  cpu_set_t m;
  CPU_ZERO(&m);
  if (pthread_getaffinity_np(pthread_self(), sizeof(m), &m) != 0) return {};
  return MaskCpus(m);
}

int GpuNumaNode(int ordinal) {
  char bus[64] = {0};
  if (bh_device_pci_bus_id(ordinal, bus, sizeof(bus)) != 0) return -1;
  // sysfs names are lower-case "dddd:bb:dd.f"
  std::string id(bus);
  for (char& ch : id) ch = static_cast<char>(std::tolower(static_cast<unsigned char>(ch)));
  std::ifstream f("/sys/bus/pci/devices/" + id + "/numa_node");
  int node = -1;
  if (!(f >> node)) return -1;
  return node;
}

std::vector<int> GpuNumaCpus(int ordinal) {
  const int node = GpuNumaNode(ordinal);
  if (node < 0) return {};
  std::ifstream f("/sys/devices/system/node/node" + std::to_string(node) + "/cpulist");
  std::string list;
  if (!std::getline(f, list)) return {};
  std::vector<int> node_cpus = ParseCpuList(list), out;
  const std::vector<int>& allowed = ProcessCpus();
  std::set_intersection(node_cpus.begin(), node_cpus.end(), allowed.begin(), allowed.end(),
                        std::back_inserter(out));
  return out;
}

bool PinCallingThreadToGpu(int ordinal) {
  thread_local int pinned = -2;  // ordinal this thread was placed for
  thread_local bool ok = false;
  if (pinned == ordinal) return ok;
  pinned = ordinal;
  ok = false;
  const char* env = std::getenv("BANDX_NUMA_PIN");
  if (env && env[0] == '0') return ok;
  // resolved once per ordinal for the process
  static std::mutex mu;
  static std::vector<std::vector<int>> cache;
  static std::vector<bool> known;
  std::vector<int> cpus;
  {
    std::lock_guard<std::mutex> lk(mu);
    if (ordinal >= static_cast<int>(known.size())) {
      known.resize(ordinal + 1, false);
      cache.resize(ordinal + 1);
    }
    if (!known[ordinal]) {
      cache[ordinal] = GpuNumaCpus(ordinal);
      known[ordinal] = true;
    }
    cpus = cache[ordinal];
  }
  // no NUMA information, or the node is all the process has: nothing to do
  if (cpus.empty() || cpus.size() == ProcessCpus().size()) return ok;
  ok = PinThread(pthread_self(), cpus);
  return ok;
}

int PinProcessToCpus(const std::vector<int>& cpus) {
  cpu_set_t m;
  CPU_ZERO(&m);
  int n = 0;
  for (int c : cpus)
    if (c >= 0 && c < CPU_SETSIZE) {
      CPU_SET(c, &m);
      ++n;
    }
  if (n == 0) return -1;
  DIR* d = opendir("/proc/self/task");
  if (!d) return -1;
  int pinned = 0;
  bool failed = false;
  while (dirent* ent = readdir(d)) {
    char* end = nullptr;
    const long tid = std::strtol(ent->d_name, &end, 10);
    if (end == ent->d_name || *end != '\0' || tid <= 0) continue;
    if (sched_setaffinity(static_cast<pid_t>(tid), sizeof(m), &m) == 0)
      ++pinned;
    else
      failed = true;  // a thread that exited meanwhile also lands here
  }
  closedir(d);
  return failed && pinned == 0 ? -1 : pinned;
}

int PinProcessToGpu(int ordinal) {
  const char* env = std::getenv("BANDX_NUMA_PIN");
  if (env && env[0] == '0') return 0;
  const std::vector<int> cpus = GpuNumaCpus(ordinal);
  if (cpus.empty() || cpus.size() == ProcessCpus().size()) return 0;
  return PinProcessToCpus(cpus);
}

}  // namespace hip
}  // namespace band
