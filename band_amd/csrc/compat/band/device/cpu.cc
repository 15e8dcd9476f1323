// Stand-in for band/device/cpu.cc (see cpu.h): the cpu_set_t-backed CpuSet
// of the reference's mobile build, with every CPUMaskFlag resolving to the
// CPUs the process may use (an x86 host has no LITTLE/big clusters).
#include "band/device/cpu.h"

#include <pthread.h>
#include <unistd.h>

#include <cstring>
#include <mutex>

namespace band {

CpuSet::CpuSet() { DisableAll(); }
void CpuSet::Enable(int cpu) {
  if (cpu >= 0 && cpu < CPU_SETSIZE) CPU_SET(cpu, &cpu_set_);
}
void CpuSet::Disable(int cpu) {
  if (cpu >= 0 && cpu < CPU_SETSIZE) CPU_CLR(cpu, &cpu_set_);
}
void CpuSet::DisableAll() { CPU_ZERO(&cpu_set_); }
bool CpuSet::IsEnabled(int cpu) const { return cpu >= 0 && cpu < CPU_SETSIZE && CPU_ISSET(cpu, &cpu_set_); }
size_t CpuSet::NumEnabled() const { return static_cast<size_t>(CPU_COUNT(&cpu_set_)); }
const unsigned long* CpuSet::GetMaskBits() const { return cpu_set_.__bits; }
std::vector<unsigned long> CpuSet::GetMaskBitsVector() const {
  return std::vector<unsigned long>(GetMaskBits(), GetMaskBits() + sizeof(cpu_set_.__bits) / sizeof(*cpu_set_.__bits));
}
bool CpuSet::operator==(const CpuSet& rhs) const { return CPU_EQUAL(&cpu_set_, &rhs.cpu_set_) != 0; }
std::string CpuSet::ToString() const {
  std::string s;
  for (size_t i = 0; i < GetCPUCount(); ++i) s += IsEnabled(static_cast<int>(i)) ? "1" : "0";
  return s;
}
CPUMaskFlag CpuSet::GetCPUMaskFlag() const {
  for (size_t i = 0; i < EnumLength<CPUMaskFlag>(); ++i) {
    const CPUMaskFlag f = static_cast<CPUMaskFlag>(i);
    if (BandCPUMaskGetSet(f) == *this) return f;
  }
  return CPUMaskFlag::kAll;
}

size_t GetCPUCount() {
  const long n = sysconf(_SC_NPROCESSORS_CONF);
  return n > 0 ? static_cast<size_t>(n) : 1;
}
size_t GetLittleCPUCount() { return 0; }
size_t GetBigCPUCount() { return GetCPUCount(); }

absl::Status SetCPUThreadAffinity(const CpuSet& mask) {
  if (pthread_setaffinity_np(pthread_self(), sizeof(cpu_set_t), &mask.GetCpuSet()) != 0)
    return absl::InternalError("Failed to set the thread's CPU affinity");
  return absl::OkStatus();
}
absl::Status GetCPUThreadAffinity(CpuSet& mask) {
  if (pthread_getaffinity_np(pthread_self(), sizeof(cpu_set_t), &mask.GetCpuSet()) != 0)
    return absl::InternalError("Failed to get the thread's CPU affinity");
  return absl::OkStatus();
}

const CpuSet& BandCPUMaskGetSet(CPUMaskFlag /*flag*/) {
  // the process's own affinity at first use: every flag is "all CPUs"
  static const CpuSet all = [] {
    CpuSet s;
    if (sched_getaffinity(0, sizeof(cpu_set_t), &s.GetCpuSet()) != 0)
      for (size_t i = 0; i < GetCPUCount(); ++i) s.Enable(static_cast<int>(i));
    return s;
  }();
  return all;
}

}  // namespace band
