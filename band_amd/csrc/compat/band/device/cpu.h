// Stand-in for band/device/cpu.h, signature-identical to
// /root/reference/band/device/cpu.h:21-57 (CpuSet, GetCPUCount,
// SetCPUThreadAffinity, BandCPUMaskGetSet).  The set holds a real cpu_set_t,
// as the reference's BAND_IS_MOBILE build does (band/device/cpu.cc:39-70);
// on this x86 harness every CPUMaskFlag maps to "all CPUs the process may
// use" (no big.LITTLE clusters), which the HIP backend reads as "no pinning",
// exactly as it reads the reference's Linux build, where IsEnabled() is
// always true (band/device/cpu.cc:72-92).
#pragma once

#include <limits.h>
#include <sched.h>
#include <stddef.h>

#include <string>
#include <vector>

#include "absl/status/status.h"
#include "band/common.h"

namespace band {

class CpuSet {
 public:
  CpuSet();
  void Enable(int cpu);
  void Disable(int cpu);
  void DisableAll();
  bool IsEnabled(int cpu) const;
  size_t NumEnabled() const;
  CPUMaskFlag GetCPUMaskFlag() const;
  // the raw cpu_set_t words (band/device/cpu.cc:52-56)
  const unsigned long* GetMaskBits() const;
  std::vector<unsigned long> GetMaskBitsVector() const;
  std::string ToString() const;
  bool operator==(const CpuSet& rhs) const;

  const cpu_set_t& GetCpuSet() const { return cpu_set_; }
  cpu_set_t& GetCpuSet() { return cpu_set_; }

 private:
  cpu_set_t cpu_set_;
};

// cpu info
size_t GetCPUCount();
size_t GetLittleCPUCount();
size_t GetBigCPUCount();

// set explicit thread affinity (calling thread)
absl::Status SetCPUThreadAffinity(const CpuSet& thread_affinity_mask);
absl::Status GetCPUThreadAffinity(CpuSet& thread_affinity_mask);

// convenient wrapper
const CpuSet& BandCPUMaskGetSet(CPUMaskFlag flag);
}  // namespace band
