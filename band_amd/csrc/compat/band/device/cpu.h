// Stand-in for band/device/cpu.h: the CpuSet handed to every executor
// (band/interface/model_executor.h:41-50).  Affinity is only honoured by
// the reference on mobile builds (band/device/util.h:12-16); the HIP
// backend records it and otherwise ignores it.
#pragma once
#include <vector>

#include "band/common.h"

namespace band {
class CpuSet {
 public:
  CpuSet() = default;
  void Enable(int cpu) { if (cpu >= 0) { if ((int)bits_.size() <= cpu) bits_.resize(cpu + 1, false); bits_[cpu] = true; } }
  bool IsEnabled(int cpu) const { return cpu >= 0 && cpu < (int)bits_.size() && bits_[cpu]; }
  int NumEnabled() const { int n = 0; for (bool b : bits_) n += b; return n; }
  std::vector<int> GetMaskBitsVector() const {
    std::vector<int> v;
    for (int i = 0; i < (int)bits_.size(); ++i) if (bits_[i]) v.push_back(i);
    return v;
  }
  CPUMaskFlag GetCPUMaskFlag() const { return flag_; }
  void SetFlag(CPUMaskFlag f) { flag_ = f; }

 private:
  std::vector<bool> bits_;
  CPUMaskFlag flag_ = CPUMaskFlag::kAll;
};

inline CpuSet BandCPUMaskGetSet(CPUMaskFlag flag) {
  CpuSet s;
  s.SetFlag(flag);
  return s;
}
}  // namespace band
