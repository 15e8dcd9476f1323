#include "backend/hip/util.h"

#include "backend/hip/device.h"

namespace band {
namespace hip {
std::set<DeviceFlag> HipUtil::GetAvailableDevices() const {
  std::set<DeviceFlag> d = {DeviceFlag::kCPU};
  if (DeviceRegistry::Get().GpuAvailable()) d.insert(DeviceFlag::kGPU);
  return d;
}
}  // namespace hip
}  // namespace band
