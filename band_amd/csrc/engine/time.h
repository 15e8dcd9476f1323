// Wall-clock helpers (band/time.h): microseconds on a monotonic clock.
#pragma once
#include <chrono>
#include <cstdint>
#include <thread>

namespace band {
namespace time {
inline int64_t NowMicros() {
  return std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}
inline void SleepForMicros(int64_t us) { std::this_thread::sleep_for(std::chrono::microseconds(us)); }
}  // namespace time
}  // namespace band
