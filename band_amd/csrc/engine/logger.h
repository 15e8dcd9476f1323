// Logging with a severity threshold and pluggable reporters (band/logger.h);
// the C API's BandSetLogSeverity / BandSetLogReporter drive it.
#pragma once
#include <functional>

namespace band {

enum class LogSeverity : int { kInternal = 0, kInfo, kWarning, kError };

class Logger {
 public:
  static Logger& Get();
  void SetVerbosity(LogSeverity severity);
  int SetReporter(std::function<void(LogSeverity, const char*)> reporter);
  bool RemoveReporter(int handle);
  void Log(LogSeverity severity, const char* fmt, ...) __attribute__((format(printf, 3, 4)));
};

}  // namespace band

#define BAND_LOG(sev, ...) ::band::Logger::Get().Log(sev, __VA_ARGS__)
