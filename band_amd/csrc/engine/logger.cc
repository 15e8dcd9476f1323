#include "engine/logger.h"

#include <cstdarg>
#include <cstdio>
#include <map>
#include <mutex>

namespace band {

namespace {
std::mutex g_mu;
LogSeverity g_threshold = LogSeverity::kWarning;
std::map<int, std::function<void(LogSeverity, const char*)>> g_reporters;
int g_next = 0;
const char* Name(LogSeverity s) {
  switch (s) {
    case LogSeverity::kInternal: return "INTERNAL";
    case LogSeverity::kInfo: return "INFO";
    case LogSeverity::kWarning: return "WARNING";
    default: return "ERROR";
  }
}
}  // namespace

Logger& Logger::Get() {
  static Logger l;
  return l;
}

void Logger::SetVerbosity(LogSeverity s) {
  std::lock_guard<std::mutex> lock(g_mu);
  g_threshold = s;
}

int Logger::SetReporter(std::function<void(LogSeverity, const char*)> r) {
  std::lock_guard<std::mutex> lock(g_mu);
  g_reporters[g_next] = std::move(r);
  return g_next++;
}

bool Logger::RemoveReporter(int handle) {
  std::lock_guard<std::mutex> lock(g_mu);
  return g_reporters.erase(handle) != 0;
}

void Logger::Log(LogSeverity s, const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  std::vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  std::lock_guard<std::mutex> lock(g_mu);
  if (static_cast<int>(s) < static_cast<int>(g_threshold)) return;
  if (g_reporters.empty()) {
    std::fprintf(stderr, "[band %s] %s\n", Name(s), buf);
  } else {
    for (auto& r : g_reporters) r.second(s, buf);
  }
}

}  // namespace band
