// mxstream — leveled logger of the native runtime (threads without the GIL): level from
// MXS_LOG_LEVEL (DEBUG/INFO/WARN/ERROR, default WARN), log4j-like layout on stderr.
#pragma once
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <ctime>
#include <mutex>
#include <string>

namespace mxs {

enum LogLevel { kDebug = 0, kInfo = 1, kWarn = 2, kError = 3 };

inline int log_threshold() {
  static const int lvl = [] {
    const char* e = std::getenv("MXS_LOG_LEVEL");
    if (!e) return (int)kWarn;
    const std::string v(e);
    if (v == "DEBUG" || v == "debug" || v == "TRACE") return (int)kDebug;
    if (v == "INFO" || v == "info") return (int)kInfo;
    if (v == "ERROR" || v == "error") return (int)kError;
    return (int)kWarn;
  }();
  return lvl;
}

inline void mxs_log(LogLevel level, const std::string& logger, const std::string& msg) {
  if ((int)level < log_threshold()) return;
  static std::mutex mu;
  static const char* names[] = {"DEBUG", "INFO", "WARN", "ERROR"};
  const auto now = std::chrono::system_clock::now();
  const std::time_t tt = std::chrono::system_clock::to_time_t(now);
  const int ms = (int)(std::chrono::duration_cast<std::chrono::milliseconds>(
                           now.time_since_epoch()).count() % 1000);
  std::tm tm{};
  localtime_r(&tt, &tm);
  char ts[32];
  std::strftime(ts, sizeof(ts), "%Y-%m-%d %H:%M:%S", &tm);
  std::lock_guard<std::mutex> g(mu);
  std::fprintf(stderr, "%s,%03d %-5s mxstream.native.%-25s - %s\n", ts, ms, names[level],
               logger.c_str(), msg.c_str());
}

}  // namespace mxs
