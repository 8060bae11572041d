// mxstream — native tracing: stage ranges for rocprofv3 (roctx) plus an
// in-process span recorder exported as Chrome trace JSON (chrome://tracing / Perfetto).
//
//   * range_push / range_pop: per-thread nested host ranges. When roctx is enabled
//     (MXS_ROCTX=1 or trace_enable_roctx(true)) each range is also a roctxRangePushA/Pop, so
//     `rocprofv3 --marker-trace` shows the engine's stages (partition, all_to_all, window_agg,
//     fire, spill, checkpoint) around the kernels they launch.
//   * complete(name, cat, track, ts_ns, dur_ns): a finished span recorded by the caller, used for
//     GPU stage spans resolved from HIP events (utils/trace.py) and for host spans.
//   * dump_chrome(path, pid): writes {"traceEvents": [...]} ("X" complete events, microseconds).
// The recorder is bounded (oldest spans dropped past the capacity) and thread-safe.
#include <pybind11/pybind11.h>

#include <rocprofiler-sdk-roctx/roctx.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <deque>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "mxs_runtime.h"

namespace py = pybind11;

namespace mxs {
namespace trace {
namespace {

struct Span {
  std::string name, cat, track;
  int64_t ts_ns, dur_ns;
};

struct Open {
  std::string name, cat;
  int64_t t0;
};

std::mutex g_mu;
std::deque<Span> g_spans;
size_t g_cap = 1 << 20;
std::atomic<bool> g_enabled{false};
std::atomic<bool> g_roctx{false};
std::atomic<int64_t> g_dropped{0};
thread_local std::vector<Open> t_stack;

bool env_flag(const char* name) {
  const char* v = std::getenv(name);
  return v && *v && std::string(v) != "0";
}

struct Init {
  Init() {
    g_roctx = env_flag("MXS_ROCTX");
    g_enabled = env_flag("MXS_TRACE");
  }
} g_init;

std::string thread_track() {
  return "host-" + std::to_string(std::hash<std::thread::id>()(std::this_thread::get_id()) % 100000);
}

void push_span(Span&& s) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (g_spans.size() >= g_cap) {
    g_spans.pop_front();
    ++g_dropped;
  }
  g_spans.push_back(std::move(s));
}

void json_escape(std::string& out, const std::string& s) {
  for (char c : s) {
    if (c == '"' || c == '\\') {
      out += '\\';
      out += c;
    } else if ((unsigned char)c < 0x20) {
      char buf[8];
      std::snprintf(buf, sizeof(buf), "\\u%04x", c);
      out += buf;
    } else {
      out += c;
    }
  }
}

}  // namespace

int64_t now_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

void range_push(const std::string& name, const std::string& cat) {
  if (g_roctx) roctxRangePushA(name.c_str());
  if (g_enabled) t_stack.push_back({name, cat, now_ns()});
}

void range_pop() {
  if (g_roctx) roctxRangePop();
  if (!g_enabled || t_stack.empty()) return;
  Open o = std::move(t_stack.back());
  t_stack.pop_back();
  const int64_t t1 = now_ns();
  push_span({std::move(o.name), std::move(o.cat), thread_track(), o.t0, t1 - o.t0});
}

void mark(const std::string& name) {
  if (g_roctx) roctxMarkA(name.c_str());
  if (g_enabled) push_span({name, "mark", thread_track(), now_ns(), 0});
}

void complete(const std::string& name, const std::string& cat, const std::string& track,
              int64_t ts_ns, int64_t dur_ns) {
  if (!g_enabled) return;
  push_span({name, cat, track, ts_ns, dur_ns < 0 ? 0 : dur_ns});
}

size_t dump_chrome(const std::string& path, int pid) {
  std::vector<Span> spans;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    spans.assign(g_spans.begin(), g_spans.end());
  }
  std::vector<std::string> tracks;
  auto track_id = [&](const std::string& t) {
    for (size_t i = 0; i < tracks.size(); ++i)
      if (tracks[i] == t) return (int)i;
    tracks.push_back(t);
    return (int)tracks.size() - 1;
  };
  std::string out = "{\"traceEvents\":[\n";
  bool first = true;
  char buf[160];
  for (const Span& s : spans) {
    const int tid = track_id(s.track);
    if (!first) out += ",\n";
    first = false;
    out += "{\"name\":\"";
    json_escape(out, s.name);
    out += "\",\"cat\":\"";
    json_escape(out, s.cat);
    std::snprintf(buf, sizeof(buf), "\",\"ph\":\"%s\",\"pid\":%d,\"tid\":%d,\"ts\":%.3f",
                  s.dur_ns > 0 ? "X" : "i", pid, tid, (double)s.ts_ns / 1e3);
    out += buf;
    if (s.dur_ns > 0) {
      std::snprintf(buf, sizeof(buf), ",\"dur\":%.3f", (double)s.dur_ns / 1e3);
      out += buf;
    } else {
      out += ",\"s\":\"t\"";
    }
    out += "}";
  }
  for (size_t i = 0; i < tracks.size(); ++i) {
    out += first ? "" : ",\n";
    first = false;
    out += "{\"name\":\"thread_name\",\"ph\":\"M\",\"pid\":" + std::to_string(pid) +
           ",\"tid\":" + std::to_string(i) + ",\"args\":{\"name\":\"";
    json_escape(out, tracks[i]);
    out += "\"}}";
  }
  out += "\n],\"displayTimeUnit\":\"ms\",\"otherData\":{\"dropped\":" +
         std::to_string(g_dropped.load()) + "}}\n";
  FILE* f = std::fopen(path.c_str(), "wb");
  if (!f) throw std::runtime_error("trace: cannot open " + path);
  const size_t w = std::fwrite(out.data(), 1, out.size(), f);
  std::fclose(f);
  if (w != out.size()) throw std::runtime_error("trace: short write to " + path);
  return spans.size();
}

}  // namespace trace
}  // namespace mxs

void bind_trace(py::module_& m) {
  using namespace mxs::trace;
  m.def("trace_now_ns", &now_ns);
  m.def("trace_enable", [](bool on) { g_enabled = on; });
  m.def("trace_enabled", []() { return g_enabled.load(); });
  m.def("trace_enable_roctx", [](bool on) { g_roctx = on; });
  m.def("trace_roctx_enabled", []() { return g_roctx.load(); });
  m.def("trace_set_capacity", [](size_t cap) {
    std::lock_guard<std::mutex> lk(g_mu);
    g_cap = cap ? cap : 1;
  });
  m.def("trace_clear", []() {
    std::lock_guard<std::mutex> lk(g_mu);
    g_spans.clear();
    g_dropped = 0;
  });
  m.def("trace_count", []() {
    std::lock_guard<std::mutex> lk(g_mu);
    return g_spans.size();
  });
  m.def("trace_push", &range_push, py::arg("name"), py::arg("cat") = "stage");
  m.def("trace_pop", &range_pop);
  m.def("trace_mark", &mark);
  m.def("trace_complete", &complete);
  m.def("trace_dump_chrome", &dump_chrome, py::arg("path"), py::arg("pid") = 0);
}
