// mxstream — pybind11 binding of the native window step (csrc/window_step.h): the Python
// KeyedWindowOperator (runtime/window_operator.py) is a thin shell over this class. Every step
// entry point runs with the GIL released; the collectives of a multi-rank step call back into the
// rank's Python process group (RCCL / gloo / loopback) with the GIL re-acquired. State buffers are
// handed to Python as DLPack tensors that share ownership of the memory.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cmath>
#include <cstring>
#include <string>

#include "window_step.h"

namespace py = pybind11;
using namespace mxs;

namespace mxs {
ExprProg expr_program(const std::vector<int32_t>& code, const std::vector<double>& consts);
namespace trace {
void range_push(const std::string& name, const std::string& cat);
void range_pop();
}  // namespace trace
}  // namespace mxs

namespace {

// ---- DLPack (the stable v0 ABI, as torch.from_dlpack consumes it) ---------------------------
struct DLDevice {
  int32_t device_type;  // 1 = CPU, 10 = ROCm
  int32_t device_id;
};
struct DLDataType {
  uint8_t code;  // 0 int, 1 uint, 2 float
  uint8_t bits;
  uint16_t lanes;
};
struct DLTensor {
  void* data;
  DLDevice device;
  int32_t ndim;
  DLDataType dtype;
  int64_t* shape;
  int64_t* strides;
  uint64_t byte_offset;
};
struct DLManagedTensor {
  DLTensor dl_tensor;
  void* manager_ctx;
  void (*deleter)(DLManagedTensor*);
};

struct ViewCtx {
  Buf keep;  // may be null (non-owning view)
  int64_t shape[1];
};

void dl_delete(DLManagedTensor* t) {
  delete static_cast<ViewCtx*>(t->manager_ctx);
  delete t;
}

void capsule_destructor(PyObject* cap) {
  // A capsule torch never consumed still owns its tensor.
  if (PyCapsule_IsValid(cap, "dltensor")) {
    auto* t = static_cast<DLManagedTensor*>(PyCapsule_GetPointer(cap, "dltensor"));
    if (t && t->deleter) t->deleter(t);
  }
}

// dtype: 'i8' 'i4' 'u1' 'f8' 'f4' (torch int64 / int32 / uint8 / float64 / float32)
py::object dl_capsule(void* data, int64_t numel, const std::string& dtype, bool gpu, int dev,
                      Buf keep) {
  auto* ctx = new ViewCtx{std::move(keep), {numel}};
  auto* t = new DLManagedTensor();
  t->dl_tensor.data = data;
  t->dl_tensor.device = DLDevice{gpu ? 10 : 1, gpu ? dev : 0};
  t->dl_tensor.ndim = 1;
  DLDataType dt{0, 64, 1};
  if (dtype == "i8") dt = {0, 64, 1};
  else if (dtype == "i4") dt = {0, 32, 1};
  else if (dtype == "u1") dt = {1, 8, 1};
  else if (dtype == "f8") dt = {2, 64, 1};
  else if (dtype == "f4") dt = {2, 32, 1};
  else throw std::invalid_argument("dl_capsule: unknown dtype " + dtype);
  t->dl_tensor.dtype = dt;
  t->dl_tensor.shape = ctx->shape;
  t->dl_tensor.strides = nullptr;
  t->dl_tensor.byte_offset = 0;
  t->manager_ctx = ctx;
  t->deleter = dl_delete;
  return py::reinterpret_steal<py::object>(PyCapsule_New(t, "dltensor", capsule_destructor));
}

// Collectives of a multi-rank step, forwarded to the Python comm adapter
// (runtime/window_operator.py _StepCommAdapter: allreduce_min(ptr, n, stream) and
// all_to_all(recv, send, nbytes, elem, stream) over the rank's process group).
struct PyStepComm : StepComm {
  py::object adapter;
  ~PyStepComm() override {
    py::gil_scoped_acquire g;
    adapter = py::object();
  }
  void allreduce_min_i64(int64_t* buf, int n, intptr_t stream) override {
    py::gil_scoped_acquire g;
    adapter.attr("allreduce_min")((intptr_t)buf, n, stream);
  }
  void all_to_all(void* recv, const void* send, int64_t bytes, int elem, intptr_t stream) override {
    py::gil_scoped_acquire g;
    adapter.attr("all_to_all")((intptr_t)recv, (intptr_t)send, bytes, elem, stream);
  }
};

template <class T>
py::object np_view(const T* p, int64_t n, const Buf& slab, int64_t cols = 0) {
  auto* keep = new Buf(slab);
  py::capsule base(keep, [](void* v) { delete static_cast<Buf*>(v); });
  if (cols > 0)
    return py::array_t<T>({(py::ssize_t)n, (py::ssize_t)cols},
                          {(py::ssize_t)(cols * sizeof(T)), (py::ssize_t)sizeof(T)}, p, base);
  return py::array_t<T>({(py::ssize_t)n}, {(py::ssize_t)sizeof(T)}, p, base);
}

WindowStepConfig make_cfg(py::dict d) {
  WindowStepConfig c;
  auto get = [&](const char* k) { return d[k]; };
  c.size = get("size").cast<int64_t>();
  c.slide = get("slide").cast<int64_t>();
  c.offset = get("offset").cast<int64_t>();
  c.lateness = get("lateness").cast<int64_t>();
  c.agg = get("agg").cast<int32_t>();
  c.gpu = get("gpu").cast<bool>();
  c.device_index = get("device_index").cast<int>();
  c.parallelism = get("parallelism").cast<int>();
  c.max_parallelism = get("max_parallelism").cast<int>();
  c.hash_mode = get("hash_mode").cast<int>();
  c.jhash = reinterpret_cast<const int32_t*>(get("jhash").cast<intptr_t>());
  py::tuple m = get("map").cast<py::tuple>();
  py::tuple f = get("filt").cast<py::tuple>();
  c.map = expr_program(m[0].cast<std::vector<int32_t>>(), m[1].cast<std::vector<double>>());
  c.filt = expr_program(f[0].cast<std::vector<int32_t>>(), f[1].cast<std::vector<double>>());
  c.max_keys = get("max_keys").cast<int64_t>();
  c.batch_capacity = get("batch_capacity").cast<int64_t>();
  c.bucket_slack = get("bucket_slack").cast<double>();
  c.cap_log2 = get("cap_log2").cast<int>();
  c.event_time = get("event_time").cast<bool>();
  c.ooo_bound = get("ooo_bound").cast<int64_t>();
  c.side_output_late = get("side_output_late").cast<bool>();
  c.late_capacity = get("late_capacity").cast<int64_t>();
  c.external_watermark = get("external_watermark").cast<bool>();
  c.combine = get("combine").cast<int>();
  c.compact = get("compact").cast<int>();
  c.narrow = get("narrow").cast<int>();
  c.dense_keys = get("dense_keys").cast<bool>();
  c.pipeline = get("pipeline").cast<int>();
  c.exchange = get("exchange").cast<int>();
  c.idle_timeout_steps = get("idle_timeout_steps").cast<int>();
  c.deterministic = get("deterministic").cast<bool>();
  c.spill = get("spill").cast<bool>();
  c.spill_load = get("spill_load").cast<double>();
  c.spill_check_steps = get("spill_check_steps").cast<int>();
  c.spill_keep_panes = get("spill_keep_panes").cast<int>();
  c.emit_kv = get("emit_kv").cast<bool>();
  c.latency_fire = get("latency_fire").cast<int>();
  c.window_keys = get("window_keys").cast<int64_t>();
  c.dim = get("dim").cast<int>();
  c.vec_avg = get("vec_avg").cast<bool>();
  c.vec_has_threshold = !get("vec_threshold").is_none();
  c.vec_threshold = c.vec_has_threshold ? get("vec_threshold").cast<double>() : 0.0;
  c.vec_mode = get("vec_mode").cast<int>();
  return c;
}

struct ViewSpec {
  const char* dtype;
  int64_t numel;
};

ViewSpec view_spec(WindowStep& s, const std::string& n) {
  const int64_t ns = s.nslots(), R = s.ring(), D = s.cfg().dim;
  if (n == "keys_g") return {"i8", ns};
  if (n == "acc_g") return {"i8", D > 0 ? 1 : R * ns};
  if (n == "vacc_g") return {"f4", R * ns * D};
  if (n == "cnt_g") return {"i4", R * ns};
  if (n == "dirty_g") return {"u1", R * ns};
  if (n == "dacc_g") return {"i8", R * ns};
  if (n == "dcnt_g") return {"i4", R * ns};
  if (n == "occ") return {"i4", s.nsub()};
  if (n == "flags") return {"i4", 4};
  if (n == "kg_dest") return {"i4", s.cfg().max_parallelism};
  if (n == "dlist" || n == "slot_mark") return {"i4", ns};
  if (n == "dlist_n") return {"i4", 1};
  if (n == "keys_m") return {"i8", s.nslots_o()};
  if (n == "acc_m") return {"i8", s.ring_m() * s.nslots_o()};
  if (n == "cnt_m") return {"i4", s.ring_m() * s.nslots_o()};
  if (n == "dirty_m") return {"u1", s.ring_m() * s.nslots_o()};
  if (n == "occ_m") return {"i4", s.nsub_o()};
  if (n == "out_keys" || n == "out_raw") return {"i8", (int64_t)(s.buffer(n)->bytes / 8)};
  if (n == "out_vals") return {"f8", (int64_t)(s.buffer(n)->bytes / 8)};
  if (n == "out_cnt") return {"i4", (int64_t)(s.buffer(n)->bytes / 4)};
  if (n == "scratch") return {"i8", (int64_t)(s.buffer(n)->bytes / 8)};
  throw std::invalid_argument("WindowStep.view: unknown buffer " + n);
}

py::dict metrics_dict(const StepMetrics& m) {
  py::dict d;
  d["num_records_in"] = m.num_records_in;
  d["num_late_records_dropped"] = m.num_late_records_dropped;
  d["num_records_out"] = m.num_records_out;
  d["num_fires"] = m.num_fires;
  d["current_watermark"] = m.current_watermark;
  d["steps"] = m.steps;
  d["bucket_regrows"] = m.bucket_regrows;
  d["ring_regrows"] = m.ring_regrows;
  py::dict x;
  auto put = [&](const char* k, int64_t v) {
    if (v) x[k] = v;
  };
  put("compact_fallbacks", m.compact_fallbacks);
  put("latency_fires", m.latency_fires);
  put("combine_regrows", m.combine_regrows);
  put("a2a_bytes", m.a2a_bytes);
  put("payload_bytes", m.payload_bytes);
  put("merge_compactions", m.merge_compactions);
  put("async_evictions", m.async_evictions);
  put("dropped_keys", m.dropped_keys);
  put("spilled_keys", m.spilled_keys);
  put("spilled_rows", m.spilled_rows);
  d["extra"] = x;
  return d;
}

void set_metric(StepMetrics& m, const std::string& k, int64_t v) {
  if (k == "num_records_in") m.num_records_in = v;
  else if (k == "num_late_records_dropped") m.num_late_records_dropped = v;
  else if (k == "num_records_out") m.num_records_out = v;
  else if (k == "num_fires") m.num_fires = v;
  else if (k == "current_watermark") m.current_watermark = v;
  else if (k == "steps") m.steps = v;
  else if (k == "bucket_regrows") m.bucket_regrows = v;
  else if (k == "ring_regrows") m.ring_regrows = v;
  else throw std::invalid_argument("WindowStep: no metric " + k);
}

py::list rows_to_py(WindowStep& s, std::vector<FireRows>&& rows) {
  py::list out;
  const int D = s.cfg().dim;
  for (auto& r : rows) {
    py::object keys = r.kv ? np_view((const uint32_t*)r.keys, r.n, r.slab)
                           : np_view((const uint64_t*)r.keys, r.n, r.slab);
    py::object vals = r.vec ? np_view(r.vecs, r.n, r.slab, D) : np_view(r.vals, r.n, r.slab);
    py::object raw = r.raw ? np_view(r.raw, r.n, r.slab) : py::none();
    py::object cnt = r.cnt ? np_view(r.cnt, r.n, r.slab) : py::none();
    out.append(py::make_tuple(r.start, r.end, keys, vals, raw, cnt, r.refire, r.seq));
  }
  return out;
}

}  // namespace

void bind_window_step(py::module_& m) {
  // the step's phases as trace ranges (roctx with MXS_ROCTX=1, Chrome trace spans)
  g_stage_range_hook = [](const char* name, bool push) {
    if (push) trace::range_push(std::string("window.") + name, "stage");
    else trace::range_pop();
  };
  m.def("dl_view", [](intptr_t ptr, int64_t numel, const std::string& dtype, bool gpu, int dev) {
    return dl_capsule(reinterpret_cast<void*>(ptr), numel, dtype, gpu, dev, nullptr);
  }, "A non-owning DLPack capsule over memory the caller keeps alive (torch.from_dlpack).");
  py::class_<WindowStep>(m, "WindowStep")
      .def(py::init([](py::dict cfg, py::object adapter, int world, int rank) {
             std::shared_ptr<StepComm> c;
             if (world > 1) {
               auto pc = std::make_shared<PyStepComm>();
               pc->adapter = adapter;
               c = pc;
             } else {
               struct One : StepComm {
                 void allreduce_min_i64(int64_t*, int, intptr_t) override {}
                 void all_to_all(void* r, const void* s, int64_t b, int, intptr_t) override {
                   if (r != s) std::memmove(r, s, (size_t)b);
                 }
               };
               c = std::make_shared<One>();
             }
             c->world = world;
             c->rank = rank;
             WindowStepConfig wc = make_cfg(cfg);
             py::gil_scoped_release nogil;
             return new WindowStep(wc, c);
           }),
           py::arg("cfg"), py::arg("comm"), py::arg("world"), py::arg("rank"))
      .def("process", [](WindowStep& s, intptr_t keys, bool key32, intptr_t ts, intptr_t vals,
                         int64_t n, intptr_t stream, intptr_t vecs) {
             py::gil_scoped_release nogil;
             s.process(reinterpret_cast<const void*>(keys), key32, reinterpret_cast<const int64_t*>(ts),
                       reinterpret_cast<const void*>(vals), n, stream,
                       reinterpret_cast<const float*>(vecs));
           }, py::arg("keys"), py::arg("key32"), py::arg("ts"), py::arg("vals"), py::arg("n"),
           py::arg("stream"), py::arg("vecs") = 0)
      .def("flush", [](WindowStep& s, intptr_t st) {
        py::gil_scoped_release nogil;
        s.flush(st);
      })
      .def("advance_watermark", [](WindowStep& s, int64_t wm, intptr_t st) {
        py::gil_scoped_release nogil;
        s.advance_watermark(wm, st);
      })
      .def("finish", [](WindowStep& s, intptr_t st) {
        py::gil_scoped_release nogil;
        s.finish(st);
      })
      .def("take", [](WindowStep& s, bool block) {
        std::vector<FireRows> rows;
        {
          py::gil_scoped_release nogil;
          rows = s.take(block);
        }
        return rows_to_py(s, std::move(rows));
      }, py::arg("block") = true)
      .def("sync_state", [](WindowStep& s, intptr_t st) {
        py::gil_scoped_release nogil;
        s.sync_state(st);
      })
      .def("drain", [](WindowStep& s) {
        py::gil_scoped_release nogil;
        s.drain_all();
      })
      .def("compact_state", [](WindowStep& s, py::object cutoff, bool wait, intptr_t st) {
        const bool has = !cutoff.is_none();
        const int64_t c = has ? cutoff.cast<int64_t>() : 0;
        py::gil_scoped_release nogil;
        return s.compact_state(has, c, wait, st);
      })
      .def("rebuild_merge_ring", [](WindowStep& s, intptr_t st) {
        py::gil_scoped_release nogil;
        s.rebuild_merge_ring(st);
      })
      .def("reset_state", [](WindowStep& s, int64_t ring) {
        py::gil_scoped_release nogil;
        s.reset_state(ring);
      })
      .def("check_table", [](WindowStep& s, intptr_t st) { s.check_table(st); })
      .def("mark_idle", &WindowStep::mark_idle)
      .def_property_readonly("idle", &WindowStep::idle)
      .def("set_proc_time", &WindowStep::set_proc_time)
      .def("view", [](WindowStep& s, const std::string& name) -> py::object {
        Buf b = s.buffer(name);
        if (!b) return py::none();
        const ViewSpec v = view_spec(s, name);
        return dl_capsule(b->p, v.numel, v.dtype, s.cfg().gpu, s.cfg().device_index, b);
      })
      .def("metrics", [](WindowStep& s) { return metrics_dict(s.metrics()); })
      .def("set_metric", [](WindowStep& s, const std::string& k, int64_t v) { set_metric(s.metrics(), k, v); })
      .def("late_side", [](WindowStep& s) {
        py::list out;
        for (auto& v : s.late_side()) {
          py::array_t<uint32_t> a((py::ssize_t)v.size());
          if (!v.empty()) std::memcpy(a.mutable_data(), v.data(), v.size() * 4);
          out.append(a);
        }
        s.late_side().clear();
        return out;
      })
      .def_property("wm", &WindowStep::wm, &WindowStep::set_wm)
      .def_property_readonly("ctl", [](WindowStep& s) -> WindowControl& { return s.ctl(); },
                             py::return_value_policy::reference_internal)
      .def_property_readonly("world", &WindowStep::world)
      .def_property_readonly("nsub", &WindowStep::nsub)
      .def_property_readonly("nsub_log2", &WindowStep::nsub_log2)
      .def_property_readonly("cap_log2", &WindowStep::cap_log2)
      .def_property_readonly("nslots", &WindowStep::nslots)
      .def_property_readonly("ring", &WindowStep::ring)
      .def_property_readonly("rec_w", &WindowStep::rec_w)
      .def_property_readonly("dense_bits", &WindowStep::dense_bits)
      .def_property_readonly("dense_mul", &WindowStep::dense_mul)
      .def_property_readonly("local_global", &WindowStep::local_global)
      .def_property_readonly("exchanging", &WindowStep::exchanging)
      .def_property_readonly("combine", &WindowStep::combine)
      .def_property_readonly("nbuckets", &WindowStep::nbuckets)
      .def_property_readonly("bucket_cap", &WindowStep::bucket_cap)
      .def_property_readonly("batch_capacity", &WindowStep::batch_capacity)
      .def_property_readonly("pipeline", &WindowStep::pipeline)
      .def_property_readonly("fire_group", &WindowStep::fire_group)
      .def_property_readonly("has_pending", &WindowStep::has_results)
      .def_property_readonly("block_hint", &WindowStep::block_hint)
      .def_property_readonly("use_dlist", &WindowStep::use_dlist)
      .def_property_readonly("async_fire", &WindowStep::async_fire)
      .def_property_readonly("two_level", &WindowStep::two_level)
      .def("set_ccap_hint", &WindowStep::set_ccap_hint)
      .def("set_timing", &WindowStep::set_timing)
      .def("set_jhash", [](WindowStep& s, intptr_t p) { s.set_jhash(reinterpret_cast<const int32_t*>(p)); })
      .def("take_stages", &WindowStep::take_stages)
      .def_property_readonly("ring_m", &WindowStep::ring_m)
      .def_property_readonly("nslots_o", &WindowStep::nslots_o)
      .def_property_readonly("nsub_o", &WindowStep::nsub_o)
      .def_property_readonly("cap_log2_o", &WindowStep::cap_log2_o)
      .def_property_readonly("has_tier", &WindowStep::has_tier)
      .def("tier", [](WindowStep& s) -> WindowTierCore* { return s.tier(); },
           py::return_value_policy::reference_internal);
}
