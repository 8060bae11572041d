// mxstream — pybind11 bindings of the native engine (_mxs_native).
//
// Buffers cross the boundary as integer addresses (torch tensor data_ptr()); the Python layer
// (mxstream/ops/native.py) owns allocation and validates shapes before every launch, so a
// kernel never sees an operand whose shape disagrees with its grid.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#include <hip/hip_runtime_api.h>

#include <cstring>
#include <stdexcept>
#include <string>
#include <tuple>
#include <vector>

#include "ingest.h"
#include "mxs_kernels.h"
#include "mxs_runtime.h"

namespace py = pybind11;
using namespace mxs;

namespace {

template <class T>
T* P(intptr_t p) {
  return reinterpret_cast<T*>(p);
}

ExprProg make_prog(const std::vector<int32_t>& code, const std::vector<double>& consts) {
  ExprProg p;
  std::memset(&p, 0, sizeof(p));
  if (code.size() % 2 != 0) throw std::invalid_argument("expr code must be (op,arg) pairs");
  if (code.size() > (size_t)2 * kExprMaxCode) throw std::invalid_argument("expr program too long");
  if (consts.size() > (size_t)kExprMaxConst) throw std::invalid_argument("too many expr consts");
  // Validate stack discipline so a malformed program can never run off the device stack.
  int sp = 0, depth = 0;
  for (size_t i = 0; i < code.size(); i += 2) {
    const int op = code[i], arg = code[i + 1];
    if (op == OP_VAR) {
      if (arg < 0 || arg >= kExprVars) throw std::invalid_argument("expr var out of range");
      ++sp;
    } else if (op == OP_CONST) {
      if (arg < 0 || arg >= (int)consts.size()) throw std::invalid_argument("expr const out of range");
      ++sp;
    } else if (op == OP_NOT || op == OP_NEG || op == OP_ABS || op == OP_TOINT) {
      if (sp < 1) throw std::invalid_argument("expr stack underflow");
    } else if (op >= OP_ADD && op <= OP_MOD) {
      if (sp < 2) throw std::invalid_argument("expr stack underflow");
      --sp;
    } else {
      throw std::invalid_argument("unknown expr op");
    }
    if (sp > kExprStack) throw std::invalid_argument("expr stack overflow");
    depth = sp > depth ? sp : depth;
  }
  if (!code.empty() && sp != 1) throw std::invalid_argument("expr must leave exactly one value");
  for (size_t i = 0; i < code.size(); ++i) p.code[i] = code[i];
  for (size_t i = 0; i < consts.size(); ++i) p.consts[i] = consts[i];
  p.ncode = (int32_t)(code.size() / 2);
  p.depth = depth;
  p.chain = expr_is_chain(p) ? 1 : 0;
  return p;
}

PartPlan make_part(py::dict d) {
  PartPlan p;
  std::memset(&p, 0, sizeof(p));
  p.max_parallelism = d["max_parallelism"].cast<int32_t>();
  p.nsub_log2 = d["nsub_log2"].cast<int32_t>();
  p.nranks = d["nranks"].cast<int32_t>();
  p.window_mode = d["window_mode"].cast<int32_t>();
  p.drop_late = d["drop_late"].cast<int32_t>();
  p.hash_mode = d["hash_mode"].cast<int32_t>();
  p.bucket_cap = d["bucket_cap"].cast<uint32_t>();
  p.ablate = d.contains("ablate") ? d["ablate"].cast<uint32_t>() : 0u;
  p.key32 = d.contains("key32") ? d["key32"].cast<int32_t>() : 0;
  p.late_ts = d["late_ts"].cast<int64_t>();
  p.tbase = d["tbase"].cast<int64_t>();
  p.pane = d["pane"].cast<int64_t>();
  if (p.window_mode && p.pane <= 0) throw std::invalid_argument("pane length must be positive");
  p.inv_pane = p.pane > 0 ? 1.0 / (double)p.pane : 0.0;
  p.dense_bits = d.contains("dense_bits") ? d["dense_bits"].cast<int32_t>() : 0;
  p.dense_mul = d.contains("dense_mul") ? d["dense_mul"].cast<uint32_t>() : 0u;
  p.key32 = d.contains("key32") ? d["key32"].cast<int32_t>() : 0;
  p.scratch = reinterpret_cast<uint64_t*>(d.contains("scratch") ? d["scratch"].cast<intptr_t>() : 0);
  p.scratch_cursor = reinterpret_cast<uint32_t*>(
      d.contains("scratch_cursor") ? d["scratch_cursor"].cast<intptr_t>() : 0);
  if ((p.scratch != nullptr) != (p.scratch_cursor != nullptr))
    throw std::invalid_argument("two-level partition: scratch and scratch_cursor together");
  if (p.dense_bits < 0 || p.dense_bits > 32 || (p.dense_bits && (p.nranks != 1 ||
      p.nsub_log2 > p.dense_bits || !(p.dense_mul & 1u))))
    throw std::invalid_argument("dense keys: one destination, nsub <= 2^bits, odd multiplier");
  p.rec_words = d.contains("rec_words") ? d["rec_words"].cast<int32_t>() : 3;
  if (p.rec_words < 1 || p.rec_words > 3) throw std::invalid_argument("rec_words must be 1, 2 or 3");
  if (p.rec_words < 3 && !p.window_mode)
    throw std::invalid_argument("compact records are for the window path");
  if (p.rec_words == 1 && p.nranks != 1 && (p.nranks << p.nsub_log2) > 512)
    throw std::invalid_argument("8-byte records to several ranks need <= 512 buckets");
  if (p.max_parallelism <= 0 || p.nranks <= 0 || p.nsub_log2 < 0 || p.nsub_log2 > 20)
    throw std::invalid_argument("bad partition plan");
  return p;
}

ScatPlan make_scat(py::dict d) {
  ScatPlan p{};
  p.max_parallelism = d["max_parallelism"].cast<int32_t>();
  p.nranks = d["nranks"].cast<int32_t>();
  p.nsub_log2 = d["nsub_log2"].cast<int32_t>();
  p.hash_mode = d["hash_mode"].cast<int32_t>();
  p.bucket_cap = d["bucket_cap"].cast<uint32_t>();
  p.n_cap = d["n_cap"].cast<uint32_t>();
  if (p.nranks < 1 || p.nsub_log2 < 0 || (p.nranks << p.nsub_log2) > 16384)
    throw std::invalid_argument("scatter_partials: bad bucket geometry");
  return p;
}

AggPlan make_agg(py::dict d) {
  AggPlan p;
  std::memset(&p, 0, sizeof(p));
  p.cap_log2 = d["cap_log2"].cast<int32_t>();
  p.nsub = d["nsub"].cast<int32_t>();
  p.ring = d["ring"].cast<int32_t>();
  p.agg = d["agg"].cast<int32_t>();
  p.nsrc = d["nsrc"].cast<int32_t>();
  p.bucket_cap = d["bucket_cap"].cast<uint32_t>();
  p.np_step = d["np_step"].cast<int32_t>();
  p.pg = d["pg"].cast<int32_t>();
  p.pane_base = d["pane_base"].cast<int64_t>();
  p.p_lo = d["p_lo"].cast<int64_t>();
  p.fired_hi = d["fired_hi"].cast<int64_t>();
  p.combined = d.contains("combined") ? d["combined"].cast<int32_t>() : 0;
  p.dense_bits = d.contains("dense_bits") ? d["dense_bits"].cast<int32_t>() : 0;
  p.dense_mul = d.contains("dense_mul") ? d["dense_mul"].cast<uint32_t>() : 0u;
  if (p.dense_bits && (p.dense_bits > 32 || !(p.dense_mul & 1u) || p.combined ||
      ((int64_t)p.nsub << p.cap_log2) != ((int64_t)1 << p.dense_bits)))
    throw std::invalid_argument("dense keys: nsub << cap_log2 == 2^bits, odd multiplier, raw records");
  if (d.contains("dlist") && d["dlist"].cast<intptr_t>()) {
    p.dlist = reinterpret_cast<uint32_t*>(d["dlist"].cast<intptr_t>());
    p.dlist_n = reinterpret_cast<uint32_t*>(d["dlist_n"].cast<intptr_t>());
    p.slot_mark = reinterpret_cast<uint32_t*>(d["slot_mark"].cast<intptr_t>());
    if (!p.dlist_n || !p.slot_mark) throw std::invalid_argument("dirty list needs dlist_n and slot_mark");
  }
  p.rec_words = d.contains("rec_words") ? d["rec_words"].cast<int32_t>() : 3;
  if (p.rec_words < 1 || p.rec_words > 3) throw std::invalid_argument("rec_words must be 1, 2 or 3");
  if (p.ring <= 0 || (p.ring & (p.ring - 1))) throw std::invalid_argument("ring must be 2^k");
  if (p.cap_log2 < 4 || p.cap_log2 > 14) throw std::invalid_argument("cap_log2 out of range");
  if (p.pg <= 0) throw std::invalid_argument("pg must be positive");
  p.split = d.contains("split") ? d["split"].cast<int32_t>() : 1;
  p.det = d.contains("det") ? d["det"].cast<int32_t>() : 0;
  if (d.contains("dacc") && d["dacc"].cast<intptr_t>()) {
    p.dacc = reinterpret_cast<uint64_t*>(d["dacc"].cast<intptr_t>());
    p.dcnt = reinterpret_cast<uint32_t*>(d["dcnt"].cast<intptr_t>());
    if (!p.dcnt || !p.dlist) throw std::invalid_argument("delta ring needs dcnt and the slot list");
  }
  // < 0: forced split of every sub-table over -split workgroups (window_agg_kernel)
  if (p.split == 0 || p.split > 1024 || p.split < -64)
    throw std::invalid_argument("agg split out of range");
  p.pmask = d.contains("pmask") ? d["pmask"].cast<uint32_t>() : 0u;
  if (p.pmask && !(p.pmask >> 31) && __builtin_popcount(p.pmask) != p.np_step)
    throw std::invalid_argument("sparse panes: np_step must equal popcount(pmask)");
  return p;
}

FirePlan make_fire(py::dict d) {
  FirePlan p;
  std::memset(&p, 0, sizeof(p));
  p.agg = d["agg"].cast<int32_t>();
  p.npanes = d["npanes"].cast<int32_t>();
  p.ring = d["ring"].cast<int32_t>();
  p.only_dirty = d["only_dirty"].cast<int32_t>();
  p.nslots = d["nslots"].cast<int64_t>();
  p.p0 = d["p0"].cast<int64_t>();
  p.wstart = d["wstart"].cast<double>();
  p.wend = d["wend"].cast<double>();
  p.out_cap = d["out_cap"].cast<uint32_t>();
  p.ablate = d.contains("ablate") ? d["ablate"].cast<uint32_t>() : 0u;
  p.key32 = d.contains("key32") ? d["key32"].cast<int32_t>() : 0;
  if (d.contains("list") && d["list"].cast<intptr_t>()) {
    p.list = reinterpret_cast<const uint32_t*>(d["list"].cast<intptr_t>());
    p.list_n = reinterpret_cast<const uint32_t*>(d["list_n"].cast<intptr_t>());
    if (!p.list_n) throw std::invalid_argument("slot list needs list_n");
  }
  py::tuple m = d["map"].cast<py::tuple>();
  py::tuple f = d["filt"].cast<py::tuple>();
  p.map = make_prog(m[0].cast<std::vector<int32_t>>(), m[1].cast<std::vector<double>>());
  p.filt = make_prog(f[0].cast<std::vector<int32_t>>(), f[1].cast<std::vector<double>>());
  if (p.npanes <= 0 || p.npanes > p.ring) throw std::invalid_argument("window panes exceed ring");
  return p;
}

RollPlan make_roll(py::dict d) {
  RollPlan p;
  std::memset(&p, 0, sizeof(p));
  p.cap_log2 = d["cap_log2"].cast<int32_t>();
  p.nsub = d["nsub"].cast<int32_t>();
  p.agg = d["agg"].cast<int32_t>();
  p.nsrc = d["nsrc"].cast<int32_t>();
  p.bucket_cap = d["bucket_cap"].cast<uint32_t>();
  p.emit = d["emit"].cast<int32_t>();
  return p;
}

IngestSpec make_ingest_spec(py::dict d) {
  IngestSpec sp;
  std::memset(&sp, 0, sizeof(sp));
  auto fields = d["fields"].cast<std::vector<int32_t>>();
  auto kinds = d["kinds"].cast<std::vector<int32_t>>();
  if (fields.empty() || fields.size() > (size_t)kIngestMaxFields || fields.size() != kinds.size())
    throw std::invalid_argument("ingest: 1..8 fields with one kind each");
  sp.nfields = (int32_t)fields.size();
  sp.nstr = 0;
  for (int f = 0; f < sp.nfields; ++f) {
    if (fields[f] < 0 || kinds[f] < IK_STR || kinds[f] > IK_ISO_SEC)
      throw std::invalid_argument("ingest: bad field spec");
    sp.field[f] = fields[f];
    sp.kind[f] = kinds[f];
    sp.sidx[f] = kinds[f] == IK_STR ? sp.nstr++ : -1;
  }
  for (int f = sp.nfields; f < kIngestMaxFields; ++f) sp.sidx[f] = -1;
  sp.ts_col = d["ts_col"].cast<int32_t>();
  if (sp.ts_col >= sp.nfields || (sp.ts_col >= 0 && kinds[sp.ts_col] == IK_STR))
    throw std::invalid_argument("ingest: bad timestamp column");
  sp.offset_s = d["offset_s"].cast<int64_t>();
  const auto sep = d["sep"].cast<std::string>();
  if (sep.size() != 1) throw std::invalid_argument("ingest: separator must be one byte");
  sp.sep = (unsigned char)sep[0];
  return sp;
}

IngestOut make_ingest_out(py::dict d) {
  IngestOut o;
  o.cols = P<int64_t>(d["cols"].cast<intptr_t>());
  o.ids = P<int32_t>(d["ids"].cast<intptr_t>());
  o.status = P<uint8_t>(d["status"].cast<intptr_t>());
  o.spos = P<int64_t>(d["spos"].cast<intptr_t>());
  o.slen = P<int32_t>(d["slen"].cast<intptr_t>());
  o.sjh = P<int32_t>(d["sjh"].cast<intptr_t>());
  o.sslot = P<int32_t>(d["sslot"].cast<intptr_t>());
  o.shash = P<uint64_t>(d["shash"].cast<intptr_t>());
  o.nflag = P<uint32_t>(d["nflag"].cast<intptr_t>());
  o.maxts = P<int64_t>(d["maxts"].cast<intptr_t>());
  o.tile_max = d.contains("tile_max") ? P<int64_t>(d["tile_max"].cast<intptr_t>()) : nullptr;
  return o;
}

DictState make_dict(py::dict d) {
  DictState s;
  s.tab_h = P<uint64_t>(d["tab_h"].cast<intptr_t>());
  s.tab_id = P<int32_t>(d["tab_id"].cast<intptr_t>());
  s.tab_first = P<int64_t>(d["tab_first"].cast<intptr_t>());
  const int64_t cap = d["cap"].cast<int64_t>();
  if (cap < 2 || (cap & (cap - 1)) || cap > (int64_t)1 << 32)
    throw std::invalid_argument("dictionary table capacity must be a power of two <= 2^32");
  s.mask = (uint32_t)(cap - 1);
  s.id_off = P<int64_t>(d["id_off"].cast<intptr_t>());
  s.id_len = P<int32_t>(d["id_len"].cast<intptr_t>());
  s.id_jh = P<int32_t>(d["id_jh"].cast<intptr_t>());
  s.arena = P<uint8_t>(d["arena"].cast<intptr_t>());
  s.arena_cap = d["arena_cap"].cast<int64_t>();
  s.id_cap = d["id_cap"].cast<int64_t>();
  s.ctr = P<int64_t>(d["ctr"].cast<intptr_t>());
  return s;
}

}  // namespace

namespace mxs {
// The validated expression program, for the other binding units (window_step_bindings.cpp).
ExprProg expr_program(const std::vector<int32_t>& code, const std::vector<double>& consts) {
  return make_prog(code, consts);
}
}  // namespace mxs
void bind_window_step(py::module_& m);

PYBIND11_MODULE(_mxs_native, m) {
  m.doc() = "mxstream native engine: gfx950 HIP kernels, C++ CPU twins and host runtime";
  m.attr("REC_BYTES") = (int)sizeof(Rec);
  m.attr("STAT_COUNT") = kStatCount;
  m.attr("EXPR_MAX_CODE") = kExprMaxCode;
  m.attr("EXPR_MAX_CONST") = kExprMaxConst;

  // Pure functions (host) — used for dictionary keys and tests.
  m.def("flink_murmur", &flink_murmur);
  m.def("java_long_hash", &java_long_hash);
  m.def("key_group", &key_group_of_hash);
  m.def("operator_index", &operator_index);
  m.def("mix64", &mix64);
  m.def("window_start", &window_start);
  m.def("expr_eval", [](std::vector<int32_t> code, std::vector<double> consts, std::vector<double> vars) {
    ExprProg p = make_prog(code, consts);
    double v[kExprVars] = {0};
    for (size_t i = 0; i < vars.size() && i < (size_t)kExprVars; ++i) v[i] = vars[i];
    return expr_eval(p, v);
  });
  m.def("expr_is_chain", [](std::vector<int32_t> code, std::vector<double> consts) {
    return make_prog(code, consts).chain != 0;
  });
  m.def("expr_eval_chain", [](std::vector<int32_t> code, std::vector<double> consts,
                              std::vector<double> vars) {
    ExprProg p = make_prog(code, consts);
    if (!p.chain) throw std::invalid_argument("not a chain program");
    double v[kExprVars] = {0};
    for (size_t i = 0; i < vars.size() && i < (size_t)kExprVars; ++i) v[i] = vars[i];
    ArrayVars va{v};
    return expr_eval_chain(p, va);
  });

  // ---- Hot path of the keyed window operator --------------------------------------------
  // Plans as native objects (built once from the dict form, mutated per step: no per-call dict
  // parsing) and one call per step half: step_begin + partition + step_finish, and the
  // aggregation. `gpu` selects the HIP launchers or the C++ twins. Buffers are the operator's
  // own (validated when allocated); the caller checks the batch columns.
  py::class_<PartPlan>(m, "PartPlanObj")
      .def(py::init(&make_part))
      .def_readwrite("late_ts", &PartPlan::late_ts)
      .def_readwrite("tbase", &PartPlan::tbase)
      .def_readwrite("rec_words", &PartPlan::rec_words)
      .def_readwrite("bucket_cap", &PartPlan::bucket_cap)
      .def_readwrite("drop_late", &PartPlan::drop_late)
      .def_property("scratch", [](const PartPlan& a) { return (intptr_t)a.scratch; },
                    [](PartPlan& a, intptr_t v) { a.scratch = reinterpret_cast<uint64_t*>(v); })
      .def_property("scratch_cursor", [](const PartPlan& a) { return (intptr_t)a.scratch_cursor; },
                    [](PartPlan& a, intptr_t v) { a.scratch_cursor = reinterpret_cast<uint32_t*>(v); });
  py::class_<AggPlan>(m, "AggPlanObj")
      .def(py::init(&make_agg))
      .def_readwrite("split", &AggPlan::split)
      .def_property("skip", [](const AggPlan& a) { return (intptr_t)a.skip; },
                    [](AggPlan& a, intptr_t v) { a.skip = reinterpret_cast<const int64_t*>(v); })
      .def_readwrite("bucket_cap", &AggPlan::bucket_cap)
      .def_readwrite("np_step", &AggPlan::np_step)
      .def_readwrite("pg", &AggPlan::pg)
      .def_readwrite("pane_base", &AggPlan::pane_base)
      .def_readwrite("p_lo", &AggPlan::p_lo)
      .def_readwrite("fired_hi", &AggPlan::fired_hi)
      .def_readwrite("rec_words", &AggPlan::rec_words)
      .def_readwrite("ring", &AggPlan::ring)
      .def_readwrite("nsrc", &AggPlan::nsrc)
      .def_readwrite("combined", &AggPlan::combined)
      .def_readwrite("pmask", &AggPlan::pmask);
  m.def("window_front", [](bool gpu, intptr_t keys, intptr_t ts, intptr_t vals, intptr_t jhash,
                           int64_t n, const PartPlan& p, intptr_t kg_dest, intptr_t cursor,
                           intptr_t out, intptr_t stats, intptr_t late_idx, uint32_t late_cap,
                           intptr_t local_maxts, int64_t bound, int32_t event_mode,
                           int64_t proc_now, intptr_t red, intptr_t flags, intptr_t stream) {
    const int nb = p.nranks << p.nsub_log2;
    py::gil_scoped_release nogil;  // loopback ranks are threads of one process
    if (gpu) {
      gpu::step_begin(P<uint32_t>(cursor), nb, P<int64_t>(stats), stream);
      if (n)
        gpu::partition(P<uint64_t>(keys), P<int64_t>(ts), P<uint64_t>(vals), P<int32_t>(jhash), n,
                       p, P<int32_t>(kg_dest), P<uint32_t>(cursor), P<Rec>(out), P<int64_t>(stats),
                       P<uint32_t>(late_idx), late_cap, stream);
      gpu::step_finish(P<int64_t>(stats), P<int64_t>(local_maxts), bound, event_mode, proc_now,
                       P<int64_t>(red), P<uint32_t>(flags), stream);
    } else {
      cpu::step_begin(P<uint32_t>(cursor), nb, P<int64_t>(stats));
      std::vector<uint64_t> wide;
      if (n && p.key32) {  // int32 key ids: sign-extended copy for the CPU kernel
        wide.resize((size_t)n);
        const int32_t* k32 = P<int32_t>(keys);
        for (int64_t i = 0; i < n; ++i) wide[(size_t)i] = (uint64_t)(int64_t)k32[i];
        keys = (intptr_t)wide.data();
      }
      if (n)
        cpu::partition(P<uint64_t>(keys), P<int64_t>(ts), P<uint64_t>(vals), P<int32_t>(jhash), n,
                       p, P<int32_t>(kg_dest), P<uint32_t>(cursor), P<Rec>(out), P<int64_t>(stats),
                       P<uint32_t>(late_idx), late_cap);
      cpu::step_finish(P<int64_t>(stats), P<int64_t>(local_maxts), bound, event_mode, proc_now,
                       P<int64_t>(red), P<uint32_t>(flags));
    }
  });
  m.def("window_agg_obj", [](bool gpu, intptr_t recs, intptr_t counts, const AggPlan& p,
                             intptr_t keys_g, intptr_t acc_g, intptr_t cnt_g, intptr_t dirty_g,
                             intptr_t occ, intptr_t flags, intptr_t stream) {
    py::gil_scoped_release nogil;
    if (gpu)
      gpu::window_agg(P<Rec>(recs), P<uint32_t>(counts), p, P<uint64_t>(keys_g), P<uint64_t>(acc_g),
                      P<uint32_t>(cnt_g), P<uint8_t>(dirty_g), P<uint32_t>(occ), P<uint32_t>(flags),
                      stream);
    else
      cpu::window_agg(P<Rec>(recs), P<uint32_t>(counts), p, P<uint64_t>(keys_g), P<uint64_t>(acc_g),
                      P<uint32_t>(cnt_g), P<uint8_t>(dirty_g), P<uint32_t>(occ), P<uint32_t>(flags));
  });

  // ---- GPU ----
  m.def("gpu_device_count", &gpu::device_count);
  m.def("cpu_set_threads", &cpu::set_threads);
  m.def("cpu_get_threads", &cpu::get_threads);
  m.def("gpu_set_spin_schedule", &gpu::set_spin_schedule);
  m.def("gpu_gen_events", [](intptr_t keys, intptr_t ts, intptr_t vals, int64_t n, uint64_t seed,
                             uint64_t stream_id, uint64_t idx0, uint64_t nkeys, int64_t ts_base,
                             int64_t ts_span, int64_t disorder, int64_t val_lo, int64_t val_span,
                             int32_t val_f64, double zipf_s, intptr_t stream, uint64_t key_base) {
    gpu::gen_events(P<uint64_t>(keys), P<int64_t>(ts), P<uint64_t>(vals), n, seed, stream_id, idx0,
                    nkeys, ts_base, ts_span, disorder, val_lo, val_span, val_f64, zipf_s, stream,
                    key_base);
  }, py::arg("keys"), py::arg("ts"), py::arg("vals"), py::arg("n"), py::arg("seed"),
     py::arg("stream_id"), py::arg("idx0"), py::arg("nkeys"), py::arg("ts_base"),
     py::arg("ts_span"), py::arg("disorder"), py::arg("val_lo"), py::arg("val_span"),
     py::arg("val_f64"), py::arg("zipf_s"), py::arg("stream"), py::arg("key_base") = 0);
  m.def("gpu_partition", [](intptr_t keys, intptr_t ts, intptr_t vals, intptr_t jhash, int64_t n,
                            py::dict plan, intptr_t kg_dest, intptr_t cursor, intptr_t out,
                            intptr_t stats, intptr_t late_idx, uint32_t late_cap, intptr_t stream) {
    gpu::partition(P<uint64_t>(keys), P<int64_t>(ts), P<uint64_t>(vals), P<int32_t>(jhash), n,
                   make_part(plan), P<int32_t>(kg_dest), P<uint32_t>(cursor), P<Rec>(out),
                   P<int64_t>(stats), P<uint32_t>(late_idx), late_cap, stream);
  });
  m.def("gpu_partition_variant", [](intptr_t keys, intptr_t ts, intptr_t vals, intptr_t jhash,
                                    int64_t n, py::dict plan, intptr_t kg_dest, intptr_t cursor,
                                    intptr_t out, intptr_t stats, intptr_t stream, int variant) {
    gpu::partition_variant(P<uint64_t>(keys), P<int64_t>(ts), P<uint64_t>(vals), P<int32_t>(jhash),
                           n, make_part(plan), P<int32_t>(kg_dest), P<uint32_t>(cursor),
                           P<Rec>(out), P<int64_t>(stats), nullptr, 0, stream, variant);
  });
  m.def("gpu_window_agg", [](intptr_t recs, intptr_t counts, py::dict plan, intptr_t keys_g,
                             intptr_t acc_g, intptr_t cnt_g, intptr_t dirty_g, intptr_t occ,
                             intptr_t flags, intptr_t stream) {
    gpu::window_agg(P<Rec>(recs), P<uint32_t>(counts), make_agg(plan), P<uint64_t>(keys_g),
                    P<uint64_t>(acc_g), P<uint32_t>(cnt_g), P<uint8_t>(dirty_g), P<uint32_t>(occ),
                    P<uint32_t>(flags), stream);
  });
  m.def("gpu_window_fire", [](intptr_t keys_g, intptr_t acc_g, intptr_t cnt_g, intptr_t dirty_g,
                              py::dict plan, intptr_t ok, intptr_t ov, intptr_t oraw, intptr_t oc,
                              intptr_t on, intptr_t stream) {
    gpu::window_fire(P<uint64_t>(keys_g), P<uint64_t>(acc_g), P<uint32_t>(cnt_g),
                     P<uint8_t>(dirty_g), make_fire(plan), P<uint64_t>(ok), P<double>(ov),
                     P<uint64_t>(oraw), P<uint32_t>(oc), P<uint32_t>(on), stream);
  });
  m.def("window_fire_many", [](bool cuda, intptr_t keys_g, intptr_t acc_g, intptr_t cnt_g,
                               intptr_t dirty_g, py::dict plan,
                               std::vector<std::tuple<int64_t, int32_t, double, double>> wins,
                               intptr_t ok, intptr_t ov, intptr_t oraw, intptr_t oc, intptr_t on,
                               intptr_t bounds, intptr_t stream, py::object stage) {
    const FirePlan base = make_fire(plan);
    std::vector<FireWin> w(wins.size());
    for (size_t i = 0; i < wins.size(); ++i) {
      w[i].p0 = std::get<0>(wins[i]);
      w[i].npanes = std::get<1>(wins[i]);
      w[i].wstart = std::get<2>(wins[i]);
      w[i].wend = std::get<3>(wins[i]);
      if (w[i].npanes <= 0 || w[i].npanes > base.ring)
        throw std::invalid_argument("window_fire_many: window panes exceed the ring");
    }
    if (!ov || !ok) throw std::invalid_argument("window_fire_many: key and value columns");
    if (cuda) {
      // stage = (keys, vals, raw, cnt, win_n, region): the per-window staging regions
      // (raw / cnt 0 in compact mode)
      const auto t = stage.cast<std::tuple<intptr_t, intptr_t, intptr_t, intptr_t, intptr_t, int64_t>>();
      FireStage st{P<uint64_t>(std::get<0>(t)), P<double>(std::get<1>(t)), P<uint64_t>(std::get<2>(t)),
                   P<uint32_t>(std::get<3>(t)), P<uint32_t>(std::get<4>(t)),
                   (uint32_t)std::get<5>(t)};
      gpu::window_fire_many(P<uint64_t>(keys_g), P<uint64_t>(acc_g), P<uint32_t>(cnt_g),
                            P<uint8_t>(dirty_g), base, w.data(), (int)w.size(), st, P<uint64_t>(ok),
                            P<double>(ov), P<uint64_t>(oraw), P<uint32_t>(oc), P<uint32_t>(on),
                            P<uint32_t>(bounds), stream);
      return;
    }
    py::gil_scoped_release nogil;
    for (size_t i = 0; i < w.size(); ++i) {
      FirePlan p = base;
      p.p0 = w[i].p0;
      p.npanes = w[i].npanes;
      p.wstart = w[i].wstart;
      p.wend = w[i].wend;
      cpu::window_fire(P<uint64_t>(keys_g), P<uint64_t>(acc_g), P<uint32_t>(cnt_g),
                       P<uint8_t>(dirty_g), p, P<uint64_t>(ok), P<double>(ov), P<uint64_t>(oraw),
                       P<uint32_t>(oc), P<uint32_t>(on));
      P<uint32_t>(bounds)[i] = *P<uint32_t>(on);
    }
  });
  // Fused GPU re-firing of several windows over the touched-slot list (plan: list / list_n);
  // stage as in window_fire_many with region = the stage split k ways; ovf: flags word (bit 16 =
  // a window outgrew its region). Returns False when the windows cannot be fused.
  m.def("gpu_window_refire_many", [](intptr_t keys_g, intptr_t acc_g, intptr_t cnt_g,
                                     intptr_t dirty_g, py::dict plan,
                                     std::vector<std::tuple<int64_t, int32_t, double, double>> wins,
                                     intptr_t ok, intptr_t ov, intptr_t oraw, intptr_t oc,
                                     intptr_t on, intptr_t bounds, intptr_t ovf, intptr_t stream,
                                     py::object stage, int64_t dlo, uint32_t dmask) {
    const FirePlan base = make_fire(plan);
    std::vector<FireWin> w(wins.size());
    for (size_t i = 0; i < wins.size(); ++i)
      w[i] = FireWin{std::get<0>(wins[i]), std::get<1>(wins[i]), std::get<2>(wins[i]),
                     std::get<3>(wins[i])};
    const auto t = stage.cast<std::tuple<intptr_t, intptr_t, intptr_t, intptr_t, intptr_t, int64_t>>();
    FireStage st{P<uint64_t>(std::get<0>(t)), P<double>(std::get<1>(t)), P<uint64_t>(std::get<2>(t)),
                 P<uint32_t>(std::get<3>(t)), P<uint32_t>(std::get<4>(t)), (uint32_t)std::get<5>(t)};
    return gpu::window_refire_many(P<uint64_t>(keys_g), P<uint64_t>(acc_g), P<uint32_t>(cnt_g),
                                   P<uint8_t>(dirty_g), base, w.data(), (int)w.size(), st,
                                   P<uint64_t>(ok), P<double>(ov), P<uint64_t>(oraw),
                                   P<uint32_t>(oc), P<uint32_t>(on), P<uint32_t>(bounds),
                                   P<uint32_t>(ovf), stream, dlo, dmask);
  }, py::arg("keys_g"), py::arg("acc_g"), py::arg("cnt_g"), py::arg("dirty_g"), py::arg("plan"),
     py::arg("wins"), py::arg("ok"), py::arg("ov"), py::arg("oraw"), py::arg("oc"), py::arg("on"),
     py::arg("bounds"), py::arg("ovf"), py::arg("stream"), py::arg("stage"), py::arg("dlo") = 0,
     py::arg("dmask") = 0);
  m.def("gpu_rolling", [](intptr_t recs, intptr_t counts, py::dict plan, intptr_t keys_g,
                          intptr_t acc_g, intptr_t cnt_g, intptr_t occ, intptr_t flags,
                          intptr_t out_vals, intptr_t stream) {
    gpu::rolling(P<Rec>(recs), P<uint32_t>(counts), make_roll(plan), P<uint64_t>(keys_g),
                 P<uint64_t>(acc_g), P<uint32_t>(cnt_g), P<uint32_t>(occ), P<uint32_t>(flags),
                 P<uint64_t>(out_vals), stream);
  });
  m.def("gpu_step_begin", [](intptr_t cursor, int nb, intptr_t stats, intptr_t stream) {
    gpu::step_begin(P<uint32_t>(cursor), nb, P<int64_t>(stats), stream);
  });
  m.def("gpu_step_finish", [](intptr_t stats, intptr_t lm, int64_t bound, int32_t ev,
                              int64_t now, intptr_t red, intptr_t flags, intptr_t stream) {
    gpu::step_finish(P<int64_t>(stats), P<int64_t>(lm), bound, ev, now, P<int64_t>(red),
                     P<uint32_t>(flags), stream);
  });
  m.def("gpu_rolling_lookup", [](intptr_t recs, intptr_t counts, int nsrc, int nsub, uint32_t bcap,
                                 int cap_log2, intptr_t keys_g, intptr_t sk, intptr_t vals,
                                 intptr_t n_out, intptr_t flags, int abits, int shift,
                                 intptr_t stream) {
    gpu::rolling_lookup(P<Rec>(recs), P<uint32_t>(counts), nsrc, nsub, bcap, cap_log2,
                        P<uint64_t>(keys_g), P<int64_t>(sk), P<uint64_t>(vals), P<uint32_t>(n_out),
                        P<uint32_t>(flags), abits, shift, stream);
  });
  m.def("gpu_rolling_lookup_direct", [](intptr_t keys, intptr_t vals, uint32_t n, int nsub_log2,
                                        int cap_log2, intptr_t keys_g, intptr_t sk, intptr_t vout,
                                        intptr_t n_out, intptr_t flags, int shift,
                                        intptr_t stream) {
    gpu::rolling_lookup_direct(P<uint64_t>(keys), P<uint64_t>(vals), n, nsub_log2, cap_log2,
                               P<uint64_t>(keys_g), P<int64_t>(sk), P<uint64_t>(vout),
                               P<uint32_t>(n_out), P<uint32_t>(flags), shift, stream);
  });
  m.def("rolling_hist_scratch_bytes", &gpu::rolling_hist_scratch_bytes);
  m.def("rolling_hist_supported", [](int agg, uint32_t count_n, int64_t nslots,
                                     std::vector<int32_t> code, std::vector<double> consts) {
    return gpu::rolling_hist_supported(agg, count_n, nslots, make_prog(code, consts));
  });
  m.def("gpu_rolling_hist", [](intptr_t keys, int64_t n, int nsub_log2, int cap_log2,
                               intptr_t keys_g, intptr_t cnt_g, intptr_t scratch,
                               size_t scratch_bytes, std::vector<int32_t> code,
                               std::vector<double> consts, intptr_t ok, intptr_t ov, intptr_t ot,
                               intptr_t on, uint32_t out_cap, intptr_t flags, int dense,
                               intptr_t stream) {
    gpu::rolling_hist(P<uint64_t>(keys), n, nsub_log2, cap_log2, P<uint64_t>(keys_g),
                      P<uint32_t>(cnt_g), P<void>(scratch), scratch_bytes, make_prog(code, consts),
                      P<uint64_t>(ok), P<uint64_t>(ov), P<int64_t>(ot), P<uint32_t>(on), out_cap,
                      P<uint32_t>(flags), dense, stream);
  });
  m.def("gpu_rolling_heads", [](intptr_t sk, intptr_t n_in, int64_t n_cap, intptr_t heads,
                                intptr_t n_heads, int shift, intptr_t stream) {
    gpu::rolling_heads(P<int64_t>(sk), P<uint32_t>(n_in), n_cap, P<uint32_t>(heads),
                       P<uint32_t>(n_heads), shift, stream);
  });
  m.def("gpu_rolling_scan", [](int agg, intptr_t sk, intptr_t perm, intptr_t vals, intptr_t n_in,
                               intptr_t heads, intptr_t n_heads, int64_t max_segments,
                               intptr_t acc_g, intptr_t cnt_g, intptr_t keys_g,
                               std::vector<int32_t> code, std::vector<double> consts,
                               intptr_t ok, intptr_t ov, intptr_t ot, intptr_t on,
                               uint32_t out_cap, int abits, int shift, intptr_t stream,
                               uint32_t count_n) {
    gpu::rolling_scan(agg, P<int64_t>(sk), P<int64_t>(perm), P<uint64_t>(vals), P<uint32_t>(n_in),
                      P<uint32_t>(heads), P<uint32_t>(n_heads), max_segments, P<uint64_t>(acc_g),
                      P<uint32_t>(cnt_g), P<uint64_t>(keys_g), make_prog(code, consts),
                      P<uint64_t>(ok), P<uint64_t>(ov), P<int64_t>(ot), P<uint32_t>(on), out_cap,
                      abits, shift, stream, count_n);
  });
  m.def("gpu_session_lookup", [](intptr_t recs, intptr_t counts, int nsrc, int nsub, uint32_t bcap,
                                 int cap_log2, intptr_t keys_g, intptr_t spill_set,
                                 uint32_t spill_mask, int spill_any, intptr_t sk, intptr_t vals,
                                 intptr_t n_out, intptr_t host_recs, intptr_t n_host,
                                 uint32_t host_cap, intptr_t n_ins, int tbits, intptr_t stream,
                                 int rec_words) {
    gpu::session_lookup(P<void>(recs), P<uint32_t>(counts), nsrc, nsub, bcap, cap_log2,
                        P<uint64_t>(keys_g), P<uint64_t>(spill_set), spill_mask, spill_any,
                        P<int64_t>(sk), P<uint64_t>(vals), P<uint32_t>(n_out), P<Rec>(host_recs),
                        P<uint32_t>(n_host), host_cap, P<uint32_t>(n_ins), tbits, stream,
                        rec_words);
  }, py::arg("recs"), py::arg("counts"), py::arg("nsrc"), py::arg("nsub"), py::arg("bcap"),
     py::arg("cap_log2"), py::arg("keys_g"), py::arg("spill_set"), py::arg("spill_mask"),
     py::arg("spill_any"), py::arg("sk"), py::arg("vals"), py::arg("n_out"), py::arg("host_recs"),
     py::arg("n_host"), py::arg("host_cap"), py::arg("n_ins"), py::arg("tbits"), py::arg("stream"),
     py::arg("rec_words") = 3);
  m.def("gpu_session_lookup_sort", [](intptr_t recs, intptr_t counts, int nsrc, int nsub,
                                      uint32_t bcap, int cap_log2, intptr_t keys_g,
                                      intptr_t spill_set, uint32_t spill_mask, int spill_any,
                                      intptr_t sk, intptr_t vals, intptr_t n_out,
                                      intptr_t host_recs, intptr_t n_host, uint32_t host_cap,
                                      intptr_t n_ins, int tbits, intptr_t stream, intptr_t skip,
                                      uint32_t skip_mask, intptr_t heads, intptr_t n_heads,
                                      int pair, int rec_words) {
    return gpu::session_lookup_sort(P<void>(recs), P<uint32_t>(counts), nsrc, nsub, bcap, cap_log2,
                                    P<uint64_t>(keys_g), P<uint64_t>(spill_set), spill_mask,
                                    spill_any, P<int64_t>(sk), P<uint64_t>(vals), P<uint32_t>(n_out),
                                    P<Rec>(host_recs), P<uint32_t>(n_host), host_cap,
                                    P<uint32_t>(n_ins), tbits, stream, P<int64_t>(skip), skip_mask,
                                    P<uint64_t>(heads), P<uint32_t>(n_heads), pair, rec_words);
  }, py::arg("recs"), py::arg("counts"), py::arg("nsrc"), py::arg("nsub"), py::arg("bcap"),
     py::arg("cap_log2"), py::arg("keys_g"), py::arg("spill_set"), py::arg("spill_mask"),
     py::arg("spill_any"), py::arg("sk"), py::arg("vals"), py::arg("n_out"), py::arg("host_recs"),
     py::arg("n_host"), py::arg("host_cap"), py::arg("n_ins"), py::arg("tbits"), py::arg("stream"),
     py::arg("skip") = 0, py::arg("skip_mask") = 0, py::arg("heads") = 0, py::arg("n_heads") = 0, py::arg("pair") = 0,
     py::arg("rec_words") = 3);
  m.def("gpu_session_heads", [](intptr_t sk, intptr_t n_in, int64_t n_cap, intptr_t heads,
                                intptr_t n_heads, intptr_t stream) {
    gpu::session_heads(P<int64_t>(sk), P<uint32_t>(n_in), n_cap, P<uint32_t>(heads),
                       P<uint32_t>(n_heads), stream);
  });
  m.def("gpu_session_merge", [](intptr_t sk, intptr_t vals, intptr_t n_in, intptr_t long_heads,
                                intptr_t n_long, int64_t n_cap, int tbits, int64_t gap,
                                int64_t lateness, int64_t wm, int64_t tbase, int agg, int cap_log2,
                                int64_t nslots, intptr_t sess, intptr_t slot_due,
                                intptr_t slot_last, intptr_t late_cnt, intptr_t keys_g,
                                intptr_t ovf_slots, intptr_t n_ovf, intptr_t ovf_rows,
                                intptr_t n_ovf_runs, uint32_t ovf_cap, intptr_t stream) {
    gpu::session_merge(P<int64_t>(sk), P<uint64_t>(vals), P<uint32_t>(n_in),
                       P<uint32_t>(long_heads), P<uint32_t>(n_long), n_cap, tbits, gap, lateness,
                       wm, tbase, agg, cap_log2, nslots, P<int64_t>(sess), P<int64_t>(slot_due),
                       P<int64_t>(slot_last), P<uint64_t>(late_cnt), P<uint64_t>(keys_g),
                       P<int64_t>(ovf_slots),
                       P<uint32_t>(n_ovf), P<int64_t>(ovf_rows), P<uint32_t>(n_ovf_runs), ovf_cap,
                       stream);
  });
  m.def("gpu_session_merge_heads", [](intptr_t sk, intptr_t vals, intptr_t n_in, intptr_t heads,
                                      intptr_t n_heads, int64_t head_cap, intptr_t long_heads,
                                      intptr_t n_long, int tbits, int64_t gap, int64_t lateness,
                                      int64_t wm, int64_t tbase, int agg, int cap_log2,
                                      int64_t nslots, intptr_t sess, intptr_t slot_due,
                                      intptr_t slot_last, intptr_t late_cnt, intptr_t keys_g,
                                      intptr_t ovf_slots, intptr_t n_ovf, intptr_t ovf_rows,
                                      intptr_t n_ovf_runs, uint32_t ovf_cap, intptr_t stream,
                                      int pair) {
    gpu::session_merge_heads(P<int64_t>(sk), P<uint64_t>(vals), P<uint32_t>(n_in),
                             P<uint64_t>(heads), P<uint32_t>(n_heads), head_cap,
                             P<uint32_t>(long_heads), P<uint32_t>(n_long), tbits, gap, lateness,
                             wm, tbase, agg, cap_log2, nslots, P<int64_t>(sess),
                             P<int64_t>(slot_due), P<int64_t>(slot_last), P<uint64_t>(late_cnt),
                             P<uint64_t>(keys_g), P<int64_t>(ovf_slots), P<uint32_t>(n_ovf), P<int64_t>(ovf_rows),
                             P<uint32_t>(n_ovf_runs), ovf_cap, stream, pair);
  }, py::arg("sk"), py::arg("vals"), py::arg("n_in"), py::arg("heads"), py::arg("n_heads"),
     py::arg("head_cap"), py::arg("long_heads"), py::arg("n_long"), py::arg("tbits"),
     py::arg("gap"), py::arg("lateness"), py::arg("wm"), py::arg("tbase"), py::arg("agg"),
     py::arg("cap_log2"), py::arg("nslots"), py::arg("sess"), py::arg("slot_due"),
     py::arg("slot_last"), py::arg("late_cnt"), py::arg("keys_g"), py::arg("ovf_slots"),
     py::arg("n_ovf"),
     py::arg("ovf_rows"), py::arg("n_ovf_runs"), py::arg("ovf_cap"), py::arg("stream"),
     py::arg("pair") = 0);
  m.def("gpu_session_fire", [](int64_t gap, int64_t lateness, int64_t wm, int agg, int cap_log2,
                               int64_t nslots, intptr_t keys_g, intptr_t sess, intptr_t slot_due,
                               std::vector<int32_t> mc, std::vector<double> mk,
                               std::vector<int32_t> fc, std::vector<double> fk, intptr_t ok,
                               intptr_t os, intptr_t oe, intptr_t ov, intptr_t oraw, intptr_t oc,
                               intptr_t on, uint32_t out_cap, intptr_t stream) {
    gpu::session_fire(gap, lateness, wm, agg, cap_log2, nslots, P<uint64_t>(keys_g),
                      P<int64_t>(sess), P<int64_t>(slot_due), make_prog(mc, mk), make_prog(fc, fk),
                      P<uint64_t>(ok), P<int64_t>(os), P<int64_t>(oe), P<double>(ov),
                      P<uint64_t>(oraw), P<uint32_t>(oc), P<uint32_t>(on), out_cap, stream);
  });
  m.def("gpu_session_evict", [](int64_t nslots, int cap_log2, intptr_t keys_g, intptr_t sess,
                                intptr_t slot_due, intptr_t slot_last, int64_t idle_before,
                                intptr_t slots, uint32_t nslots_list, intptr_t spill_set,
                                uint32_t spill_mask, intptr_t st_key, intptr_t st_start,
                                intptr_t st_end, intptr_t st_acc, intptr_t st_cnt,
                                intptr_t st_flags, intptr_t n_rows, uint32_t row_cap,
                                intptr_t n_evicted, intptr_t stream) {
    gpu::session_evict(nslots, cap_log2, P<uint64_t>(keys_g), P<int64_t>(sess),
                       P<int64_t>(slot_due), P<int64_t>(slot_last), idle_before, P<int64_t>(slots),
                       nslots_list, P<uint64_t>(spill_set), spill_mask, P<int64_t>(st_key),
                       P<int64_t>(st_start), P<int64_t>(st_end), P<int64_t>(st_acc),
                       P<int64_t>(st_cnt), P<int64_t>(st_flags), P<uint32_t>(n_rows), row_cap,
                       P<uint32_t>(n_evicted), stream);
  });
  m.def("gpu_sort_pairs_temp_bytes", &gpu::sort_pairs_temp_bytes);
  m.def("gpu_sort_pairs", [](intptr_t temp, size_t temp_bytes, intptr_t kin, intptr_t kout,
                             intptr_t vin, intptr_t vout, int64_t n, int begin_bit, int end_bit,
                             intptr_t stream) {
    gpu::sort_pairs(reinterpret_cast<void*>(temp), temp_bytes, P<uint64_t>(kin), P<uint64_t>(kout),
                    P<uint64_t>(vin), P<uint64_t>(vout), n, begin_bit, end_bit, stream);
  });
  m.def("gpu_keygroups", [](intptr_t keys, int64_t n, int hash_mode, intptr_t jhash, int max_par,
                            intptr_t kg, intptr_t stream) {
    gpu::keygroups(P<uint64_t>(keys), n, hash_mode, P<int32_t>(jhash), max_par, P<int32_t>(kg),
                   stream);
  });
  m.def("cpu_keygroups", [](intptr_t keys, int64_t n, int hash_mode, intptr_t jhash, int max_par,
                            intptr_t kg) {
    cpu::keygroups(P<uint64_t>(keys), n, hash_mode, P<int32_t>(jhash), max_par, P<int32_t>(kg));
  });
  m.def("gpu_table_insert", [](intptr_t keys, int64_t n, int nsub_log2, int cap_log2,
                               intptr_t keys_g, intptr_t slots, intptr_t stream) {
    gpu::table_insert(P<uint64_t>(keys), n, nsub_log2, cap_log2, P<uint64_t>(keys_g),
                      P<int64_t>(slots), stream);
  });
  m.def("cpu_table_insert", [](intptr_t keys, int64_t n, int nsub_log2, int cap_log2,
                               intptr_t keys_g, intptr_t slots) {
    cpu::table_insert(P<uint64_t>(keys), n, nsub_log2, cap_log2, P<uint64_t>(keys_g),
                      P<int64_t>(slots));
  });
  // Fired rows -> one pinned host slab: one hipMemcpyAsync per column on `stream`, no sync
  // (window_operator.to_host_arrays syncs once). copies = [(src, nbytes, dst_offset)].
  m.def("gpu_h2d_async", [](intptr_t dst, intptr_t src, int64_t bytes, intptr_t stream) {
    return gpu::h2d_async((void*)dst, (const void*)src, (size_t)bytes, stream);
  });
  // Wait for a HIP event by polling hipEventQuery with the GIL released: the host resumes
  // within a microsecond of the event (a blocking hipEventSynchronize sleeps in the driver and
  // wakes tens of microseconds late), and other Python threads (loopback ranks, workers) keep
  // the interpreter meanwhile -- the Python `while not ev.query()` loop held it. Returns the
  // hipError_t of the final query (0 = complete).
  m.def("gpu_event_spin", [](intptr_t ev) {
    py::gil_scoped_release nogil;
    hipError_t e;
    while ((e = hipEventQuery((hipEvent_t)ev)) == hipErrorNotReady) __builtin_ia32_pause();
    return (int)e;
  });
  // Packed-row exchange (parallel/exchange.py): cols = [(src ptr, dst ptr, words per row)].
  auto xcols = [](const std::vector<std::tuple<intptr_t, intptr_t, int>>& cols) {
    if (cols.empty() || cols.size() > 8) throw std::invalid_argument("exchange_rows: 1..8 columns");
    XRowCols c{};
    c.ncol = (int)cols.size();
    c.rw = 0;
    for (int k = 0; k < c.ncol; ++k) {
      c.src[k] = P<const uint32_t>(std::get<0>(cols[k]));
      c.dst[k] = P<uint32_t>(std::get<1>(cols[k]));
      c.words[k] = std::get<2>(cols[k]);
      c.rw += c.words[k];
    }
    return c;
  };
  m.def("xrows_blocks", &gpu::xrows_blocks);
  m.def("gpu_xrows_count", [](intptr_t dest, int64_t n, int world, intptr_t blk, intptr_t counts,
                              intptr_t bad, intptr_t stream) {
    gpu::xrows_count(P<int64_t>(dest), n, world, P<uint32_t>(blk), P<uint32_t>(counts),
                     P<uint32_t>(bad), stream);
  });
  m.def("gpu_xrows_scatter", [xcols](intptr_t dest, int64_t n, int world, intptr_t blk,
                                     uint32_t cap, const std::vector<std::tuple<intptr_t, intptr_t, int>>& cols,
                                     intptr_t send, intptr_t ovf, intptr_t stream) {
    gpu::xrows_scatter(P<int64_t>(dest), n, world, P<uint32_t>(blk), cap, xcols(cols),
                       P<uint32_t>(send), P<uint32_t>(ovf), stream);
  });
  m.def("gpu_xrows_unpack", [xcols](intptr_t recv, intptr_t rc, int world, uint32_t cap,
                                    const std::vector<std::tuple<intptr_t, intptr_t, int>>& cols,
                                    intptr_t stream) {
    gpu::xrows_unpack(P<uint32_t>(recv), P<uint32_t>(rc), world, cap, xcols(cols), stream);
  });
  m.def("cpu_xrows_count", [](intptr_t dest, int64_t n, int world, intptr_t counts, intptr_t bad) {
    cpu::xrows_count(P<int64_t>(dest), n, world, P<uint32_t>(counts), P<uint32_t>(bad));
  });
  m.def("cpu_xrows_scatter", [xcols](intptr_t dest, int64_t n, int world, uint32_t cap,
                                     const std::vector<std::tuple<intptr_t, intptr_t, int>>& cols,
                                     intptr_t send, intptr_t ovf) {
    cpu::xrows_scatter(P<int64_t>(dest), n, world, cap, xcols(cols), P<uint32_t>(send),
                       P<uint32_t>(ovf));
  });
  m.def("cpu_xrows_unpack", [xcols](intptr_t recv, intptr_t rc, int world, uint32_t cap,
                                    const std::vector<std::tuple<intptr_t, intptr_t, int>>& cols) {
    cpu::xrows_unpack(P<uint32_t>(recv), P<uint32_t>(rc), world, cap, xcols(cols));
  });
  m.def("gpu_host_register_flags", [](intptr_t p, int64_t bytes, unsigned flags) {
    py::gil_scoped_release nogil;
    return (int)hipHostRegister((void*)p, (size_t)bytes, flags);
  });
  m.def("gpu_host_register", [](intptr_t p, int64_t bytes) {
    return gpu::host_register((void*)p, (size_t)bytes);
  });
  m.def("gpu_host_unregister", [](intptr_t p) { return gpu::host_unregister((void*)p); });
  m.def("gpu_d2h_many", [](intptr_t dst, const std::vector<std::tuple<intptr_t, int64_t, int64_t>>& copies,
                           intptr_t stream) {
    for (const auto& c : copies) {
      const int e = gpu::d2h_async((char*)dst + std::get<2>(c), (const void*)std::get<0>(c),
                                   (size_t)std::get<1>(c), stream);
      if (e != 0) throw std::runtime_error("hipMemcpyAsync D2H failed: " + std::to_string(e));
    }
  });
  m.def("gpu_h2d_kernel", [](intptr_t dst, intptr_t src, int64_t bytes, intptr_t stream,
                             int max_blocks) {
    return gpu::h2d_kernel((void*)dst, (const void*)src, bytes, stream, max_blocks);
  }, py::arg("dst"), py::arg("src"), py::arg("bytes"), py::arg("stream"),
     py::arg("max_blocks") = 1024);
  // Kernel variant of gpu_d2h_many (16-byte granules); returns the hipError_t code (0 = ok).
  m.def("gpu_d2h_kernel", [](intptr_t dst, const std::vector<std::tuple<intptr_t, int64_t, int64_t>>& copies,
                             intptr_t stream) {
    if (copies.size() > (size_t)kD2HMax) throw std::invalid_argument("gpu_d2h_kernel: too many columns");
    D2HCopy c[kD2HMax];
    for (size_t i = 0; i < copies.size(); ++i)
      c[i] = D2HCopy{(const void*)std::get<0>(copies[i]), std::get<1>(copies[i]), std::get<2>(copies[i])};
    return gpu::d2h_kernel((void*)dst, c, (int)copies.size(), stream);
  });
  // Copy kernel whose row count is read on the device (no host sync before the copy):
  // copies = [(src, max_bytes, dst_offset, element_size)] (element_size 0: copy max_bytes as is);
  // n_dev = uint32 row counter. Returns the hipError_t code (0 = ok).
  m.def("gpu_d2h_counted", [](intptr_t dst,
                              const std::vector<std::tuple<intptr_t, int64_t, int64_t, int64_t>>& copies,
                              intptr_t n_dev, intptr_t stream, int max_blocks) {
    if (copies.empty() || copies.size() > (size_t)kD2HMax)
      throw std::invalid_argument("gpu_d2h_counted: 1..8 columns");
    D2HCopy c[kD2HMax];
    for (size_t i = 0; i < copies.size(); ++i)
      c[i] = D2HCopy{(const void*)std::get<0>(copies[i]), std::get<1>(copies[i]),
                     std::get<2>(copies[i]), std::get<3>(copies[i])};
    return gpu::d2h_kernel((void*)dst, c, (int)copies.size(), stream, P<uint32_t>(n_dev),
                           max_blocks);
  }, py::arg("dst"), py::arg("copies"), py::arg("n_dev"), py::arg("stream"),
     py::arg("max_blocks") = 1024);
  // Keyed-window compaction / eviction (host-DRAM spill tier). out = (key, pane, acc, cnt, dirty,
  // n, cap, counters) pointers.
  auto compact_out = [](const std::vector<intptr_t>& o, uint32_t cap) {
    if (o.size() != 7) throw std::invalid_argument("window_compact: 7 output pointers");
    return CompactOut{P<uint64_t>(o[0]), P<int64_t>(o[1]), P<uint64_t>(o[2]), P<uint32_t>(o[3]),
                      P<uint8_t>(o[4]), P<uint32_t>(o[5]), cap, P<uint32_t>(o[6])};
  };
  m.def("gpu_window_compact", [compact_out](intptr_t keys_g, intptr_t acc_g, intptr_t cnt_g,
                                            intptr_t dirty_g, int nsub, int cap_log2, int ring,
                                            int64_t p_lo, int np, int64_t cutoff,
                                            std::vector<intptr_t> o, uint32_t cap, intptr_t occ,
                                            intptr_t stream) {
    gpu::window_compact(P<uint64_t>(keys_g), P<uint64_t>(acc_g), P<uint32_t>(cnt_g),
                        P<uint8_t>(dirty_g), nsub, cap_log2, ring, p_lo, np, cutoff,
                        compact_out(o, cap), P<uint32_t>(occ), stream);
  });
  m.def("gpu_window_rows_pane_sort", [](intptr_t key, intptr_t pane, intptr_t acc, intptr_t cnt,
                                         intptr_t dirty, intptr_t n_dev, uint32_t cap,
                                         int64_t p_lo, int np, intptr_t okey, intptr_t oacc,
                                         intptr_t ocnt, intptr_t odirty, intptr_t counts,
                                         intptr_t stream) {
    gpu::window_rows_pane_sort(P<uint64_t>(key), P<int64_t>(pane), P<uint64_t>(acc),
                               P<uint32_t>(cnt), P<uint8_t>(dirty), P<uint32_t>(n_dev), cap, p_lo,
                               np, P<uint64_t>(okey), P<uint64_t>(oacc), P<uint32_t>(ocnt),
                               P<uint8_t>(odirty), P<uint32_t>(counts), stream);
  });
  m.def("cpu_window_compact", [compact_out](intptr_t keys_g, intptr_t acc_g, intptr_t cnt_g,
                                            intptr_t dirty_g, int nsub, int cap_log2, int ring,
                                            int64_t p_lo, int np, int64_t cutoff,
                                            std::vector<intptr_t> o, uint32_t cap, intptr_t occ) {
    py::gil_scoped_release nogil;
    cpu::window_compact(P<uint64_t>(keys_g), P<uint64_t>(acc_g), P<uint32_t>(cnt_g),
                        P<uint8_t>(dirty_g), nsub, cap_log2, ring, p_lo, np, cutoff,
                        compact_out(o, cap), P<uint32_t>(occ));
  });
  // print() rows formatted where the columns live (csrc/row_format.h). `d`: cols [(kind,
  // width, ptr)], arena / id_off / id_len / n_ids of the dictionary, sub / sub0 / par, prefix
  // bytes + offsets (npfx), as_tuple. Stage "len": lengths + flag; "write": bytes at `end`.
  auto fmt_args = [](const py::dict& d) {
    FmtArgs a{};
    const auto cols = d["cols"].cast<std::vector<std::tuple<int, int, intptr_t>>>();
    if (cols.empty() || cols.size() > (size_t)kFmtMaxCols)
      throw std::invalid_argument("format_rows: 1..8 columns");
    a.ncols = (int32_t)cols.size();
    for (size_t j = 0; j < cols.size(); ++j) {
      const int kind = std::get<0>(cols[j]), width = std::get<1>(cols[j]);
      if (kind < 0 || kind > 2 || (width != 4 && width != 8) || (kind == 1 && width != 8))
        throw std::invalid_argument("format_rows: column kind / width");
      a.col[j] = FmtCol{kind, width, reinterpret_cast<const void*>(std::get<2>(cols[j]))};
      if (kind == 0 && d["n_ids"].cast<int64_t>() > 0 && !d["arena"].cast<intptr_t>())
        throw std::invalid_argument("format_rows: string column without a dictionary");
    }
    a.as_tuple = d["as_tuple"].cast<bool>() ? 1 : 0;
    if (!a.as_tuple && a.ncols != 1) throw std::invalid_argument("format_rows: arity");
    a.arena = P<uint8_t>(d["arena"].cast<intptr_t>());
    a.id_off = P<int64_t>(d["id_off"].cast<intptr_t>());
    a.id_len = P<int32_t>(d["id_len"].cast<intptr_t>());
    a.n_ids = d["n_ids"].cast<int64_t>();
    a.sub = P<int32_t>(d["sub"].cast<intptr_t>());
    a.sub0 = d["sub0"].cast<int64_t>();
    a.par = d["par"].cast<int32_t>();
    a.npfx = d["npfx"].cast<int32_t>();
    a.pfx = P<char>(d["pfx"].cast<intptr_t>());
    a.pfx_off = P<int32_t>(d["pfx_off"].cast<intptr_t>());
    return a;
  };
  m.def("format_rows_len", [fmt_args](bool gpu, const py::dict& d, int64_t n, intptr_t len,
                                      intptr_t bad, intptr_t stream) {
    const FmtArgs a = fmt_args(d);
    if (gpu) {
      gpu::format_rows_len(a, n, P<int64_t>(len), P<uint32_t>(bad), stream);
    } else {
      py::gil_scoped_release nogil;
      cpu::format_rows_len(a, n, P<int64_t>(len), P<uint32_t>(bad));
    }
  });
  m.def("format_rows_write", [fmt_args](bool gpu, const py::dict& d, int64_t n, intptr_t end,
                                        intptr_t out, intptr_t stream) {
    const FmtArgs a = fmt_args(d);
    if (gpu) {
      gpu::format_rows_write(a, n, P<int64_t>(end), P<char>(out), stream);
    } else {
      py::gil_scoped_release nogil;
      cpu::format_rows_write(a, n, P<int64_t>(end), P<char>(out));
    }
  });
  // Tiered firing: rows -> per-key combine table (mxs_kernels.h tier_merge).
  m.def("tier_merge", [](bool gpu, intptr_t keys, intptr_t acc, intptr_t cnt, int64_t n,
                         intptr_t n_dev, int mode, int agg, intptr_t tkeys, intptr_t tacc,
                         intptr_t tcnt, intptr_t tdirty, uint32_t mask, intptr_t flags,
                         intptr_t stream) {
    if (gpu) {
      gpu::tier_merge(P<uint64_t>(keys), P<uint64_t>(acc), P<uint32_t>(cnt), n,
                      P<uint32_t>(n_dev), mode, agg, P<uint64_t>(tkeys), P<uint64_t>(tacc),
                      P<uint32_t>(tcnt), P<uint8_t>(tdirty), mask, P<uint32_t>(flags), stream);
    } else {
      py::gil_scoped_release nogil;
      cpu::tier_merge(P<uint64_t>(keys), P<uint64_t>(acc), P<uint32_t>(cnt), n,
                      P<uint32_t>(n_dev), mode, agg, P<uint64_t>(tkeys), P<uint64_t>(tacc),
                      P<uint32_t>(tcnt), P<uint8_t>(tdirty), mask, P<uint32_t>(flags));
    }
  });
  m.def("gpu_direct_agg_probe", [](intptr_t keys, intptr_t ts, intptr_t vals, int64_t n,
                                   int64_t tbase, int64_t pane, int ring, int64_t nslots,
                                   uint32_t mul, int bits, int64_t pane_base, intptr_t acc,
                                   intptr_t cnt, int mode, intptr_t sink, int grid,
                                   intptr_t stream) {
    gpu::direct_agg_probe(P<uint64_t>(keys), P<int64_t>(ts), P<uint64_t>(vals), n, tbase, pane,
                          ring, nslots, mul, bits, pane_base, P<uint64_t>(acc), P<uint32_t>(cnt),
                          mode, P<uint64_t>(sink), grid, stream);
  });
  m.def("gpu_dirty_clear", [](intptr_t list, intptr_t list_n, uint32_t cap, int ring,
                              int64_t nslots, intptr_t dirty_g, intptr_t mark, int64_t p_lo, int np,
                              intptr_t stream, intptr_t dacc, intptr_t dcnt) {
    gpu::dirty_clear(P<uint32_t>(list), P<uint32_t>(list_n), cap, ring, nslots, P<uint8_t>(dirty_g),
                     P<uint32_t>(mark), p_lo, np, stream, P<uint64_t>(dacc), P<uint32_t>(dcnt));
  }, py::arg("list"), py::arg("list_n"), py::arg("cap"), py::arg("ring"), py::arg("nslots"),
     py::arg("dirty_g"), py::arg("mark"), py::arg("p_lo"), py::arg("np"), py::arg("stream"),
     py::arg("dacc") = 0, py::arg("dcnt") = 0);
  m.def("cpu_dirty_clear", [](intptr_t list, intptr_t list_n, uint32_t cap, int ring,
                              int64_t nslots, intptr_t dirty_g, intptr_t mark, int64_t p_lo, int np,
                              intptr_t dacc, intptr_t dcnt) {
    cpu::dirty_clear(P<uint32_t>(list), P<uint32_t>(list_n), cap, ring, nslots, P<uint8_t>(dirty_g),
                     P<uint32_t>(mark), p_lo, np, P<uint64_t>(dacc), P<uint32_t>(dcnt));
  }, py::arg("list"), py::arg("list_n"), py::arg("cap"), py::arg("ring"), py::arg("nslots"),
     py::arg("dirty_g"), py::arg("mark"), py::arg("p_lo"), py::arg("np"), py::arg("dacc") = 0,
     py::arg("dcnt") = 0);
  m.def("gpu_scatter_partials", [](intptr_t keys, intptr_t acc, intptr_t cnt, intptr_t n_in,
                                   py::dict plan, intptr_t jhash, intptr_t kg_dest,
                                   intptr_t cursor, intptr_t out, intptr_t flags, intptr_t stream) {
    gpu::scatter_partials(P<uint64_t>(keys), P<uint64_t>(acc), P<uint32_t>(cnt), P<uint32_t>(n_in),
                          make_scat(plan), P<int32_t>(jhash), P<int32_t>(kg_dest),
                          P<uint32_t>(cursor), P<Rec>(out), P<uint32_t>(flags), stream);
  });
  m.def("cpu_scatter_partials", [](intptr_t keys, intptr_t acc, intptr_t cnt, intptr_t n_in,
                                   py::dict plan, intptr_t jhash, intptr_t kg_dest,
                                   intptr_t cursor, intptr_t out, intptr_t flags) {
    cpu::scatter_partials(P<uint64_t>(keys), P<uint64_t>(acc), P<uint32_t>(cnt), P<uint32_t>(n_in),
                          make_scat(plan), P<int32_t>(jhash), P<int32_t>(kg_dest),
                          P<uint32_t>(cursor), P<Rec>(out), P<uint32_t>(flags));
  });
  m.def("gpu_window_combine", [](intptr_t recs, intptr_t counts, int nbuckets, py::dict plan,
                                 intptr_t out, uint32_t ccap, intptr_t out_counts, intptr_t flags,
                                 intptr_t stream) {
    gpu::window_combine(P<Rec>(recs), P<uint32_t>(counts), nbuckets, make_agg(plan), P<Rec>(out),
                        ccap, P<uint32_t>(out_counts), P<uint32_t>(flags), stream);
  });
  m.def("cpu_window_combine", [](intptr_t recs, intptr_t counts, int nbuckets, py::dict plan,
                                 intptr_t out, uint32_t ccap, intptr_t out_counts, intptr_t flags) {
    cpu::window_combine(P<Rec>(recs), P<uint32_t>(counts), nbuckets, make_agg(plan), P<Rec>(out),
                        ccap, P<uint32_t>(out_counts), P<uint32_t>(flags));
  });
  // nlines: the number of lines, or (nlines_dev != 0) the bound the outputs are sized for, the
  // count itself read by the kernel from nlines_dev (line_starts' device total, no host sync).
  m.def("gpu_parse_text", [](intptr_t text, int64_t text_len, intptr_t starts, int64_t nlines,
                             std::vector<int32_t> fields, std::vector<int32_t> kinds,
                             std::string sep, int64_t offset_s, intptr_t cols, intptr_t jhash,
                             intptr_t status, intptr_t stream, intptr_t nlines_dev,
                             intptr_t nflag) {
    if (fields.size() != kinds.size() || sep.size() != 1)
      throw std::invalid_argument("parse_text: spec / separator");
    gpu::parse_text(reinterpret_cast<const char*>(text), text_len, P<int64_t>(starts), nlines,
                    fields.data(), kinds.data(), (int)fields.size(), sep[0], offset_s,
                    P<int64_t>(cols), P<int32_t>(jhash), P<uint8_t>(status), stream,
                    P<int64_t>(nlines_dev), P<uint32_t>(nflag));
  }, py::arg("text"), py::arg("text_len"), py::arg("starts"), py::arg("nlines"), py::arg("fields"),
     py::arg("kinds"), py::arg("sep"), py::arg("offset_s"), py::arg("cols"), py::arg("jhash"),
     py::arg("status"), py::arg("stream"), py::arg("nlines_dev") = 0, py::arg("nflag") = 0);
  m.def("gpu_f64_order_bits", [](intptr_t v, int64_t n, intptr_t o, intptr_t stream) {
    gpu::f64_order_bits(P<uint64_t>(v), n, P<uint64_t>(o), stream);
  });
  m.def("cpu_f64_order_bits", [](intptr_t v, int64_t n, intptr_t o) {
    cpu::f64_order_bits(P<uint64_t>(v), n, P<uint64_t>(o));
  });
  m.def("gpu_segment_median_select", [](intptr_t heads, int64_t nseg, int64_t total, intptr_t ord,
                                        intptr_t out, intptr_t stream) {
    gpu::segment_median_select(P<int64_t>(heads), nseg, total, P<uint64_t>(ord), P<double>(out),
                               stream);
  });
  m.def("cpu_segment_median_select", [](intptr_t heads, int64_t nseg, int64_t total, intptr_t ord,
                                        intptr_t out) {
    py::gil_scoped_release nogil;
    cpu::segment_median_select(P<int64_t>(heads), nseg, total, P<uint64_t>(ord), P<double>(out));
  });
  m.def("gpu_segment_median", [](intptr_t heads, int64_t nseg, int64_t total, intptr_t ord,
                                 intptr_t out, intptr_t stream) {
    gpu::segment_median(P<int64_t>(heads), nseg, total, P<uint64_t>(ord), P<double>(out), stream);
  });
  m.def("cpu_segment_median", [](intptr_t heads, int64_t nseg, int64_t total, intptr_t ord,
                                 intptr_t out) {
    cpu::segment_median(P<int64_t>(heads), nseg, total, P<uint64_t>(ord), P<double>(out));
  });
  m.def("gpu_session_slot_insert", [](intptr_t keys, int64_t n, int nsub_log2, int cap_log2,
                                      intptr_t keys_g, intptr_t slots, intptr_t ins,
                                      intptr_t stream) {
    gpu::session_slot_insert(P<uint64_t>(keys), n, nsub_log2, cap_log2, P<uint64_t>(keys_g),
                             P<int64_t>(slots), P<uint32_t>(ins), stream);
  });
  m.def("gpu_session_promote", [](intptr_t slots, intptr_t rec, intptr_t last, int64_t n,
                                  intptr_t sess, intptr_t due, intptr_t slast, intptr_t n_bad,
                                  intptr_t stream) {
    gpu::session_promote(P<int64_t>(slots), P<int64_t>(rec), P<int64_t>(last), n, P<int64_t>(sess),
                         P<int64_t>(due), P<int64_t>(slast), P<uint32_t>(n_bad), stream);
  });
  m.def("gpu_session_promote_rows", [](intptr_t rows, int64_t n, int nsub_log2, int cap_log2,
                                       intptr_t keys_g, intptr_t slots, intptr_t sess, intptr_t due,
                                       intptr_t slast, intptr_t ins, intptr_t n_bad,
                                       intptr_t stream) {
    gpu::session_promote_rows(P<int64_t>(rows), n, nsub_log2, cap_log2, P<uint64_t>(keys_g),
                              P<int64_t>(slots), P<int64_t>(sess), P<int64_t>(due),
                              P<int64_t>(slast), P<uint32_t>(ins), P<uint32_t>(n_bad), stream);
  });
  m.def("gpu_set_rehash", [](intptr_t old, int64_t n_old, intptr_t neu, uint32_t new_mask,
                             intptr_t stream) {
    gpu::set_rehash(P<uint64_t>(old), n_old, P<uint64_t>(neu), new_mask, stream);
  });
  m.def("gpu_set_insert", [](intptr_t set, uint32_t mask, intptr_t keys, int64_t n,
                             intptr_t stream) {
    gpu::set_insert_keys(P<uint64_t>(set), mask, P<int64_t>(keys), n, stream);
  });
  m.def("gpu_set_probe", [](intptr_t set, uint32_t mask, intptr_t keys, int64_t n, intptr_t hit,
                            intptr_t n_hit, intptr_t stream) {
    gpu::set_probe(P<uint64_t>(set), mask, P<int64_t>(keys), n, P<uint8_t>(hit),
                   P<uint32_t>(n_hit), stream);
  });
  m.def("gpu_set_erase", [](intptr_t set, uint32_t mask, intptr_t keys, int64_t n,
                            intptr_t stream) {
    gpu::set_erase(P<uint64_t>(set), mask, P<int64_t>(keys), n, stream);
  });
  m.def("gpu_session_rehash", [](int64_t nslots, int cap_log2, intptr_t keys_o, intptr_t sess_o,
                                 intptr_t due_o, intptr_t last_o, intptr_t keys_n, intptr_t sess_n,
                                 intptr_t due_n, intptr_t last_n, intptr_t ins, intptr_t stream) {
    gpu::session_rehash(nslots, cap_log2, P<uint64_t>(keys_o), P<int64_t>(sess_o),
                        P<int64_t>(due_o), P<int64_t>(last_o), P<uint64_t>(keys_n),
                        P<int64_t>(sess_n), P<int64_t>(due_n), P<int64_t>(last_n),
                        P<uint32_t>(ins), stream);
  });
  m.def("gpu_filter_compact_scratch_bytes", &gpu::filter_compact_scratch_bytes);
  // ---- device text ingest + string dictionary (csrc/ingest*.{h,hip,cpp}) ----
  m.def("ingest_parse", [](bool cuda, intptr_t text, int64_t text_len, intptr_t starts, int64_t n,
                           py::dict spec, py::dict out, py::dict dict, intptr_t stream) {
    const IngestSpec sp = make_ingest_spec(spec);
    const IngestOut o = make_ingest_out(out);
    const DictState d = make_dict(dict);
    if (cuda) {
      gpu::ingest_parse(P<char>(text), text_len, P<int64_t>(starts), n, sp, o, d, stream);
    } else {
      py::gil_scoped_release nogil;
      cpu::ingest_parse(P<char>(text), text_len, P<int64_t>(starts), n, sp, o, d);
    }
  });
  m.def("dict_assign_new", [](bool cuda, intptr_t text, int64_t n, int32_t nstr, py::dict out,
                              py::dict dict, intptr_t scratch, intptr_t newpos, intptr_t stream) {
    const IngestOut o = make_ingest_out(out);
    const DictState d = make_dict(dict);
    if (cuda) {
      gpu::dict_assign_new(P<char>(text), n, nstr, o, d, P<void>(scratch), P<int64_t>(newpos),
                           stream);
    } else {
      py::gil_scoped_release nogil;
      cpu::dict_assign_new(P<char>(text), n, nstr, o, d, P<int64_t>(newpos));
    }
  });
  m.def("dict_find_new", [](bool cuda, int64_t n, int32_t nstr, py::dict out, py::dict dict,
                            intptr_t scratch, intptr_t newpos, intptr_t stream) {
    const IngestOut o = make_ingest_out(out);
    const DictState d = make_dict(dict);
    if (cuda) gpu::dict_find_new(n, nstr, o, d, P<void>(scratch), P<int64_t>(newpos), stream);
    else cpu::dict_find_new(n, nstr, o, d, P<int64_t>(newpos));
  });
  m.def("dict_insert_ids", [](bool cuda, intptr_t buf, intptr_t offs, intptr_t lens, int64_t k,
                              int64_t id0, py::dict dict, intptr_t stream) {
    const DictState d = make_dict(dict);
    if (cuda) {
      gpu::dict_insert_ids(P<uint8_t>(buf), P<int64_t>(offs), P<int32_t>(lens), k, id0, d, stream);
    } else {
      cpu::dict_insert_ids(P<uint8_t>(buf), P<int64_t>(offs), P<int32_t>(lens), k, id0, d);
    }
  });
  m.def("dict_resolve", [](bool cuda, intptr_t text, int64_t n, int32_t nstr, py::dict out,
                           py::dict dict, intptr_t stream) {
    const IngestOut o = make_ingest_out(out);
    const DictState d = make_dict(dict);
    if (cuda) gpu::dict_resolve(P<char>(text), n, nstr, o, d, stream);
    else cpu::dict_resolve(P<char>(text), n, nstr, o, d);
  });
  m.def("dict_rehash", [](bool cuda, intptr_t old_h, intptr_t old_id, int64_t old_cap,
                          py::dict dict, intptr_t stream) {
    const DictState d = make_dict(dict);
    if (cuda) gpu::dict_rehash(P<uint64_t>(old_h), P<int32_t>(old_id), old_cap, d, stream);
    else cpu::dict_rehash(P<uint64_t>(old_h), P<int32_t>(old_id), old_cap, d);
  });
  m.def("ingest_filter_compact", [](bool cuda, intptr_t cols, int64_t n, int32_t nf,
                                    int32_t dbl_mask, std::vector<int32_t> code,
                                    std::vector<double> consts, intptr_t scratch, intptr_t idx,
                                    intptr_t total, intptr_t stream) {
    if (nf < 1 || nf > kIngestMaxFields) throw std::invalid_argument("ingest filter: 1..8 columns");
    const ExprProg p = make_prog(code, consts);
    if (cuda) {
      gpu::ingest_filter_compact(P<int64_t>(cols), n, nf, dbl_mask, p, P<void>(scratch),
                                 P<int64_t>(idx), P<int64_t>(total), stream);
    } else {
      py::gil_scoped_release nogil;
      cpu::ingest_filter_compact(P<int64_t>(cols), n, nf, dbl_mask, p, P<int64_t>(idx),
                                 P<int64_t>(total));
    }
  });
  m.def("ingest_gather", [](bool cuda, intptr_t cols, int64_t n, int32_t nf, intptr_t ids,
                            int32_t nstr, intptr_t idx, intptr_t total, intptr_t out_cols,
                            intptr_t out_ids, int64_t out_stride, intptr_t stream) {
    if (cuda) {
      gpu::ingest_gather(P<int64_t>(cols), n, nf, P<int32_t>(ids), nstr, P<int64_t>(idx),
                         P<int64_t>(total), P<int64_t>(out_cols), P<int32_t>(out_ids), out_stride,
                         stream);
    } else {
      cpu::ingest_gather(P<int64_t>(cols), n, nf, P<int32_t>(ids), nstr, P<int64_t>(idx),
                         P<int64_t>(total), P<int64_t>(out_cols), P<int32_t>(out_ids), out_stride);
    }
  });
  m.def("cpu_line_starts", [](intptr_t buf, int64_t n, intptr_t idx, intptr_t total) {
    py::gil_scoped_release nogil;
    cpu::line_starts(P<uint8_t>(buf), n, P<int64_t>(idx), P<int64_t>(total));
  });
  // cap: entries of idx (starts past it are counted, not written; total is always exact)
  m.def("gpu_line_starts", [](intptr_t buf, int64_t n, intptr_t scratch, intptr_t idx,
                              intptr_t total, intptr_t stream, int64_t cap) {
    gpu::line_starts(P<uint8_t>(buf), n, P<void>(scratch), P<int64_t>(idx), P<int64_t>(total),
                     stream, cap < 0 ? INT64_MAX : cap);
  }, py::arg("buf"), py::arg("n"), py::arg("scratch"), py::arg("idx"), py::arg("total"),
     py::arg("stream"), py::arg("cap") = -1);
  m.def("gpu_expr_filter_compact", [](intptr_t x, int64_t n, std::vector<int32_t> code,
                                      std::vector<double> consts, intptr_t scratch, intptr_t idx,
                                      intptr_t total, intptr_t stream) {
    gpu::expr_filter_compact(P<double>(x), n, make_prog(code, consts), P<void>(scratch),
                             P<int64_t>(idx), P<int64_t>(total), stream);
  });
  m.def("gpu_expr_filter", [](intptr_t x, int64_t n, std::vector<int32_t> code,
                              std::vector<double> consts, intptr_t keep, intptr_t stream) {
    gpu::expr_filter(P<double>(x), n, make_prog(code, consts), P<uint8_t>(keep), stream);
  });

  // ---- CPU twins ----
  m.def("cpu_gen_events", [](intptr_t keys, intptr_t ts, intptr_t vals, int64_t n, uint64_t seed,
                             uint64_t stream_id, uint64_t idx0, uint64_t nkeys, int64_t ts_base,
                             int64_t ts_span, int64_t disorder, int64_t val_lo, int64_t val_span,
                             int32_t val_f64, double zipf_s, uint64_t key_base) {
    py::gil_scoped_release nogil;
    cpu::gen_events(P<uint64_t>(keys), P<int64_t>(ts), P<uint64_t>(vals), n, seed, stream_id, idx0,
                    nkeys, ts_base, ts_span, disorder, val_lo, val_span, val_f64, zipf_s, key_base);
  }, py::arg("keys"), py::arg("ts"), py::arg("vals"), py::arg("n"), py::arg("seed"),
     py::arg("stream_id"), py::arg("idx0"), py::arg("nkeys"), py::arg("ts_base"),
     py::arg("ts_span"), py::arg("disorder"), py::arg("val_lo"), py::arg("val_span"),
     py::arg("val_f64"), py::arg("zipf_s"), py::arg("key_base") = 0);
  m.def("cpu_partition", [](intptr_t keys, intptr_t ts, intptr_t vals, intptr_t jhash, int64_t n,
                            py::dict plan, intptr_t kg_dest, intptr_t cursor, intptr_t out,
                            intptr_t stats, intptr_t late_idx, uint32_t late_cap) {
    PartPlan pp = make_part(plan);
    py::gil_scoped_release nogil;
    cpu::partition(P<uint64_t>(keys), P<int64_t>(ts), P<uint64_t>(vals), P<int32_t>(jhash), n, pp,
                   P<int32_t>(kg_dest), P<uint32_t>(cursor), P<Rec>(out), P<int64_t>(stats),
                   P<uint32_t>(late_idx), late_cap);
  });
  m.def("cpu_window_agg", [](intptr_t recs, intptr_t counts, py::dict plan, intptr_t keys_g,
                             intptr_t acc_g, intptr_t cnt_g, intptr_t dirty_g, intptr_t occ,
                             intptr_t flags) {
    AggPlan ap = make_agg(plan);
    py::gil_scoped_release nogil;
    cpu::window_agg(P<Rec>(recs), P<uint32_t>(counts), ap, P<uint64_t>(keys_g), P<uint64_t>(acc_g),
                    P<uint32_t>(cnt_g), P<uint8_t>(dirty_g), P<uint32_t>(occ), P<uint32_t>(flags));
  });
  m.def("cpu_window_fire", [](intptr_t keys_g, intptr_t acc_g, intptr_t cnt_g, intptr_t dirty_g,
                              py::dict plan, intptr_t ok, intptr_t ov, intptr_t oraw, intptr_t oc,
                              intptr_t on) {
    FirePlan fp = make_fire(plan);
    py::gil_scoped_release nogil;
    cpu::window_fire(P<uint64_t>(keys_g), P<uint64_t>(acc_g), P<uint32_t>(cnt_g),
                     P<uint8_t>(dirty_g), fp, P<uint64_t>(ok), P<double>(ov), P<uint64_t>(oraw),
                     P<uint32_t>(oc), P<uint32_t>(on));
  });
  m.def("cpu_rolling", [](intptr_t recs, intptr_t counts, py::dict plan, intptr_t keys_g,
                          intptr_t acc_g, intptr_t cnt_g, intptr_t occ, intptr_t flags,
                          intptr_t out_vals) {
    RollPlan rp = make_roll(plan);
    py::gil_scoped_release nogil;
    cpu::rolling(P<Rec>(recs), P<uint32_t>(counts), rp, P<uint64_t>(keys_g), P<uint64_t>(acc_g),
                 P<uint32_t>(cnt_g), P<uint32_t>(occ), P<uint32_t>(flags), P<uint64_t>(out_vals));
  });
  m.def("cpu_step_begin", [](intptr_t cursor, int nb, intptr_t stats) {
    cpu::step_begin(P<uint32_t>(cursor), nb, P<int64_t>(stats));
  });
  m.def("cpu_step_finish", [](intptr_t stats, intptr_t lm, int64_t bound, int32_t ev, int64_t now,
                              intptr_t red, intptr_t flags) {
    cpu::step_finish(P<int64_t>(stats), P<int64_t>(lm), bound, ev, now, P<int64_t>(red),
                     P<uint32_t>(flags));
  });
  m.def("cpu_rolling_rows", [](intptr_t recs, intptr_t counts, int nsrc, int nsub, uint32_t bcap,
                               int cap_log2, int agg, intptr_t keys_g, intptr_t acc_g,
                               intptr_t cnt_g, intptr_t flags, std::vector<int32_t> code,
                               std::vector<double> consts, intptr_t ok, intptr_t ov, intptr_t ot,
                               intptr_t on, uint32_t out_cap, uint32_t count_n) {
    ExprProg f = make_prog(code, consts);
    py::gil_scoped_release nogil;
    cpu::rolling_rows(P<Rec>(recs), P<uint32_t>(counts), nsrc, nsub, bcap, cap_log2, agg,
                      P<uint64_t>(keys_g), P<uint64_t>(acc_g), P<uint32_t>(cnt_g),
                      P<uint32_t>(flags), f, P<uint64_t>(ok), P<uint64_t>(ov), P<int64_t>(ot),
                      P<uint32_t>(on), out_cap, count_n);
  });
  m.def("cpu_expr_filter_compact", [](intptr_t x, int64_t n, std::vector<int32_t> code,
                                      std::vector<double> consts, intptr_t idx, intptr_t total) {
    ExprProg p = make_prog(code, consts);
    py::gil_scoped_release nogil;
    cpu::expr_filter_compact(P<double>(x), n, p, P<int64_t>(idx), P<int64_t>(total));
  });
  m.def("cpu_expr_filter", [](intptr_t x, int64_t n, std::vector<int32_t> code,
                              std::vector<double> consts, intptr_t keep) {
    ExprProg p = make_prog(code, consts);
    py::gil_scoped_release nogil;
    cpu::expr_filter(P<double>(x), n, p, P<uint8_t>(keep));
  });

  bind_runtime(m);
  bind_sessions(m);
  bind_vector(m);
  bind_trace(m);
  bind_check(m);
  bind_reader(m);
  bind_format(m);
  bind_listwin(m);
  bind_window_tier(m);
  bind_window_control(m);
  bind_window_step(m);
}
