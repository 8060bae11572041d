// mxstream — shared host/device definitions.
//
// Everything in this header is compiled twice: once into the gfx950 code object (HIP kernels in
// kernels_hip.hip) and once into the host C++ twins (kernels_cpu.cpp), so the CPU engine and the
// GPU engine compute bit-identical key groups, sub-table ids, pane ids and expression results.
//
// Flink parity notes:
//   * key group   = murmur(javaHash(key)) % maxParallelism   (Flink KeyGroupRangeAssignment)
//   * subtask     = kg * parallelism / maxParallelism          (operatorIndex)
//   * window start= ts - (ts - offset + size) % size           (TimeWindow.getWindowStartWithOffset)
//   * late        = lastWindow.maxTs + allowedLateness <= wm   (WindowOperator.isElementLate, all windows)
// Reference call sites: chapter2/src/main/java/me/zjy/ComputeCpuMax.java:26 (keyBy),
// chapter3/src/main/java/me/zjy/BandwidthMonitorWithEventTime.java:46 (sliding event-time window).
#pragma once
#include <math.h>
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define MXS_HD __host__ __device__ __forceinline__
#else
#define MXS_HD inline
#endif

namespace mxs {

// Empty slot marker of the keyed hash tables. User keys are 64-bit ids (integer keys, or string
// dictionary ids assigned by the host); the all-ones id is reserved.
constexpr uint64_t kEmptyKey = ~0ull;
// Tombstone marker of tables with deletion (sessions). Keys >= kTombKey (ids -1 and -2) are
// reserved: the partition pass reports them instead of routing them.
constexpr uint64_t kTombKey = ~1ull;
constexpr uint32_t kNoSlot = 0xFFFFFFFFu;

// Shuffle / bucket record: 24 bytes, AoS so one all-to-all moves a whole bucket range.
//   key : 64-bit key id
//   val : 64-bit payload (int64 or float64 bit pattern)
//   t   : pane id relative to the step's pane base (window ops) or ts relative to ts base
//   aux : original index of the event inside its source batch (ordered operators) / user field
struct alignas(8) Rec {
  uint64_t key;
  uint64_t val;
  uint32_t t;
  uint32_t aux;
};
static_assert(sizeof(Rec) == 24, "Rec must be 24 bytes");

// Compact 16-byte record (window path with integer aggregates whose values fit int32): one
// 16-byte vector per record, 4 records per 64-byte sector.
struct alignas(16) RecC {
  uint64_t key;
  uint32_t val;  // int32 value (sign-extended on load)
  uint32_t t;    // relative pane; 0xFFFFFFFF = hole
};
static_assert(sizeof(RecC) == 16, "RecC must be 16 bytes");

// Narrow 8-byte record (window path with integer aggregates when one destination owns every
// key: G = 1 or local-global aggregation): 32-bit key id, value in 28 bits (signed), relative
// pane in 4 bits; vt = value << 4 | t, t = 15 marks a hole. A record that does not fit sets
// overflow bit 16 and the step is redone with 16-byte records (sticky).
struct RecN {
  uint32_t key;
  uint32_t vt;
};
static_assert(sizeof(RecN) == 8, "RecN must be 8 bytes");
constexpr uint32_t kNarrowHoleT = 15u;
// Skewed synthetic keys: a power law with exponent s over ranks [0, nkeys) (rank 0 hottest),
// by inverting the continuous CDF of x^-s on [1, nkeys + 1] at u = the top 53 bits of r.
// A Zipf-like workload for hot-key benchmarks; not bit-identical between CPU and GPU.
MXS_HD uint64_t zipf_key(uint64_t r, uint64_t nkeys, double s) {
  const double u = (double)((r >> 11) + 1) * (1.0 / 9007199254740992.0);  // (0, 1]
  const double top = (double)nkeys + 1.0;
  double x;
  if (s > 0.999999 && s < 1.000001) {
    x = exp(u * log(top));
  } else {
    const double a = 1.0 - s;
    x = pow(1.0 + u * (pow(top, a) - 1.0), 1.0 / a);
  }
  const double k = floor(x) - 1.0;
  return k < 0.0 ? 0ull : k >= (double)nkeys ? nkeys - 1 : (uint64_t)k;
}

MXS_HD bool narrow_fits(uint64_t key, int64_t v, uint32_t t) {
  return key < 0xFFFFFFFFull && v >= -(int64_t(1) << 27) && v < (int64_t(1) << 27) &&
         t < kNarrowHoleT;
}

// ---------------------------------------------------------------------------------------------
// Java / Flink hashing
// ---------------------------------------------------------------------------------------------
MXS_HD int32_t rotl32(int32_t x, int r) {
  uint32_t u = (uint32_t)x;
  return (int32_t)((u << r) | (u >> (32 - r)));
}

// Flink MathUtils.murmurHash(int) — returns a non-negative int.
MXS_HD int32_t flink_murmur(int32_t code) {
  uint32_t h = (uint32_t)code;
  h *= 0xcc9e2d51u;
  h = (uint32_t)rotl32((int32_t)h, 15);
  h *= 0x1b873593u;
  h = (uint32_t)rotl32((int32_t)h, 13);
  h = h * 5u + 0xe6546b64u;
  h ^= 4u;
  // bitMix (fmix32)
  h ^= h >> 16;
  h *= 0x85ebca6bu;
  h ^= h >> 13;
  h *= 0xc2b2ae35u;
  h ^= h >> 16;
  int32_t c = (int32_t)h;
  if (c >= 0) return c;
  if (c != (int32_t)0x80000000) return -c;
  return 0;
}

// java.lang.Long.hashCode
MXS_HD int32_t java_long_hash(int64_t v) {
  uint64_t u = (uint64_t)v;
  return (int32_t)(uint32_t)(u ^ (u >> 32));
}

MXS_HD int32_t key_group_of_hash(int32_t java_hash, int32_t max_parallelism) {
  // flink_murmur is non-negative, so for a power-of-two max parallelism (Flink's default 128)
  // the remainder is a mask -- an int32 division is ~30 instructions per element on the GPU,
  // and the partition evaluates this for every record at G > 1.
  const int32_t h = flink_murmur(java_hash);
  return (max_parallelism & (max_parallelism - 1)) == 0 ? (h & (max_parallelism - 1))
                                                        : h % max_parallelism;
}

MXS_HD int32_t operator_index(int32_t key_group, int32_t parallelism, int32_t max_parallelism) {
  return (int32_t)(((int64_t)key_group * parallelism) / max_parallelism);
}

// splitmix64 finaliser: the engine-internal hash that picks a key's probe start in its sub-table
// (low bits; the sub-table itself comes from sub_table_of) — independent of the Flink key-group
// hash so that every rank's sub-tables stay balanced whatever key groups it owns.
MXS_HD uint64_t mix64(uint64_t x) {
  x += 0x9e3779b97f4a7c15ull;
  x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ull;
  x = (x ^ (x >> 27)) * 0x94d049bb133111ebull;
  return x ^ (x >> 31);
}

// Counter-based RNG for the synthetic source (stateless, reproducible for any G / batch split).
MXS_HD uint64_t rng64(uint64_t seed, uint64_t stream, uint64_t idx) {
  return mix64(mix64(seed ^ (stream * 0xd1b54a32d192ed03ull)) + idx * 0x9e3779b97f4a7c15ull);
}

MXS_HD uint64_t mulhi_u64(uint64_t a, uint64_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __umul64hi(a, b);
#else
  return (uint64_t)(((unsigned __int128)a * b) >> 64);
#endif
}

// r * n >> 32 for n <= 2^32: a uniform draw in [0, n) from 32 random bits (one 32x32 -> 64
// multiply on the device instead of the four of a 64-bit high product).
MXS_HD uint64_t draw32(uint32_t r, uint64_t n) { return ((uint64_t)r * n) >> 32; }

// One synthetic event (the source of the benchmarks and tests; CPU and GPU bit-identical except
// with zipf_s > 0): two splitmix64 words per event -- the key from the high half of the first
// (all of it for key spaces beyond 2^32 or the power law), the disorder from the low half of
// the second and the value from its high half (32-bit draws whenever the range fits).
// `base` = rng64's per-(seed, stream) word mix64(seed ^ stream * C), hoisted by the caller.
MXS_HD void gen_event(uint64_t base, uint64_t idx, int64_t i, uint64_t nkeys, int64_t ts_base,
                      double span_per_event, uint64_t disorder_p1, int64_t val_lo,
                      uint64_t val_span, double zipf_s, uint64_t& key, int64_t& t, int64_t& v) {
  const uint64_t r = mix64(base + idx * 0x9e3779b97f4a7c15ull);
  const uint64_t r2 = mix64(r);
  key = zipf_s > 0.0 ? zipf_key(r, nkeys, zipf_s)
                     : (nkeys <= (1ull << 32) ? draw32((uint32_t)(r >> 32), nkeys) : mulhi_u64(r, nkeys));
  t = ts_base + (int64_t)((double)i * span_per_event);
  if (disorder_p1 > 1)
    t -= (int64_t)(disorder_p1 <= (1ull << 32) ? draw32((uint32_t)r2, disorder_p1)
                                               : mulhi_u64(r2, disorder_p1));
  v = val_lo + (int64_t)(val_span == 0 ? 0
                         : val_span <= (1ull << 32) ? draw32((uint32_t)(r2 >> 32), val_span)
                                                    : mulhi_u64(mix64(r2), val_span));
}

// ---------------------------------------------------------------------------------------------
// Window math (Flink 1.8 TimeWindow semantics, Java '%' = truncated remainder)
// ---------------------------------------------------------------------------------------------
MXS_HD int64_t window_start(int64_t ts, int64_t offset, int64_t size) {
  return ts - (ts - offset + size) % size;
}

// Floor division for pane ids (panes are a partition of the time axis, also for ts < 0).
MXS_HD int64_t floor_div(int64_t a, int64_t b) {
  int64_t q = a / b;
  if ((a % b != 0) && ((a < 0) != (b < 0))) --q;
  return q;
}

// Window-assignment parameters shared by the partition pass and the fire pass.
struct WinParams {
  int64_t size;       // window size (ms)
  int64_t slide;      // slide (ms); == size for tumbling
  int64_t offset;     // window offset (ms)
  int64_t pane;       // pane length = gcd(size, slide)
  int64_t lateness;   // allowed lateness (ms)
};

// True iff every window the element belongs to is already past its cleanup time.
MXS_HD bool element_is_late(int64_t ts, const WinParams& w, int64_t wm) {
  const int64_t last_start = window_start(ts, w.offset, w.slide);
  const int64_t cleanup = last_start + w.size - 1 + w.lateness;
  return cleanup <= wm;
}

MXS_HD int64_t pane_of(int64_t ts, const WinParams& w) { return floor_div(ts - w.offset, w.pane); }

// ---------------------------------------------------------------------------------------------
// Aggregation kinds
// ---------------------------------------------------------------------------------------------
enum AggKind : int32_t {
  AGG_SUM_I64 = 0,
  AGG_SUM_F64 = 1,
  AGG_MIN_I64 = 2,
  AGG_MAX_I64 = 3,
  AGG_MIN_F64 = 4,
  AGG_MAX_F64 = 5,
  AGG_COUNT = 6,  // value ignored, result = count
  AGG_AVG_F64 = 7,  // acc = sum f64, result = sum / count (ComputeCpuAvg.java:47-50)
  AGG_AVG_I64 = 8,  // acc = sum i64, result = (double)sum / count
};

MXS_HD bool agg_is_f64(int32_t k) {
  return k == AGG_SUM_F64 || k == AGG_MIN_F64 || k == AGG_MAX_F64 || k == AGG_AVG_F64;
}

MXS_HD double as_f64(uint64_t bits) {
  union { uint64_t u; double d; } c;
  c.u = bits;
  return c.d;
}
MXS_HD uint64_t f64_bits(double d) {
  union { uint64_t u; double d; } c;
  c.d = d;
  return c.u;
}

// ---------------------------------------------------------------------------------------------
// Deterministic f64 sums (AggPlan.det): a step's per-slot sum is accumulated as a 128-bit
// two's-complement fixed-point number with 64 fraction bits. Integer addition is associative and
// commutative, so the result does not depend on the order in which LDS atomics (or the C++
// twin's loop) add the values; it is converted to a double once. Values are truncated to
// multiples of 2^-64 (|x| < 2^-64 adds 0) and must satisfy |x| < 2^63; NaN/Inf are rejected.
// ---------------------------------------------------------------------------------------------
MXS_HD bool f64_to_fx(double x, uint64_t* lo, uint64_t* hi) {
  const uint64_t bits = f64_bits(x);
  const int ex = (int)((bits >> 52) & 0x7FF);
  *lo = 0;
  *hi = 0;
  if (ex == 0x7FF) return false;  // Inf / NaN
  if (ex == 0) return true;       // zero / subnormal: below the fixed-point resolution
  const uint64_t m = (bits & ((1ull << 52) - 1)) | (1ull << 52);
  const int sh = ex - 1011;       // x = m * 2^(ex - 1075); fixed = x * 2^64 = m * 2^sh
  if (sh > 74) return false;      // |x| >= 2^63
  unsigned __int128 mag;
  if (sh >= 0) mag = (unsigned __int128)m << sh;
  else mag = -sh >= 64 ? 0 : (unsigned __int128)(m >> -sh);
  if (bits >> 63) mag = (unsigned __int128)0 - mag;
  *lo = (uint64_t)mag;
  *hi = (uint64_t)(mag >> 64);
  return true;
}

MXS_HD int clz64(uint64_t v) {
#if defined(__HIP_DEVICE_COMPILE__)
  return v ? __clzll((long long)v) : 64;
#else
  return v ? __builtin_clzll(v) : 64;
#endif
}

MXS_HD double fx_to_f64(uint64_t lo, uint64_t hi) {
  unsigned __int128 v = ((unsigned __int128)hi << 64) | lo;
  const bool neg = (int64_t)hi < 0;
  if (neg) v = (unsigned __int128)0 - v;
  const uint64_t vh = (uint64_t)(v >> 64), vl = (uint64_t)v;
  if (!vh && !vl) return 0.0;
  // Top 64 significant bits -> double (one u64 -> f64 rounding), times 2^(shift - 64).
  const int shift = vh ? 64 - clz64(vh) : 0;
  const uint64_t top = shift ? (uint64_t)(v >> shift) : vl;
  const double scale = as_f64((uint64_t)(1023 + shift - 64) << 52);
  const double d = (double)top * scale;
  return neg ? -d : d;
}

// Combine two partial accumulators (host side and device write-back).
MXS_HD uint64_t agg_combine(int32_t k, uint64_t a, uint64_t b) {
  switch (k) {
    case AGG_SUM_I64:
    case AGG_AVG_I64:
    case AGG_COUNT:
      return (uint64_t)((int64_t)a + (int64_t)b);
    case AGG_SUM_F64:
    case AGG_AVG_F64:
      return f64_bits(as_f64(a) + as_f64(b));
    case AGG_MIN_I64:
      return ((int64_t)a < (int64_t)b) ? a : b;
    case AGG_MAX_I64:
      return ((int64_t)a > (int64_t)b) ? a : b;
    case AGG_MIN_F64:
      return (as_f64(a) < as_f64(b)) ? a : b;
    case AGG_MAX_F64:
      return (as_f64(a) > as_f64(b)) ? a : b;
  }
  return a;
}

// Identity of agg_combine (the initial accumulator of a table combined with atomics).
MXS_HD uint64_t agg_identity(int32_t k) {
  switch (k) {
    case AGG_MIN_I64:
      return (uint64_t)INT64_MAX;
    case AGG_MAX_I64:
      return (uint64_t)INT64_MIN;
    case AGG_MIN_F64:
      return 0x7FF0000000000000ull;  // +inf
    case AGG_MAX_F64:
      return 0xFFF0000000000000ull;  // -inf
    default:
      return 0;
  }
}

// The accumulator value a single element contributes.
MXS_HD uint64_t agg_lift(int32_t k, uint64_t v) { return k == AGG_COUNT ? 1ull : v; }

// Final window result as double (what getResult / the chained map sees).
MXS_HD double agg_result_f64(int32_t k, uint64_t acc, uint32_t cnt) {
  switch (k) {
    case AGG_SUM_F64:
    case AGG_MIN_F64:
    case AGG_MAX_F64:
      return as_f64(acc);
    case AGG_AVG_F64:
      return cnt == 0 ? 0.0 : as_f64(acc) / (double)cnt;
    case AGG_AVG_I64:
      return cnt == 0 ? 0.0 : (double)(int64_t)acc / (double)cnt;
    case AGG_COUNT:
      return (double)cnt;
    default:
      return (double)(int64_t)acc;
  }
}

// ---------------------------------------------------------------------------------------------
// Expression VM — the planner traces user map/filter lambdas (e.g. the Mbps map + `< 100` filter
// of BandwidthMonitorWithEventTime.java:48-55) into this bytecode; the fire kernel and the
// stateless filter kernel evaluate it per row. Java double semantics: every op rounds once, no
// contraction (kernels are built with -ffp-contract=off).
// ---------------------------------------------------------------------------------------------
enum ExprOp : int32_t {
  OP_END = 0,
  OP_VAR = 1,    // push vars[arg]
  OP_CONST = 2,  // push consts[arg]
  OP_ADD = 3,
  OP_SUB = 4,
  OP_MUL = 5,
  OP_DIV = 6,
  OP_LT = 7,
  OP_LE = 8,
  OP_GT = 9,
  OP_GE = 10,
  OP_EQ = 11,
  OP_NE = 12,
  OP_AND = 13,
  OP_OR = 14,
  OP_NOT = 15,
  OP_NEG = 16,
  OP_ABS = 17,
  OP_MIN = 18,
  OP_MAX = 19,
  OP_MOD = 20,   // Java double %, fmod
  OP_TOINT = 21, // (long) cast toward zero
};

constexpr int kExprMaxCode = 64;
constexpr int kExprMaxConst = 16;
constexpr int kExprStack = 16;

// Variables visible to window epilogues:
//   0 = aggregated result (double), 1 = count, 2 = window start, 3 = window end,
//   4 = key (as double), 5 = raw accumulator as integer (double), 6 = previous program's output
constexpr int kExprVars = 8;

struct ExprProg {
  int32_t code[kExprMaxCode];  // (op, arg) pairs
  double consts[kExprMaxConst];
  int32_t ncode;               // number of (op,arg) pairs; 0 = empty program
  int32_t depth;               // max stack depth (validated on the host)
  int32_t chain;               // 1: "VAR, (CONST|VAR, binop)*" — evaluated without a stack
};

// The VM is templated on where its stack lives: a local array on the host, a per-lane LDS
// column on the GPU (a runtime-indexed private array would be spilled to scratch memory).
struct LocalStack {
  double v[kExprStack];
  MXS_HD double get(int i) const { return v[i]; }
  MXS_HD void set(int i, double x) { v[i] = x; }
};

template <class Stack, class Vars>
MXS_HD double expr_eval_t(const ExprProg& p, Stack& st, const Vars& vars) {
  int sp = 0;
  for (int i = 0; i < p.ncode; ++i) {
    const int32_t op = p.code[2 * i];
    const int32_t arg = p.code[2 * i + 1];
    switch (op) {
      case OP_VAR: st.set(sp++, vars.get(arg)); break;
      case OP_CONST: st.set(sp++, p.consts[arg]); break;
      case OP_NOT: st.set(sp - 1, st.get(sp - 1) == 0.0 ? 1.0 : 0.0); break;
      case OP_NEG: st.set(sp - 1, -st.get(sp - 1)); break;
      case OP_ABS: { const double a = st.get(sp - 1); st.set(sp - 1, a < 0 ? -a : a); break; }
      case OP_TOINT: st.set(sp - 1, (double)(int64_t)st.get(sp - 1)); break;
      default: {
        const double b = st.get(--sp);
        const double a = st.get(sp - 1);
        double r = 0.0;
        switch (op) {
          case OP_ADD: r = a + b; break;
          case OP_SUB: r = a - b; break;
          case OP_MUL: r = a * b; break;
          case OP_DIV: r = a / b; break;
          case OP_LT: r = a < b; break;
          case OP_LE: r = a <= b; break;
          case OP_GT: r = a > b; break;
          case OP_GE: r = a >= b; break;
          case OP_EQ: r = a == b; break;
          case OP_NE: r = a != b; break;
          case OP_AND: r = (a != 0.0) && (b != 0.0); break;
          case OP_OR: r = (a != 0.0) || (b != 0.0); break;
          case OP_MIN: r = a < b ? a : b; break;
          case OP_MAX: r = a > b ? a : b; break;
#if defined(__HIP_DEVICE_COMPILE__)
          case OP_MOD: r = fmod(a, b); break;
#else
          case OP_MOD: r = __builtin_fmod(a, b); break;
#endif
          default: break;
        }
        st.set(sp - 1, r);
      }
    }
  }
  return sp > 0 ? st.get(sp - 1) : 0.0;
}

// Binary op of the VM (shared by the stack VM's semantics and the chain evaluator).
MXS_HD double expr_binop(int32_t op, double a, double b) {
  switch (op) {
    case OP_ADD: return a + b;
    case OP_SUB: return a - b;
    case OP_MUL: return a * b;
    case OP_DIV: return a / b;
    case OP_LT: return a < b;
    case OP_LE: return a <= b;
    case OP_GT: return a > b;
    case OP_GE: return a >= b;
    case OP_EQ: return a == b;
    case OP_NE: return a != b;
    case OP_AND: return (a != 0.0) && (b != 0.0);
    case OP_OR: return (a != 0.0) || (b != 0.0);
    case OP_MIN: return a < b ? a : b;
    case OP_MAX: return a > b ? a : b;
#if defined(__HIP_DEVICE_COMPILE__)
    case OP_MOD: return fmod(a, b);
#else
    case OP_MOD: return __builtin_fmod(a, b);
#endif
    default: return 0.0;
  }
}

// Stack-free evaluation of chain programs (the traced epilogues of the reference jobs:
// `sum * 8.0 / 60 / 1024 / 1024`, `mbps < 100.0`): the running value is the left operand of
// every binop, so it stays in a register — the same double ops in the same order as the VM
// (bit-identical results), without the VM's per-op LDS stack traffic.
template <class Vars>
MXS_HD double expr_eval_chain(const ExprProg& p, const Vars& vars) {
  double x = vars.get(p.code[1]);
  for (int i = 1; i + 1 < p.ncode; i += 2) {
    const int32_t pop = p.code[2 * i], parg = p.code[2 * i + 1];
    const double b = pop == OP_CONST ? p.consts[parg] : vars.get(parg);
    x = expr_binop(p.code[2 * (i + 1)], x, b);
  }
  return x;
}

// Host-side classification (bindings: make_prog).
inline bool expr_is_chain(const ExprProg& p) {
  if (p.ncode < 1 || p.code[0] != OP_VAR || (p.ncode - 1) % 2 != 0) return false;
  for (int i = 1; i < p.ncode; i += 2) {
    const int32_t pop = p.code[2 * i], op = p.code[2 * (i + 1)];
    if (pop != OP_CONST && pop != OP_VAR) return false;
    if (op < OP_ADD || op > OP_MOD || op == OP_NOT || op == OP_NEG || op == OP_ABS) return false;
  }
  return true;
}

struct ArrayVars {
  const double* v;
  MXS_HD double get(int i) const { return v[i]; }
};

MXS_HD double expr_eval(const ExprProg& p, const double* vars) {
  LocalStack st;
  ArrayVars va{vars};
  return expr_eval_t(p, st, va);
}

// ---------------------------------------------------------------------------------------------
// Division-free pane arithmetic. CDNA has no integer divider: a 64-bit `/` or `%` is a software
// routine of ~100 instructions. Pane ids are floor(t_rel / pane) with t_rel >= 0 relative to the
// step's base; the quotient comes from one f64 multiply by the host-computed reciprocal and is
// corrected by at most one (exact for t_rel < 2^52).
// ---------------------------------------------------------------------------------------------
MXS_HD int64_t fast_floor_div_pos(int64_t t_rel, int64_t d, double inv_d) {
  int64_t q = (int64_t)((double)t_rel * inv_d);
  const int64_t r = t_rel - q * d;
  if (r < 0) --q;
  else if (r >= d) ++q;
  return q;
}

// ---------------------------------------------------------------------------------------------
// Partition plan (keyBy + window assignment + late check) shared by CPU and GPU.
// ---------------------------------------------------------------------------------------------
struct PartPlan {
  int32_t max_parallelism;   // Flink maxParallelism (128 by default)
  int32_t nsub_log2;         // sub-tables per rank = 1 << nsub_log2
  int32_t nranks;            // G (destination ranks)
  int32_t window_mode;       // 0 = keyed (no window, t = 0), 1 = windowed (t = pane - pane_base)
  int32_t drop_late;         // 1: elements with ts < late_ts are dropped (and optionally side-output)
  int32_t hash_mode;         // 0: Long.hashCode(key); 1: jhash table lookup (string dict ids)
  uint32_t bucket_cap;       // fixed capacity of one (dest, sub) bucket in the send buffer
  uint32_t ablate;           // profiling-only ablation bits (0 in production): 1 = skip scatter stores
  // ts < late_ts  <=>  every window of the element is past cleanup (maxTs + lateness <= wm):
  // late_ts is the smallest window start whose cleanup time is still ahead of the watermark.
  int64_t late_ts;
  int64_t tbase;             // pane_start(pane_base): records carry floor((ts - tbase) / pane)
  int64_t pane;              // pane length (ms)
  double inv_pane;           // 1.0 / pane
  int32_t rec_words;         // 3: 24-byte Rec; 2: 16-byte RecC (int32 values, GPU window path)
  int32_t dense_bits;        // > 0: dense key ids < 2^dense_bits, directly addressed (dense_slot)
  uint32_t dense_mul;        // odd multiplier of the dense slot bijection
  int32_t key32;             // 1: the key column is int32 (dictionary ids), sign-extended on load
  // GPU, 8-byte records, one destination, more than 512 buckets: a two-level partition -- the
  // LDS-staged compact kernel into nb / 2^L coarse buckets (this scratch, bucket_cap << L each),
  // then a split kernel per coarse bucket into its 2^L fine buckets. 0: the plain scatter.
  uint64_t* scratch;
  uint32_t* scratch_cursor;  // [512] coarse fills
};

// Sub-table of a key: a 32-bit multiplicative hash of both key halves (3 32-bit multiplies).
// Independent of the slot hash (low bits of mix64) and about half the VALU of a second mix64 —
// the partition pass evaluates it twice per event and is VALU-bound.
MXS_HD uint32_t sub_table_of(uint64_t key, int nsub_log2) {
  if (nsub_log2 == 0) return 0u;
  uint32_t h = (uint32_t)key * 0x9E3779B1u ^ (uint32_t)(key >> 32) * 0x85EBCA77u;
  h ^= h >> 15;
  h *= 0x2C1B3C6Du;
  h ^= h >> 13;
  return h >> (32 - nsub_log2);
}

// Home slot of a key inside its sub-table (low bits; linear probing from there): a second,
// independent 32-bit hash (murmur3-style mix of both halves). Every keyed table kernel, its C++
// twin and the invariant checker probe from this slot.
MXS_HD uint32_t slot_hash(uint64_t key) {
  uint32_t h = (uint32_t)key * 0xCC9E2D51u ^ (uint32_t)(key >> 32) * 0x1B873593u;
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  return h;
}

// Dense key ids (dictionary ids of string keys, or any id space [0, 2^bits)): the state is
// directly addressed, no hash-table probe. A bijection on [0, 2^bits) -- multiplication by an
// odd constant mod 2^bits -- spreads consecutive ids over the sub-tables (high bits) and gives
// each id its own slot; the host keeps the inverse to name the key of a slot.
MXS_HD uint32_t dense_slot(uint64_t key, uint32_t mul, int bits) {
  const uint32_t m = bits >= 32 ? 0xFFFFFFFFu : ((1u << bits) - 1u);
  return ((uint32_t)key * mul) & m;
}

// Sub-table of a key on a single-destination plan (hashed, or dense high bits).
MXS_HD uint32_t sub_of(uint64_t key, const PartPlan& p) {
  if (p.dense_bits > 0)
    return p.nsub_log2 ? dense_slot(key, p.dense_mul, p.dense_bits) >> (p.dense_bits - p.nsub_log2)
                       : 0u;
  return sub_table_of(key, p.nsub_log2);
}

MXS_HD uint32_t bucket_of(uint64_t key, int32_t jhash, const PartPlan& p, const int32_t* kg_dest) {
  const uint32_t sub = sub_of(key, p);
  if (p.nranks == 1) return sub;  // one rank owns every key group: no Java hash / murmur needed
  const int32_t kg = key_group_of_hash(jhash, p.max_parallelism);
  const int32_t dest = kg_dest[kg];
  return ((uint32_t)dest << p.nsub_log2) | sub;
}

// Relative pane of a (non-late) element; returns false when it cannot be represented
// (ts before the step base, or more than 2^32 panes ahead) — reported as an overflow.
MXS_HD bool rel_pane(int64_t ts, const PartPlan& p, uint32_t* t_out, int64_t* pane_abs_rel) {
  const int64_t d = ts - p.tbase;
  if (d < 0 || d >= (int64_t)1 << 52) return false;
  if (d < ((int64_t)1 << 31) && p.pane < ((int64_t)1 << 31)) {
    // 32-bit fast path (the common case: a step spans < 24 days of event time): u32 -> f64
    // conversion, one f64 multiply, f64 -> u32, one 32-bit multiply for the +-1 correction —
    // instead of the 64-bit integer <-> f64 conversion sequences (the partition is VALU-bound).
    const uint32_t du = (uint32_t)d, pu = (uint32_t)p.pane;
    uint32_t q = (uint32_t)((double)du * p.inv_pane);
    const uint32_t qp = q * pu;  // <= du + pu < 2^32
    if (qp > du) --q;
    else if (du - qp >= pu) ++q;
    *t_out = q;
    *pane_abs_rel = q;
    return true;
  }
  const int64_t q = fast_floor_div_pos(d, p.pane, p.inv_pane);
  if (q >= ((int64_t)1 << 32)) return false;
  *t_out = (uint32_t)q;
  *pane_abs_rel = q;
  return true;
}

// Stats block written by the partition pass (all int64):
//   [0] max ts (all events, used for the watermark)    [1] min pane of non-late events
//   [2] max pane of non-late events                     [3] late (dropped) events
//   [4] overflow flags: bit0 bucket capacity exceeded,  [5] events accepted
//       bit1 an element's pane is not representable
// Panes in [1]/[2] are relative to the step's pane base.
constexpr int kStatMaxTs = 0, kStatMinPane = 1, kStatMaxPane = 2, kStatLate = 3, kStatOverflow = 4,
              kStatAccepted = 5, kStatMaxBucket = 6, kStatPaneMask = 7, kStatCount = 8;
// kStatPaneMask (GPU partitions): bit j = some accepted record has relative pane j (j < 31);
// bit 31 = a record has relative pane >= 31 (the mask is then not used). 0 = not computed.


// ------------------------------------------------------------------------------------------
// Text field parsing shared by the C++ runtime (csrc/runtime.cpp, throws Java exceptions) and the
// GPU parse kernel (csrc/parse_hip.hip, flags the line): one source of truth for semantics.
// ------------------------------------------------------------------------------------------
// Long.parseLong / Integer.parseInt grammar: [+-]digits. Returns 0 ok, 1 format error, 2 overflow.
MXS_HD int parse_long_ascii(const char* s, int64_t len, int64_t lo, int64_t hi, int64_t* out) {
  if (len <= 0) return 1;
  int64_t i = 0;
  bool neg = false;
  if (s[0] == '+' || s[0] == '-') {
    neg = s[0] == '-';
    i = 1;
    if (len == 1) return 1;
  }
  // Java's Long.parseLong: accumulate negatively (covers INT64_MIN), check before each step.
  int64_t v = 0;
  const int64_t limit = neg ? lo : -hi;
  const int64_t multmin = limit / 10;
  for (; i < len; ++i) {
    const char c = s[i];
    if (c < '0' || c > '9') return 1;
    const int d = c - '0';
    if (v < multmin) return 2;
    v *= 10;
    if (v < limit + d) return 2;
    v -= d;
  }
  *out = neg ? v : -v;
  return 0;
}

MXS_HD int64_t days_from_civil_hd(int64_t y, unsigned m, unsigned d) {
  y -= m <= 2;
  const int64_t era = (y >= 0 ? y : y - 399) / 400;
  const unsigned yoe = (unsigned)(y - era * 400);
  const unsigned doy = (153 * (m + (m > 2 ? -3 : 9)) + 2) / 5 + d - 1;
  const unsigned doe = yoe * 365 + yoe / 4 - yoe / 100 + doy;
  return era * 146097 + (int64_t)doe - 719468;
}

// LocalDateTime.parse (ISO_LOCAL_DATE_TIME: yyyy-MM-ddTHH:mm[:ss[.f{1,9}]]) at a fixed offset.
// Returns false on a DateTimeParseException.
MXS_HD bool iso_local_datetime(const char* s, int64_t len, int64_t offset_s, int64_t* epoch_s,
                               int64_t* millis) {
  if (len < 16) return false;
  int v[5] = {0, 0, 0, 0, 0};
  const int pos[5] = {0, 5, 8, 11, 14}, w[5] = {4, 2, 2, 2, 2};
  for (int f = 0; f < 5; ++f)
    for (int k = 0; k < w[f]; ++k) {
      const char c = s[pos[f] + k];
      if (c < '0' || c > '9') return false;
      v[f] = v[f] * 10 + (c - '0');
    }
  if (s[4] != '-' || s[7] != '-' || s[10] != 'T' || s[13] != ':') return false;
  int sec = 0, ms = 0;
  int64_t p = 16;
  if (p < len) {
    if (s[p] != ':' || p + 3 > len) return false;
    for (int k = 1; k <= 2; ++k) {
      const char c = s[p + k];
      if (c < '0' || c > '9') return false;
      sec = sec * 10 + (c - '0');
    }
    p += 3;
    if (p < len) {
      if (s[p] != '.') return false;
      ++p;
      int nd = 0, frac = 0;
      for (; p < len; ++p) {
        const char c = s[p];
        if (c < '0' || c > '9') return false;
        if (nd < 3) frac = frac * 10 + (c - '0');
        ++nd;
      }
      if (nd == 0 || nd > 9) return false;
      for (int k = nd; k < 3; ++k) frac *= 10;
      ms = frac;
    }
  }
  const int y = v[0], mo = v[1], d = v[2], h = v[3], mi = v[4];
  if (mo < 1 || mo > 12 || d < 1) return false;
  const bool leap = (y % 4 == 0 && y % 100 != 0) || y % 400 == 0;
  const int mdays = mo == 2 ? (leap ? 29 : 28) : (mo == 4 || mo == 6 || mo == 9 || mo == 11) ? 30 : 31;
  if (d > mdays || h > 23 || mi > 59 || sec > 59) return false;
  *epoch_s = days_from_civil_hd(y, (unsigned)mo, (unsigned)d) * 86400 + h * 3600 + mi * 60 + sec -
             offset_s;
  *millis = ms;
  return true;
}

// java.lang.String.hashCode() of UTF-8 text, over its UTF-16 code units (invalid bytes decode
// to U+FFFD, supplementary code points to surrogate pairs): keyBy on a String field hashes the
// Java string (ComputeCpuMax.java:26 keyBy(0) -> Tuple1<String>.hashCode()). Shared by the host
// StringDict (csrc/runtime.cpp) and the GPU dictionary (csrc/ingest_hip.hip).
MXS_HD int32_t java_hash_utf8(const char* s, int64_t n) {
  uint32_t h = 0;
  int64_t i = 0;
  while (i < n) {
    const uint32_t c = (unsigned char)s[i];
    uint32_t cp = 0xFFFDu;
    int64_t len = 1;
    if (c < 0x80u) {
      cp = c;
    } else if ((c >> 5) == 0x6u && i + 1 < n && ((unsigned char)s[i + 1] >> 6) == 2u) {
      cp = ((c & 0x1Fu) << 6) | ((unsigned char)s[i + 1] & 0x3Fu);
      len = 2;
    } else if ((c >> 4) == 0xEu && i + 2 < n && ((unsigned char)s[i + 1] >> 6) == 2u &&
               ((unsigned char)s[i + 2] >> 6) == 2u) {
      cp = ((c & 0x0Fu) << 12) | (((unsigned char)s[i + 1] & 0x3Fu) << 6) |
           ((unsigned char)s[i + 2] & 0x3Fu);
      len = 3;
    } else if ((c >> 3) == 0x1Eu && i + 3 < n && ((unsigned char)s[i + 1] >> 6) == 2u &&
               ((unsigned char)s[i + 2] >> 6) == 2u && ((unsigned char)s[i + 3] >> 6) == 2u) {
      cp = ((c & 0x07u) << 18) | (((unsigned char)s[i + 1] & 0x3Fu) << 12) |
           (((unsigned char)s[i + 2] & 0x3Fu) << 6) | ((unsigned char)s[i + 3] & 0x3Fu);
      len = 4;
    }
    if (cp >= 0x10000u) {
      cp -= 0x10000u;
      h = 31u * h + (0xD800u + (cp >> 10));
      h = 31u * h + (0xDC00u + (cp & 0x3FFu));
    } else {
      h = 31u * h + cp;
    }
    i += len;
  }
  return (int32_t)h;
}

// Order-preserving map of an f64 bit pattern to u64 (ascending = Java Double.compareTo order:
// -0.0 < 0.0, every NaN canonical and largest) and its inverse.
MXS_HD uint64_t f64_order_bits(uint64_t b) {
  if ((b & 0x7FF0000000000000ull) == 0x7FF0000000000000ull && (b & 0x000FFFFFFFFFFFFFull))
    b = 0x7FF8000000000000ull;  // NaN
  return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}
MXS_HD uint64_t f64_from_order_bits(uint64_t o) {
  return (o >> 63) ? (o & 0x7FFFFFFFFFFFFFFFull) : ~o;
}

}  // namespace mxs
