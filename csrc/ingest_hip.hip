// mxstream — GPU text ingest with a device string dictionary (gfx950). See csrc/ingest.h for the
// pipeline; this file holds the kernels and their launchers.
//
// Layout choices:
//  * one thread per line (lines are 30-60 bytes; a wave parses 64 lines, the batch is streamed
//    from HBM once, the bytes of a line stay in the thread's L1/L2 lines);
//  * the dictionary table is open addressing on the 64-bit content hash: a lookup of a known
//    string is one relaxed 8-byte load of an L2-resident slot (the monitored key spaces --
//    hosts, channels -- are thousands to millions of strings);
//  * new strings are found without any per-string atomics on the hot path: the first position of
//    a claimed slot is an atomic min that is skipped once a smaller position is visible, and ids
//    are handed out by an order-preserving compaction of the first occurrences, so they equal
//    the host StringDict's ids (first appearance order) whatever the wave schedule was.
#include <hip/hip_runtime.h>

#include <stdexcept>
#include <string>

#include "ingest.h"
#include "line_tile.h"
#include "mxs_kernels.h"

namespace mxs {
namespace {

#define ING_CHECK(x)                                                                   \
  do {                                                                                 \
    const hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess)                                                              \
      throw std::runtime_error(std::string("ingest: ") + hipGetErrorString(e_));      \
  } while (0)

inline int ing_grid(int64_t n, int threads, int cap) {
  int64_t g = (n + threads - 1) / threads;
  if (g < 1) g = 1;
  return (int)(g > cap ? cap : g);
}

__device__ __forceinline__ int64_t wave_max_i64(int64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const int64_t w = __shfl_xor(v, o, 64);
    v = w > v ? w : v;
  }
  return v;
}

// The device twin of ingest.h ingest_line with one copy of each field parser: the output
// columns are visited in a loop that is not unrolled, each finding its split field from a
// cursor over the line (one forward scan when the columns ask for ascending split indices,
// a rescan from the line start otherwise). ingest_line's unrolled per-column copies of every
// parser made a 34K-instruction kernel whose instruction fetch, not its work, set its time.
// Same results as ingest_line (Java String.split semantics: trailing empty fields dropped, ""
// splits to [""]).
template <class Text>
__device__ uint8_t ingest_line_dev(Text text, int64_t a, int64_t b, int64_t li, int64_t n,
                                   const IngestSpec& sp, const IngestOut& o, int64_t* ts_val) {
  const char sep = (char)sp.sep;
  uint8_t st = 0;
  int idx = 0;       // split index of the field starting at `cur`
  int64_t cur = a;
#pragma unroll 1
  for (int f = 0; f < sp.nfields; ++f) {
    const int want = sp.field[f];
    if (want < idx) {
      idx = 0;
      cur = a;
    }
    bool exists = true;
    while (idx < want) {  // skip to the start of field `want`
      int64_t p = cur;
      while (p < b && text[p] != sep) ++p;
      if (p >= b) {
        exists = false;
        break;
      }
      cur = p + 1;
      ++idx;
    }
    int64_t fe = cur;
    bool present = false;
    if (exists) {
      while (fe < b && text[fe] != sep) ++fe;
      if (fe > cur) {
        present = true;
      } else if (a == b) {
        present = want == 0;
      } else {  // an empty field counts only when a later field is not empty
        for (int64_t p = fe; p < b; ++p)
          if (text[p] != sep) {
            present = true;
            break;
          }
      }
    }
    const int32_t kind = sp.kind[f];
    if (kind == IK_STR) {
      const int64_t p = li * sp.nstr + sp.sidx[f];
      if (!present) {
        o.slen[p] = -1;
        st = 1;  // ArrayIndexOutOfBounds: the host reports it
        continue;
      }
      const char* q = text_at(text, cur);
      const int64_t len = fe - cur;
      o.spos[p] = cur;
      o.slen[p] = (int32_t)len;
      o.sjh[p] = java_hash_utf8(q, len);
      o.shash[p] = text_hash64(q, len);
      continue;
    }
    if (!present) {
      st = 1;
      continue;
    }
    const char* q = text_at(text, cur);
    const int64_t len = fe - cur;
    int64_t v = 0;
    bool ok = true;
    switch (kind) {
      case IK_DOUBLE: {
        double d;
        ok = fast_parse_double(q, len, &d);
        v = (int64_t)f64_bits(d);
        break;
      }
      case IK_LONG:
      case IK_RAW_LONG:
        ok = parse_long_ascii(q, len, INT64_MIN, INT64_MAX, &v) == 0;
        break;
      case IK_INT:
        ok = parse_long_ascii(q, len, INT32_MIN, INT32_MAX, &v) == 0;
        break;
      case IK_TS_INTSEC:
      case IK_TS_MS:
      case IK_ISO_SEC: {
        int64_t es = 0, ms = 0;
        ok = iso_local_datetime(q, len, sp.offset_s, &es, &ms);
        v = kind == IK_TS_MS ? es * 1000 + ms
            : kind == IK_ISO_SEC ? (int64_t)(int32_t)(uint32_t)(uint64_t)es
                                 : (int64_t)(int32_t)(uint32_t)(uint64_t)es * 1000;  // (int) quirk
        break;
      }
      default: ok = false;
    }
    if (!ok) {
      st = 1;
      continue;
    }
    o.cols[(int64_t)f * n + li] = v;
    if (f == sp.ts_col) *ts_val = v;
  }
  return st;
}

// One workgroup per tile of 256 lines: the tile's bytes are staged into LDS (line_tile.h), every
// thread splits and parses its line there, then probes the dictionary for its string fields.
template <class Text>
__device__ __forceinline__ void ingest_one_line(Text text, const char* __restrict__ gtext,
                                                int64_t text_len,
                                                const int64_t* __restrict__ starts, int64_t n,
                                                int64_t li, const IngestSpec& sp,
                                                const IngestOut& o, const DictState& d,
                                                int64_t* local_max, uint32_t* local_flag) {
  const int64_t a = starts[li];
  int64_t b = li + 1 < n ? starts[li + 1] - 1 : text_len;  // exclusive end (drop '\n')
  if (b > text_len) b = text_len;
  if (b > a && text[b - 1] == '\n') --b;  // the last line of a batch ending in '\n'
  if (b > a && text[b - 1] == '\r') --b;  // SocketTextStreamFunction strips a trailing '\r'
  int64_t ts = INT64_MIN;
  const uint8_t st = ingest_line_dev(text, a, b, li, n, sp, o, &ts);
  o.status[li] = st;
  *local_flag += st;
  if (!st && ts > *local_max) *local_max = ts;
  (void)gtext;
  // Dictionary probe of every string field of the line.
  for (int s = 0; s < sp.nstr; ++s) {
    const int64_t p = li * sp.nstr + s;
    int32_t slot = -1;
    if (o.slen[p] >= 0) {
      const uint64_t h = o.shash[p];
      uint32_t q = dict_home(h, d.mask);
      for (uint32_t i = 0; i <= d.mask; ++i) {
        // A plain (L1-cacheable) load: slots only go 0 -> hash, so a stale 0 just sends this
        // thread to the CAS below, which returns the slot's hash; an agent-scope load went to
        // L2 for every string of every line.
        const uint64_t k = d.tab_h[q];
        if (k == h) {
          slot = (int32_t)q;
          break;
        }
        if (k == 0) {
          const uint64_t prev = atomicCAS((unsigned long long*)&d.tab_h[q], 0ull,
                                          (unsigned long long)h);
          if (prev == 0 || prev == h) {
            slot = (int32_t)q;
            break;
          }
        }
        q = (q + 1) & d.mask;
      }
      if (slot < 0) {
        atomicOr((unsigned long long*)&d.ctr[2], (unsigned long long)kDictErrFull);
      } else if (d.tab_id[slot] < 0 && d.tab_first[slot] > p) {
        atomicMin((unsigned long long*)&d.tab_first[slot], (unsigned long long)p);
      }
    }
    o.sslot[p] = slot;
  }
}

// 16 KB tiles (256 lines of up to ~60 bytes): eight 256-thread workgroups per CU, the 32-wave
// limit, where the 24 KB tile of line_tile.h allows six. Longer lines go to the global kernel.
constexpr int kIngestTileBytes = 16 * 1024;

// GLOBAL = false: tiles whose bytes fit the LDS tile, parsed there (the other tiles' workgroups
// return at once); GLOBAL = true: the launch after it parses only the tiles that did not fit,
// from global memory. Two kernels instead of both paths in one keep each one's code small.
template <bool GLOBAL>
__global__ __launch_bounds__(256) void ingest_parse_kernel(
    const char* __restrict__ text, int64_t text_len, const int64_t* __restrict__ starts,
    int64_t n, IngestSpec sp, IngestOut o, DictState d) {
  __shared__ __attribute__((aligned(16))) char tile[GLOBAL ? 16 : kIngestTileBytes];
  int64_t local_max = INT64_MIN;
  uint32_t local_flag = 0;
  const int64_t l0 = (int64_t)blockIdx.x * kTileLines;
  const int64_t l1 = l0 + kTileLines < n ? l0 + kTileLines : n;
  const int64_t lo = starts[l0];
  int64_t hi = l1 < n ? starts[l1] : text_len;
  if (hi > text_len) hi = text_len;
  if (tile_fits_lds(text, lo, hi, kIngestTileBytes) == GLOBAL) return;  // workgroup-uniform
  const int64_t li = l0 + threadIdx.x;
  if constexpr (GLOBAL) {
    if (li < l1) ingest_one_line(text, text, text_len, starts, n, li, sp, o, d, &local_max, &local_flag);
  } else {
    const LdsText lt = stage_line_tile(text, lo, hi, tile, kIngestTileBytes);
    if (li < l1) ingest_one_line(lt, text, text_len, starts, n, li, sp, o, d, &local_max, &local_flag);
  }
  // The workgroup's flag count and max timestamp: the max goes to its tile slot (reduced by
  // tile_max_reduce_kernel), the flag count -- rare -- straight to the counter.
  __shared__ int64_t s_max[kTileLines / 64];
  __shared__ uint32_t s_fl[kTileLines / 64];
  local_max = wave_max_i64(local_max);
  uint32_t fl = local_flag;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) fl += __shfl_xor(fl, off, 64);
  if ((threadIdx.x & 63) == 0) {
    s_max[threadIdx.x >> 6] = local_max;
    s_fl[threadIdx.x >> 6] = fl;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int64_t m = INT64_MIN;
    uint32_t f = 0;
    for (int w = 0; w < kTileLines / 64; ++w) {
      m = s_max[w] > m ? s_max[w] : m;
      f += s_fl[w];
    }
    if (f) atomicAdd(o.nflag, f);
    if (o.tile_max)
      o.tile_max[blockIdx.x] = m;
    else if (m != INT64_MIN)
      atomicMax((long long*)o.maxts, (long long)m);
  }
}

// Max of the per-tile maxima into the batch maximum (one workgroup, one atomic).
__global__ __launch_bounds__(1024) void tile_max_reduce_kernel(const int64_t* __restrict__ tile_max,
                                                               int64_t tiles, int64_t* maxts) {
  __shared__ int64_t s_w[16];
  int64_t m = INT64_MIN;
  for (int64_t t = threadIdx.x; t < tiles; t += blockDim.x) m = tile_max[t] > m ? tile_max[t] : m;
  m = wave_max_i64(m);
  if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 0; w < 16; ++w) m = s_w[w] > m ? s_w[w] : m;
    if (m != INT64_MIN) atomicMax((long long*)maxts, (long long)m);
  }
}

// New-string mask: position p holds the first occurrence of a string whose slot has no id yet.
// Tile layout of filter_mask_kernel (kFcItems x 256 positions per workgroup, one ballot word per
// wave and item), so filter_scan / filter_write finish the compaction.
__global__ __launch_bounds__(256) void dict_new_mask_kernel(const int32_t* __restrict__ sslot,
                                                            int64_t np, DictState d,
                                                            uint64_t* __restrict__ masks,
                                                            uint32_t* __restrict__ counts) {
  __shared__ uint32_t wcnt[kFcWords];
  const int64_t tile = (int64_t)blockIdx.x * kFcTile;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
  for (int j = 0; j < kFcItems; ++j) {
    const int64_t p = tile + j * 256 + threadIdx.x;
    bool is_new = false;
    if (p < np) {
      const int32_t s = sslot[p];
      is_new = s >= 0 && d.tab_id[s] < 0 && d.tab_first[s] == p;
    }
    const uint64_t m = __ballot(is_new);
    if (lane == 0) {
      masks[(size_t)blockIdx.x * kFcWords + j * 4 + wave] = m;
      wcnt[j * 4 + wave] = (uint32_t)__popcll(m);
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t c = 0;
    for (int w = 0; w < kFcWords; ++w) c += wcnt[w];
    counts[blockIdx.x] = c;
  }
}

// The k-th new string (first-occurrence order) gets id n_ids + k; its bytes go to the arena.
__global__ __launch_bounds__(256) void dict_assign_kernel(const char* __restrict__ text,
                                                          const int64_t* __restrict__ newpos,
                                                          int64_t bound, IngestOut o, DictState d) {
  const int64_t n_new = d.ctr[3], n_ids = d.ctr[0];
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n_new && k < bound;
       k += stride) {
    const int64_t p = newpos[k];
    const int32_t s = o.sslot[p];
    const int64_t id = n_ids + k;
    const int32_t len = o.slen[p];
    if (id >= d.id_cap) {
      atomicOr((unsigned long long*)&d.ctr[2], (unsigned long long)kDictErrCapacity);
      continue;
    }
    const int64_t off = (int64_t)atomicAdd((unsigned long long*)&d.ctr[1], (unsigned long long)len);
    if (off + len > d.arena_cap) {
      atomicOr((unsigned long long*)&d.ctr[2], (unsigned long long)kDictErrCapacity);
      continue;
    }
    const char* src = text + o.spos[p];
    for (int32_t c = 0; c < len; ++c) d.arena[off + c] = (uint8_t)src[c];
    d.id_off[id] = off;
    d.id_len[id] = len;
    d.id_jh[id] = o.sjh[p];
    d.tab_first[s] = INT64_MAX;
    d.tab_id[s] = (int32_t)id;
  }
}

__global__ void dict_commit_kernel(DictState d) {
  if (threadIdx.x == 0 && blockIdx.x == 0) d.ctr[0] += d.ctr[3];
}

// Every string field gets its slot's id, after a byte comparison with the arena copy.
__global__ __launch_bounds__(256) void dict_resolve_kernel(const char* __restrict__ text,
                                                           int64_t n, int32_t nstr, IngestOut o,
                                                           DictState d) {
  const int64_t np = n * nstr;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < np; p += stride) {
    const int32_t s = o.sslot[p];
    int32_t id = -1;
    if (s >= 0) {
      id = d.tab_id[s];
      bool same = id >= 0 && d.id_len[id] == o.slen[p];
      if (same) {
        const char* a = text + o.spos[p];
        const uint8_t* b = d.arena + d.id_off[id];
        for (int32_t c = 0; c < o.slen[p] && same; ++c) same = (uint8_t)a[c] == b[c];
      }
      if (!same) {
        atomicOr((unsigned long long*)&d.ctr[2], (unsigned long long)kDictErrCollision);
        id = -1;
      }
    }
    const int64_t li = p / nstr, si = p - li * nstr;
    o.ids[si * n + li] = id;
  }
}

// Agreed ids (several ranks, csrc/ingest.h): string i of a packed list gets id id0 + i -- in the
// slot this batch's parse claimed for it, or in a fresh slot (a string new on another rank).
__global__ __launch_bounds__(256) void dict_insert_ids_kernel(const uint8_t* __restrict__ buf,
                                                              const int64_t* __restrict__ offs,
                                                              const int32_t* __restrict__ lens,
                                                              int64_t k, int64_t id0, DictState d) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  if (blockIdx.x == 0 && threadIdx.x == 0) d.ctr[0] = id0 + k;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < k; i += stride) {
    const char* str = (const char*)buf + offs[i];
    const int32_t len = lens[i];
    const uint64_t h = text_hash64(str, len);
    uint32_t q = dict_home(h, d.mask);
    int32_t slot = -1;
    for (uint32_t t = 0; t <= d.mask; ++t) {
      const uint64_t prev = atomicCAS((unsigned long long*)&d.tab_h[q], 0ull, (unsigned long long)h);
      if (prev == 0 || prev == h) {
        slot = (int32_t)q;
        break;
      }
      q = (q + 1) & d.mask;
    }
    const int64_t id = id0 + i;
    if (slot < 0 || id >= d.id_cap) {
      atomicOr((unsigned long long*)&d.ctr[2], (unsigned long long)(slot < 0 ? kDictErrFull
                                                                             : kDictErrCapacity));
      continue;
    }
    const int64_t off = (int64_t)atomicAdd((unsigned long long*)&d.ctr[1], (unsigned long long)len);
    if (off + len > d.arena_cap) {
      atomicOr((unsigned long long*)&d.ctr[2], (unsigned long long)kDictErrCapacity);
      continue;
    }
    for (int32_t c = 0; c < len; ++c) d.arena[off + c] = (uint8_t)str[c];
    d.id_off[id] = off;
    d.id_len[id] = len;
    d.id_jh[id] = java_hash_utf8(str, len);
    d.tab_first[slot] = INT64_MAX;
    d.tab_id[slot] = (int32_t)id;
  }
}

// Grow: re-insert the assigned entries of the old table into an empty one.
__global__ __launch_bounds__(256) void dict_rehash_kernel(const uint64_t* __restrict__ old_h,
                                                          const int32_t* __restrict__ old_id,
                                                          int64_t old_cap, DictState d) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < old_cap; i += stride) {
    const uint64_t h = old_h[i];
    const int32_t id = old_id[i];
    if (h == 0 || id < 0) continue;
    uint32_t q = dict_home(h, d.mask);
    for (uint32_t k = 0; k <= d.mask; ++k) {
      const uint64_t prev = atomicCAS((unsigned long long*)&d.tab_h[q], 0ull,
                                      (unsigned long long)h);
      if (prev == 0) {
        d.tab_id[q] = id;
        break;
      }
      q = (q + 1) & d.mask;
    }
  }
}

// Expression-VM operand stack as a per-lane LDS column (no runtime-indexed private array).
struct IngLds {
  double* base;
  int stride;
  __device__ __forceinline__ double get(int i) const { return base[i * stride]; }
  __device__ __forceinline__ void set(int i, double x) { base[i * stride] = x; }
};

// Traced filter over the parsed columns (var j = column j as double): the tile ballots of
// filter_mask_kernel. String columns read as their dictionary id.
struct ColVars {
  const int64_t* cols;
  int64_t n;
  int64_t row;
  int32_t nf;
  int32_t dbl_mask;  // bit f: column f holds f64 bit patterns
  __device__ double get(int j) const {
    if (j >= nf) return 0.0;
    const int64_t v = cols[(int64_t)j * n + row];
    return ((dbl_mask >> j) & 1) ? as_f64((uint64_t)v) : (double)v;
  }
};

__global__ __launch_bounds__(256) void ingest_filter_mask_kernel(const int64_t* __restrict__ cols,
                                                                 int64_t n, int32_t nf,
                                                                 int32_t dbl_mask, ExprProg prog,
                                                                 uint64_t* __restrict__ masks,
                                                                 uint32_t* __restrict__ counts) {
  extern __shared__ __attribute__((aligned(16))) double fsm[];
  IngLds stack{fsm + threadIdx.x, 256};
  __shared__ uint32_t wcnt[kFcWords];
  const int64_t tile = (int64_t)blockIdx.x * kFcTile;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
  for (int j = 0; j < kFcItems; ++j) {
    const int64_t i = tile + j * 256 + threadIdx.x;
    bool keep = false;
    if (i < n) {
      ColVars vars{cols, n, i, nf, dbl_mask};
      keep = (prog.chain ? expr_eval_chain(prog, vars) : expr_eval_t(prog, stack, vars)) != 0.0;
    }
    const uint64_t m = __ballot(keep);
    if (lane == 0) {
      masks[(size_t)blockIdx.x * kFcWords + j * 4 + wave] = m;
      wcnt[j * 4 + wave] = (uint32_t)__popcll(m);
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t c = 0;
    for (int w = 0; w < kFcWords; ++w) c += wcnt[w];
    counts[blockIdx.x] = c;
  }
}

// Gather the kept rows of every column (int64 words) in input order.
__global__ __launch_bounds__(256) void ingest_gather_kernel(const int64_t* __restrict__ cols,
                                                            int64_t n, int32_t nf,
                                                            const int32_t* __restrict__ ids,
                                                            int32_t nstr,
                                                            const int64_t* __restrict__ idx,
                                                            const int64_t* __restrict__ total,
                                                            int64_t* __restrict__ out_cols,
                                                            int32_t* __restrict__ out_ids,
                                                            int64_t out_stride) {
  const int64_t m = *total;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < m && k < n; k += stride) {
    const int64_t r = idx[k];
    for (int f = 0; f < nf; ++f) out_cols[(int64_t)f * out_stride + k] = cols[(int64_t)f * n + r];
    for (int s = 0; s < nstr; ++s) out_ids[(int64_t)s * out_stride + k] = ids[(int64_t)s * n + r];
  }
}

}  // namespace

namespace gpu {

void ingest_parse(const char* text, int64_t text_len, const int64_t* starts, int64_t n,
                  const IngestSpec& sp, const IngestOut& o, const DictState& d, intptr_t stream) {
  if (n <= 0) return;
  if (sp.nfields < 1 || sp.nfields > kIngestMaxFields) throw std::invalid_argument("ingest: fields");
  const int64_t tiles = (n + kTileLines - 1) / kTileLines;
  if (tiles > INT32_MAX) throw std::invalid_argument("ingest: batch too large");
  hipLaunchKernelGGL(ingest_parse_kernel<false>, dim3((uint32_t)tiles), dim3(kTileLines), 0,
                     (hipStream_t)stream, text, text_len, starts, n, sp, o, d);
  ING_CHECK(hipGetLastError());
  hipLaunchKernelGGL(ingest_parse_kernel<true>, dim3((uint32_t)tiles), dim3(kTileLines), 0,
                     (hipStream_t)stream, text, text_len, starts, n, sp, o, d);
  ING_CHECK(hipGetLastError());
  if (o.tile_max) {
    hipLaunchKernelGGL(tile_max_reduce_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream,
                       o.tile_max, tiles, o.maxts);
    ING_CHECK(hipGetLastError());
  }
}

void dict_find_new(int64_t n, int32_t nstr, const IngestOut& o, const DictState& d,
                   void* scratch, int64_t* newpos, intptr_t stream) {
  const int64_t np = n * nstr;
  if (np <= 0) {
    ING_CHECK(hipMemsetAsync(&d.ctr[3], 0, 8, (hipStream_t)stream));
    return;
  }
  const int64_t nt = (np + kFcTile - 1) / kFcTile;
  uint64_t* masks = (uint64_t*)scratch;
  int64_t* offs = (int64_t*)(masks + nt * kFcWords);
  uint32_t* counts = (uint32_t*)(offs + nt);
  hipLaunchKernelGGL(dict_new_mask_kernel, dim3((uint32_t)nt), dim3(256), 0, (hipStream_t)stream,
                     o.sslot, np, d, masks, counts);
  ING_CHECK(hipGetLastError());
  compact_from_masks(masks, counts, nt, np, offs, newpos, &d.ctr[3], stream);
}

void dict_resolve(const char* text, int64_t n, int32_t nstr, const IngestOut& o,
                  const DictState& d, intptr_t stream) {
  const int64_t np = n * nstr;
  if (np <= 0) return;
  hipLaunchKernelGGL(dict_resolve_kernel, dim3(ing_grid(np, 256, 8192)), dim3(256), 0,
                     (hipStream_t)stream, text, n, nstr, o, d);
  ING_CHECK(hipGetLastError());
}

void dict_assign_new(const char* text, int64_t n, int32_t nstr, const IngestOut& o,
                     const DictState& d, void* scratch, int64_t* newpos, intptr_t stream) {
  const int64_t np = n * nstr;
  if (np <= 0) return;
  dict_find_new(n, nstr, o, d, scratch, newpos, stream);
  hipLaunchKernelGGL(dict_assign_kernel, dim3(ing_grid(np, 256, 2048)), dim3(256), 0,
                     (hipStream_t)stream, text, newpos, np, o, d);
  ING_CHECK(hipGetLastError());
  hipLaunchKernelGGL(dict_commit_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, d);
  ING_CHECK(hipGetLastError());
  dict_resolve(text, n, nstr, o, d, stream);
}

void dict_insert_ids(const uint8_t* buf, const int64_t* offs, const int32_t* lens, int64_t k,
                     int64_t id0, const DictState& d, intptr_t stream) {
  if (k <= 0) return;
  hipLaunchKernelGGL(dict_insert_ids_kernel, dim3(ing_grid(k, 256, 2048)), dim3(256), 0,
                     (hipStream_t)stream, buf, offs, lens, k, id0, d);
  ING_CHECK(hipGetLastError());
}

void dict_rehash(const uint64_t* old_h, const int32_t* old_id, int64_t old_cap, const DictState& d,
                 intptr_t stream) {
  if (old_cap <= 0) return;
  hipLaunchKernelGGL(dict_rehash_kernel, dim3(ing_grid(old_cap, 256, 8192)), dim3(256), 0,
                     (hipStream_t)stream, old_h, old_id, old_cap, d);
  ING_CHECK(hipGetLastError());
}

void ingest_filter_compact(const int64_t* cols, int64_t n, int32_t nf, int32_t dbl_mask,
                           const ExprProg& prog, void* scratch, int64_t* idx, int64_t* total,
                           intptr_t stream) {
  if (n <= 0) {
    ING_CHECK(hipMemsetAsync(total, 0, 8, (hipStream_t)stream));
    return;
  }
  const int64_t nt = (n + kFcTile - 1) / kFcTile;
  uint64_t* masks = (uint64_t*)scratch;
  int64_t* offs = (int64_t*)(masks + nt * kFcWords);
  uint32_t* counts = (uint32_t*)(offs + nt);
  const size_t lds = (size_t)(prog.depth > 0 ? prog.depth : 1) * 256 * sizeof(double);
  hipLaunchKernelGGL(ingest_filter_mask_kernel, dim3((uint32_t)nt), dim3(256), lds,
                     (hipStream_t)stream, cols, n, nf, dbl_mask, prog, masks, counts);
  ING_CHECK(hipGetLastError());
  compact_from_masks(masks, counts, nt, n, offs, idx, total, stream);
}

void ingest_gather(const int64_t* cols, int64_t n, int32_t nf, const int32_t* ids, int32_t nstr,
                   const int64_t* idx, const int64_t* total, int64_t* out_cols, int32_t* out_ids,
                   int64_t out_stride, intptr_t stream) {
  if (n <= 0) return;
  hipLaunchKernelGGL(ingest_gather_kernel, dim3(ing_grid(n, 256, 4096)), dim3(256), 0,
                     (hipStream_t)stream, cols, n, nf, ids, nstr, idx, total, out_cols, out_ids,
                     out_stride);
  ING_CHECK(hipGetLastError());
}

}  // namespace gpu
}  // namespace mxs
