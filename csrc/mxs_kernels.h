// mxstream — kernel launcher interface (GPU: kernels_hip.hip, CPU twins: kernels_cpu.cpp).
//
// All buffers are raw pointers owned by the caller (torch tensors on the Python side); `stream`
// is a hipStream_t passed as an integer. The CPU twins take the same arguments (stream ignored)
// and are bit-compatible with the GPU kernels for integer aggregates; float sums are exact on
// CPU (arrival order) and order-independent up to rounding on GPU.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include "mxs_common.h"
#include "row_format.h"

namespace mxs {

// Plan of the keyed-window aggregation pass (one workgroup per sub-table on the GPU).
struct AggPlan {
  int32_t cap_log2;     // slots per sub-table = 1 << cap_log2
  int32_t nsub;         // sub-tables on this rank
  int32_t ring;         // pane ring length R (power of two)
  int32_t agg;          // AggKind
  int32_t nsrc;         // number of source segments per sub-table (G after the all-to-all)
  uint32_t bucket_cap;  // capacity of one (src, sub) segment
  int32_t np_step;      // panes touched by this step: [pane_base + p_lo, + np_step)
  int32_t pg;           // panes staged in LDS per pass (GPU only)
  int64_t pane_base;    // records carry pane - pane_base
  int64_t p_lo;         // first pane (relative to pane_base) touched this step
  int64_t fired_hi;     // absolute pane id: panes <= fired_hi are in an already-fired window
  int32_t combined;     // records are pre-aggregated (aux = element count, val = exported acc)
  int32_t rec_words;    // 3: Rec (24 B); 2: RecC (16 B)
  // Touched-slot list of late-but-allowed data (optional, all three or none): the first time a
  // slot receives data for an already-fired pane it is marked and appended, so re-firings visit
  // only those slots instead of sweeping the table.
  uint32_t* dlist;      // [nslots] slot ids
  uint32_t* dlist_n;    // list length
  uint32_t* slot_mark;  // [nslots] 1 = listed
  int32_t dense_bits;   // > 0: directly addressed dense key ids (slot = dense_slot(key))
  uint32_t dense_mul;
  // Hot sub-tables (dense ids, one source, additive aggregates, no touched-slot list): up to
  // `split` workgroups share one sub-table's records (>= kAggSliceMin each) and merge into the
  // state with atomic adds; 1 = one workgroup per sub-table.
  int32_t split;
  // 1: deterministic f64 sums (AGG_SUM_F64 / AGG_AVG_F64): per-step slot sums in 128-bit fixed
  // point (mxs_common.h f64_to_fx), bit-identical between runs and between the GPU and the C++
  // twin. A value outside the fixed-point range sets flags[0] bit 3.
  int32_t det;
  // Local-global aggregation with allowed lateness: the contributions of late-but-allowed data
  // (panes <= fired_hi) are also accumulated into this delta ring (same layout as acc_g/cnt_g),
  // so a re-firing ships only the deltas to the window's owner. Needs the touched-slot list.
  uint64_t* dacc;
  uint32_t* dcnt;
  // Optional device word (the all-reduced combiner check of a records exchange): non-zero means
  // some rank's combined bucket overflowed, so this step's records are incomplete -- the
  // aggregation leaves the state untouched and the host redoes the step's exchange once it reads
  // the check (window_operator.py _verify_combine), instead of waiting for it before the
  // all-to-all.
  const int64_t* skip;
  // Sparse pane groups: non-zero (bit 31 clear) = the relative panes with records this step
  // (the partition's kStatPaneMask); np_step then counts the set bits and the LDS rows of a pass
  // map to those panes only -- the empty panes between a late pane and the current ones cost no
  // record pass. 0: the dense range [p_lo, p_lo + np_step).
  uint32_t pmask;
};

// Plan of one window firing.
struct FirePlan {
  int32_t agg;
  int32_t npanes;       // panes combined by the window
  int32_t ring;
  int32_t only_dirty;   // 1: re-fire only slots touched by late data
  int64_t nslots;       // nsub << cap_log2
  int64_t p0;           // first absolute pane of the window
  double wstart, wend;  // window bounds (ms) for the epilogue vars
  uint32_t out_cap;
  uint32_t ablate;      // profiling-only ablation bits (0 in production): 1 = skip the epilogue VM
  ExprProg map;         // value epilogue (empty = identity)
  ExprProg filt;        // predicate on the mapped value (empty = true)
  const uint32_t* list;    // optional: visit only these slots (touched-slot list) ...
  const uint32_t* list_n;  // ... of this length (device counter)
  // Compact rows (key id + mapped value: 12 bytes instead of 28) for sinks that read nothing
  // else: keys written as uint32 (dense ids) into the key column's first 4*n bytes; a null
  // out_raw / out_cnt column is not written.
  int32_t key32;
  // Fused re-firing only: clear each listed slot's dirty bytes and touched mark once its
  // windows are evaluated (dirty_clear's work, same thread; non-null = on).
  uint32_t* clear_mark;
};

// One window of a batched firing (window_fire_many): the per-window fields of FirePlan.
struct FireWin {
  int64_t p0;
  int32_t npanes;
  double wstart, wend;
};

// Staging of a batched firing on the GPU: window w of the batch writes its rows to
// [w * region, (w + 1) * region) of these columns at counter win_n[w] (region >= nslots).
struct FireStage {
  uint64_t* keys;
  double* vals;
  uint64_t* raw;
  uint32_t* cnt;
  uint32_t* win_n;
  uint32_t region;
};

// Local-global window aggregation (G > 1): where the rows of a locally fired window go.
struct ScatPlan {
  int32_t max_parallelism;  // Flink maxParallelism (key groups)
  int32_t nranks;           // G
  int32_t nsub_log2;        // owner sub-tables per rank = 1 << nsub_log2
  int32_t hash_mode;        // 0: Long.hashCode(key); 1: jhash table lookup (string dict ids)
  uint32_t bucket_cap;      // capacity of one (owner, sub-table) bucket
  uint32_t n_cap;           // rows readable in the input columns
};

// Rolling keyed state plan (ValueState / rolling reduce, no windows).
struct RollPlan {
  int32_t cap_log2;
  int32_t nsub;
  int32_t agg;
  int32_t nsrc;
  uint32_t bucket_cap;
  int32_t emit;         // 1: write the post-update value of every record (ordered operators)
};

// ---- GPU launchers (kernels_hip.hip) --------------------------------------------------------
// Keyed-window table maintenance (host-DRAM spill tier): rows of evicted (key, pane) state.
struct CompactOut {
  uint64_t* key;
  int64_t* pane;
  uint64_t* acc;
  uint32_t* cnt;
  uint8_t* dirty;
  uint32_t* n;        // rows written (device counter)
  uint32_t cap;       // row capacity (>= occupied slots x live panes)
  uint32_t* counters; // [0] keys dropped (no live data), [1] keys evicted, [2] overflow flag
};

constexpr int kD2HMax = 8;
struct D2HCopy {
  const void* src;
  int64_t bytes;    // bytes to copy (16-byte multiple); with a device row count: the maximum
  int64_t dst_off;
  int64_t esz = 0;  // > 0: bytes = min(bytes, round16(*n_dev * esz)) -- rows counted on the device
};
struct D2HBatch {
  D2HCopy c[kD2HMax];
  int n;
  const uint32_t* n_dev;  // device row count (fired rows), read by the copy kernel; may be null
};

constexpr int64_t kRollHistMaxSlots = 16384;  // LDS running-count table of the emit pass

// Order-preserving compaction tiles (filter_mask / line_starts / ingest masks): a 256-thread
// workgroup owns kFcTile rows, one 64-bit ballot word per wave and item.
constexpr int kFcItems = 16;  // 4096 rows per tile: few enough tiles for the one-workgroup scan
constexpr int kFcWords = kFcItems * 4;  // 64-bit words per 256-thread tile
constexpr int kFcTile = kFcItems * 256;

struct IngestSpec;
struct IngestOut;
struct DictState;

// Columns of a packed-row exchange (parallel/exchange.py): up to 8 columns whose rows are
// whole 32-bit words; src = the sender's columns, dst = the receiver's compacted outputs.
struct XRowCols {
  const uint32_t* src[8];
  uint32_t* dst[8];
  int words[8];
  int ncol;
  int rw;  // words of one packed row (sum of words[])
};

namespace gpu {
// Packed-row exchange (csrc/exchange_hip.hip): per-workgroup destination counts + their scan
// (blk_cnt: xrows_blocks(n) x world words, scanned in place; counts: world totals), the stable
// scatter into [world][cap] packed rows, and the receive-side compaction.
int64_t xrows_blocks(int64_t n);
void xrows_count(const int64_t* dest, int64_t n, int world, uint32_t* blk_cnt, uint32_t* counts,
                 uint32_t* bad, intptr_t stream);
void xrows_scatter(const int64_t* dest, int64_t n, int world, const uint32_t* blk_off,
                   uint32_t cap, const XRowCols& c, uint32_t* send, uint32_t* ovf,
                   intptr_t stream);
void xrows_unpack(const uint32_t* recv, const uint32_t* rc, int world, uint32_t cap,
                  const XRowCols& c, intptr_t stream);
// print() rows in Java text (csrc/row_format.h): lengths (+ a flag for rows the device cannot
// format), then, after an inclusive scan of the lengths into `end`, the bytes.
void format_rows_len(const FmtArgs& a, int64_t n, int64_t* len, uint32_t* bad, intptr_t stream);
void format_rows_write(const FmtArgs& a, int64_t n, const int64_t* end, char* out,
                       intptr_t stream);
// Host-to-device copy by the copy kernel reading a pinned (mapped) host buffer; 16-byte
// granules. Returns the hipError_t code (0 = ok).
int h2d_kernel(void* dst_dev, const void* src_host, int64_t bytes, intptr_t stream,
               int max_blocks = 1024);
int device_count();
int set_spin_schedule();
// Async device->host copy on `stream` (hipMemcpyAsync); returns the hipError_t code.
int d2h_async(void* dst, const void* src, size_t bytes, intptr_t stream);
// Async host -> device copy (hipMemcpyAsync); page-lock / release an existing host buffer
// (hipHostRegister keeps its ordinary cacheable mapping: host writes into it run at memcpy
// speed, unlike some pinned allocations). All return the hipError_t code.
int h2d_async(void* dst, const void* src, size_t bytes, intptr_t stream);
int host_register(void* p, size_t bytes);
int host_unregister(void* p);
// Up to kD2HMax device buffers -> one pinned (mapped) host slab by a copy kernel on `stream`;
// every size, source address and slab offset a multiple of 16 bytes. Returns hipError_t.
int d2h_kernel(void* dst_host, const D2HCopy* copies, int n, intptr_t stream,
               const uint32_t* n_dev = nullptr, int max_blocks = 1024);
// Experiment: pane accumulation by global atomics from the source columns (see kernels_hip).
void direct_agg_probe(const uint64_t* keys, const int64_t* ts, const uint64_t* vals, int64_t n,
                      int64_t tbase, int64_t pane, int ring, int64_t nslots, uint32_t mul,
                      int bits, int64_t pane_base, uint64_t* acc_g, uint32_t* cnt_g, int mode,
                      uint64_t* sink, int grid, intptr_t stream);
void gen_events(uint64_t* keys, int64_t* ts, uint64_t* vals, int64_t n, uint64_t seed,
                uint64_t stream_id, uint64_t idx0, uint64_t nkeys, int64_t ts_base,
                int64_t ts_span, int64_t disorder, int64_t val_lo, int64_t val_span,
                int32_t val_f64, double zipf_s, intptr_t stream, uint64_t key_base = 0);
void partition(const uint64_t* keys, const int64_t* ts, const uint64_t* vals,
               const int32_t* jhash_tab, int64_t n, const PartPlan& plan, const int32_t* kg_dest,
               uint32_t* cursor, Rec* out, int64_t* stats, uint32_t* late_idx, uint32_t late_cap,
               intptr_t stream);
void partition_variant(const uint64_t* keys, const int64_t* ts, const uint64_t* vals,
                       const int32_t* jhash_tab, int64_t n, const PartPlan& plan,
                       const int32_t* kg_dest, uint32_t* cursor, Rec* out, int64_t* stats,
                       uint32_t* late_idx, uint32_t late_cap, intptr_t stream, int variant);
void window_agg(const Rec* recs, const uint32_t* counts, const AggPlan& plan, uint64_t* keys_g,
                uint64_t* acc_g, uint32_t* cnt_g, uint8_t* dirty_g, uint32_t* occupancy,
                uint32_t* flags, intptr_t stream);
void window_fire(const uint64_t* keys_g, const uint64_t* acc_g, const uint32_t* cnt_g,
                 const uint8_t* dirty_g, const FirePlan& plan, uint64_t* out_keys,
                 double* out_vals, uint64_t* out_raw, uint32_t* out_cnt, uint32_t* out_n,
                 intptr_t stream);
// Several windows in one call: each window's rows follow the previous ones at the shared
// cursor out_n; bounds[i] = rows of windows 0..i (device).
// Fused re-firing of k windows over the touched-slot list (plan.list / list_n): one pass loads
// the union of the windows' panes (<= 16) per listed slot. Staging region per window =
// st.region (the caller splits the stage k ways); a window that outgrows it sets bit 16 of *ovf
// (re-run unfused). Returns false (nothing launched) when the union is too wide or k > 32.
bool window_refire_many(const uint64_t* keys_g, const uint64_t* acc_g, const uint32_t* cnt_g,
                        const uint8_t* dirty_g, const FirePlan& base, const FireWin* wins, int k,
                        const FireStage& st, uint64_t* out_keys, double* out_vals,
                        uint64_t* out_raw, uint32_t* out_cnt, uint32_t* out_n, uint32_t* bounds,
                        uint32_t* ovf, intptr_t stream, int64_t dlo = 0, uint32_t dmask_abs = 0);
void window_fire_many(const uint64_t* keys_g, const uint64_t* acc_g, const uint32_t* cnt_g,
                      const uint8_t* dirty_g, const FirePlan& base, const FireWin* wins, int k,
                      const FireStage& stage, uint64_t* out_keys, double* out_vals,
                      uint64_t* out_raw, uint32_t* out_cnt, uint32_t* out_n, uint32_t* bounds,
                      intptr_t stream);
void rolling(const Rec* recs, const uint32_t* counts, const RollPlan& plan, uint64_t* keys_g,
             uint64_t* acc_g, uint32_t* cnt_g, uint32_t* occupancy, uint32_t* flags,
             uint64_t* out_vals, intptr_t stream);
void expr_filter(const double* x, int64_t n, const ExprProg& prog, uint8_t* keep, intptr_t stream);
// Indices of the rows that pass (input order) and their number; scratch: filter_compact_scratch_bytes.
int64_t filter_compact_scratch_bytes(int64_t n);
// Line-start offsets of a text batch, in order (scratch: filter_compact_scratch_bytes(n)).
void line_starts(const uint8_t* buf, int64_t n, void* scratch, int64_t* idx, int64_t* total,
                 intptr_t stream, int64_t cap = INT64_MAX);
void expr_filter_compact(const double* x, int64_t n, const ExprProg& prog, void* scratch,
                         int64_t* idx, int64_t* total, intptr_t stream);
// Scan + write half of the compaction over tile masks/counts made by any mask kernel.
void compact_from_masks(const uint64_t* masks, const uint32_t* counts, int64_t nt, int64_t n,
                        int64_t* offs, int64_t* idx, int64_t* total, intptr_t stream);
// Device text ingest + string dictionary (csrc/ingest_hip.hip, csrc/ingest.h).
void ingest_parse(const char* text, int64_t text_len, const int64_t* starts, int64_t n,
                  const IngestSpec& sp, const IngestOut& o, const DictState& d, intptr_t stream);
void dict_assign_new(const char* text, int64_t n, int32_t nstr, const IngestOut& o,
                     const DictState& d, void* scratch, int64_t* newpos, intptr_t stream);
void dict_rehash(const uint64_t* old_h, const int32_t* old_id, int64_t old_cap, const DictState& d,
                 intptr_t stream);
// Several ranks agree on ids: find this batch's new strings (no ids yet) ...
void dict_find_new(int64_t n, int32_t nstr, const IngestOut& o, const DictState& d,
                   void* scratch, int64_t* newpos, intptr_t stream);
// ... insert the agreed list (string i -> id id0 + i) ...
void dict_insert_ids(const uint8_t* buf, const int64_t* offs, const int32_t* lens, int64_t k,
                     int64_t id0, const DictState& d, intptr_t stream);
// ... and resolve the batch's string fields to ids.
void dict_resolve(const char* text, int64_t n, int32_t nstr, const IngestOut& o,
                  const DictState& d, intptr_t stream);
void ingest_filter_compact(const int64_t* cols, int64_t n, int32_t nf, int32_t dbl_mask,
                           const ExprProg& prog, void* scratch, int64_t* idx, int64_t* total,
                           intptr_t stream);
void ingest_gather(const int64_t* cols, int64_t n, int32_t nf, const int32_t* ids, int32_t nstr,
                   const int64_t* idx, const int64_t* total, int64_t* out_cols, int32_t* out_ids,
                   int64_t out_stride, intptr_t stream);
void step_begin(uint32_t* cursor, int nb, int64_t* stats, intptr_t stream);
void rolling_lookup_direct(const uint64_t* keys, const uint64_t* vals, uint32_t n, int nsub_log2,
                           int cap_log2, uint64_t* keys_g, int64_t* sort_key, uint64_t* vals_out,
                           uint32_t* n_out, uint32_t* flags, int shift, intptr_t stream);
void rolling_lookup(const Rec* recs, const uint32_t* counts, int nsrc, int nsub,
                    uint32_t bucket_cap, int cap_log2, uint64_t* keys_g, int64_t* sort_key,
                    uint64_t* vals_out, uint32_t* n_out, uint32_t* flags, int abits, int shift,
                    intptr_t stream);
void rolling_heads(const int64_t* sk, const uint32_t* n_in, int64_t n_cap, uint32_t* heads,
                   uint32_t* n_heads, int shift, intptr_t stream);
// Sort-free rolling COUNT for state tables of <= kRollHistMaxSlots slots (rolling_hist_hip.hip):
// hist -> cross-chunk prefix -> tile-ranked emit; the same rows as lookup_direct + sort + scan.
size_t rolling_hist_scratch_bytes(int64_t n, int64_t nslots);
bool rolling_hist_supported(int agg, uint32_t count_n, int64_t nslots, const ExprProg& filt);
void rolling_hist(const uint64_t* keys, int64_t n, int nsub_log2, int cap_log2, uint64_t* keys_g,
                  uint32_t* cnt_g, void* scratch, size_t scratch_bytes, const ExprProg& filt,
                  uint64_t* out_key, uint64_t* out_val, int64_t* out_tag, uint32_t* out_n,
                  uint32_t out_cap, uint32_t* flags, int dense, intptr_t stream);
// rec_words: the bucketed records' width (3 = 24-byte Rec, 2 = 16-byte RecC); the diverted
// host records are always written as 24-byte Rec.
void session_lookup(const void* recs, const uint32_t* counts, int nsrc, int nsub, uint32_t bcap,
                    int cap_log2, uint64_t* keys_g, uint64_t* spill_set, uint32_t spill_mask,
                    int spill_any, int64_t* sk, uint64_t* vals, uint32_t* n_out, Rec* host_recs,
                    uint32_t* n_host, uint32_t host_cap, uint32_t* n_inserted, int tbits,
                    intptr_t stream, int rec_words = 3);
// Fused lookup + per-sub-table LDS segmented sort: writes the kept records in (slot, ts) order
// (the stable sort of session_lookup's keys without holes). Returns false (nothing launched)
// when a sub-table's records cannot be staged in LDS (then: session_lookup + a device sort).
bool session_lookup_sort(const void* recs, const uint32_t* counts, int nsrc, int nsub,
                         uint32_t bcap, int cap_log2, uint64_t* keys_g, uint64_t* spill_set,
                         uint32_t spill_mask, int spill_any, int64_t* sort_out, uint64_t* vals_out,
                         uint32_t* n_out, Rec* host_recs, uint32_t* n_host, uint32_t host_cap,
                         uint32_t* n_inserted, int tbits, intptr_t stream,
                         const int64_t* skip = nullptr, uint32_t skip_mask = 0,
                         uint64_t* heads_out = nullptr, uint32_t* n_heads = nullptr,
                         int pair = 0, int rec_words = 3);
void session_heads(const int64_t* sk, const uint32_t* n_in, int64_t n_cap, uint32_t* heads,
                   uint32_t* n_heads, intptr_t stream);
void session_merge(const int64_t* sk, const uint64_t* vals, const uint32_t* n_in,
                   uint32_t* long_heads, uint32_t* n_long, int64_t n_cap, int tbits, int64_t gap,
                   int64_t lateness, int64_t wm, int64_t tbase, int agg, int cap_log2,
                   int64_t nslots, int64_t* sess, int64_t* slot_due, int64_t* slot_last,
                   uint64_t* late_cnt, const uint64_t* keys_g, int64_t* ovf_slots,
                   uint32_t* n_ovf, int64_t* ovf_rows, uint32_t* n_ovf_runs, uint32_t ovf_cap,
                   intptr_t stream);
// session_merge over the segment list of session_lookup_sort (position | length << 32).
void session_merge_heads(const int64_t* sk, const uint64_t* vals, const uint32_t* n_in,
                         const uint64_t* heads, const uint32_t* n_heads, int64_t head_cap,
                         uint32_t* long_heads, uint32_t* n_long, int tbits, int64_t gap,
                         int64_t lateness, int64_t wm, int64_t tbase, int agg, int cap_log2,
                         int64_t nslots, int64_t* sess, int64_t* slot_due, int64_t* slot_last,
                         uint64_t* late_cnt, const uint64_t* keys_g, int64_t* ovf_slots,
                         uint32_t* n_ovf, int64_t* ovf_rows, uint32_t* n_ovf_runs,
                         uint32_t ovf_cap, intptr_t stream, int pair = 0);
void session_fire(int64_t gap, int64_t lateness, int64_t wm, int agg, int cap_log2,
                  int64_t nslots, const uint64_t* keys_g, int64_t* sess, int64_t* slot_due,
                  const ExprProg& map, const ExprProg& filt, uint64_t* out_key, int64_t* out_start,
                  int64_t* out_end, double* out_val, uint64_t* out_raw, uint32_t* out_cnt,
                  uint32_t* out_n, uint32_t out_cap, intptr_t stream);
void session_evict(int64_t nslots, int cap_log2, uint64_t* keys_g, int64_t* sess,
                   int64_t* slot_due, int64_t* slot_last, int64_t idle_before, const int64_t* slots,
                   uint32_t nslots_list, uint64_t* spill_set, uint32_t spill_mask, int64_t* st_key,
                   int64_t* st_start, int64_t* st_end, int64_t* st_acc, int64_t* st_cnt,
                   int64_t* st_flags, uint32_t* n_rows, uint32_t row_cap, uint32_t* n_evicted,
                   intptr_t stream);
size_t sort_pairs_temp_bytes(int64_t n, int begin_bit, int end_bit);
void sort_pairs(void* temp, size_t temp_bytes, const uint64_t* keys_in, uint64_t* keys_out,
                const uint64_t* vals_in, uint64_t* vals_out, int64_t n, int begin_bit, int end_bit,
                intptr_t stream);
void keygroups(const uint64_t* keys, int64_t n, int hash_mode, const int32_t* jhash, int max_par,
               int32_t* kg, intptr_t stream);
void table_insert(const uint64_t* keys, int64_t n, int nsub_log2, int cap_log2, uint64_t* keys_g,
                  int64_t* slots, intptr_t stream);
void window_combine(const Rec* recs, const uint32_t* counts, int nbuckets, const AggPlan& plan,
                    Rec* out, uint32_t ccap, uint32_t* out_counts, uint32_t* flags,
                    intptr_t stream);
void parse_text(const char* text, int64_t text_len, const int64_t* starts, int64_t nlines,
                const int32_t* fields, const int32_t* kinds, int nfields, char sep,
                int64_t offset_s, int64_t* cols, int32_t* jhash, uint8_t* status,
                intptr_t stream, const int64_t* nlines_dev = nullptr, uint32_t* nflag = nullptr);
void f64_order_bits(const uint64_t* v, int64_t n, uint64_t* o, intptr_t stream);
void segment_median(const int64_t* heads, int64_t nseg, int64_t total, const uint64_t* ord,
                    double* out, intptr_t stream);
// The same medians over segments whose values are NOT sorted (selection per segment).
void segment_median_select(const int64_t* heads, int64_t nseg, int64_t total,
                           const uint64_t* ord, double* out, intptr_t stream);
void set_erase(uint64_t* set, uint32_t mask, const int64_t* keys, int64_t n, intptr_t stream);
void set_insert_keys(uint64_t* set, uint32_t mask, const int64_t* keys, int64_t n,
                     intptr_t stream);
void set_probe(const uint64_t* set, uint32_t mask, const int64_t* keys, int64_t n, uint8_t* hit,
               uint32_t* n_hit, intptr_t stream);
// Insert keys into the session slot table (tombstone reuse); slot -1 when a sub-table is full.
void session_promote_rows(const int64_t* rows, int64_t n, int nsub_log2, int cap_log2,
                          uint64_t* keys_g, int64_t* slots, int64_t* sess, int64_t* slot_due,
                          int64_t* slot_last, uint32_t* inserted, uint32_t* n_bad,
                          intptr_t stream);
void session_promote(const int64_t* slots, const int64_t* rec, const int64_t* last, int64_t n,
                     int64_t* sess, int64_t* slot_due, int64_t* slot_last, uint32_t* n_bad,
                     intptr_t stream);
void session_slot_insert(const uint64_t* keys, int64_t n, int nsub_log2, int cap_log2,
                         uint64_t* keys_g, int64_t* slots, uint32_t* inserted, intptr_t stream);
// Re-insert the live keys of a spill set into a fresh (empty-filled) set of new_mask + 1 entries.
void set_rehash(const uint64_t* old, int64_t n_old, uint64_t* neu, uint32_t new_mask,
                intptr_t stream);
void session_rehash(int64_t nslots, int cap_log2, const uint64_t* keys_o, const int64_t* sess_o,
                    const int64_t* due_o, const int64_t* last_o, uint64_t* keys_n, int64_t* sess_n,
                    int64_t* due_n, int64_t* last_n, uint32_t* inserted, intptr_t stream);
void rolling_scan(int agg, const int64_t* sk, const int64_t* perm, const uint64_t* vals,
                  const uint32_t* n_in, const uint32_t* heads, const uint32_t* n_heads,
                  int64_t max_segments, uint64_t* acc_g, uint32_t* cnt_g, const uint64_t* keys_g,
                  const ExprProg& filt, uint64_t* out_key, uint64_t* out_val, int64_t* out_tag,
                  uint32_t* out_n, uint32_t out_cap, int abits, int shift, intptr_t stream,
                  uint32_t count_n = 0);
// idle: this partition is idle (red[2] = +inf: no say in the MIN watermark); host_red: also
// store the reduced vector into this pinned host buffer (one rank: no all-reduce in between, so
// the step's host read needs no separate copy).
// fill_word (with the bucket cursors): red[3] carries -(largest bucket fill) instead of
// -(overflow bit) (an overflow is -2^40): the MIN all-reduce then gives every rank the global
// fill that sizes the exchange.
// next_cursor / next_stats (both or neither): the buffers of a later step, zeroed and reset
// here as step_begin would -- that step then skips its step_begin launch (WindowStep rotates
// three cursor / stats sets, so the set reset here is no longer read by anything queued).
void step_finish(const int64_t* stats, int64_t* local_maxts, int64_t bound, int32_t event_mode,
                 int64_t proc_now, int64_t* red, const uint32_t* flags, intptr_t stream,
                 int32_t idle = 0, int64_t* host_red = nullptr, int32_t fill_word = 0,
                 const uint32_t* cursor = nullptr, int nb = 0, uint32_t* next_cursor = nullptr,
                 int64_t* next_stats = nullptr);
// The combiner's overflow check as a MIN all-reduce operand: chk = [-(flags[0] & 2),
// -max(counts[0..nb))], and chk[2] = sum(counts) (this rank's combined records).
void combine_check(const uint32_t* flags, const uint32_t* counts, int nb, int64_t* chk,
                   intptr_t stream);
void fill_u64(uint64_t* p, int64_t n, uint64_t v, intptr_t stream);
// Purge of consecutive pane slabs: zero acc (acc_bytes per slot: 8, or 4 x dim for vectors),
// cnt and dirty of slots [so, so + n) in one launch (16-byte stores).
void zero_panes(void* acc, int acc_bytes, uint32_t* cnt, uint8_t* dirty, int64_t so, int64_t n,
                intptr_t stream);
// Exchange repack (keyBy all-to-all without padding): bucket b's first min(counts[b], dst_cap)
// records (`words` u64 words each) from stride src_cap to stride dst_cap, so the equal-split
// all-to-all moves dst_cap-record slices sized to the largest fill over all ranks instead of the
// fixed partition capacity. xstat (optional): += [dst bytes, payload bytes] of this repack.
void bucket_repack(const uint64_t* src, const uint32_t* counts, int nb, uint32_t src_cap,
                   uint32_t dst_cap, int words, uint64_t* dst, uint64_t* xstat, intptr_t stream);
// -max(counts[0..nb)) into *out (a MIN all-reduce operand: the largest fill over the ranks).
void neg_max_u32(const uint32_t* counts, int nb, int64_t* out, intptr_t stream);
// Sign-extend int32 key ids to int64 (paths that do not read an int32 key column).
void widen_i32(const int32_t* in, int64_t n, int64_t* out, intptr_t stream);
void scatter_partials(const uint64_t* keys, const uint64_t* acc, const uint32_t* cnt,
                      const uint32_t* n_in, const ScatPlan& plan, const int32_t* jhash,
                      const int32_t* kg_dest, uint32_t* cursor, Rec* out, uint32_t* flags,
                      intptr_t stream);
// Per sub-table: drop keys without live data, move keys whose newest data pane <= cutoff out
// (rows), rehash the kept keys into a tombstone-free table carrying their pane state along
// (live panes [p_lo, p_lo + np) of the ring). occupancy[sub] = kept keys.
void window_compact(uint64_t* keys_g, uint64_t* acc_g, uint32_t* cnt_g, uint8_t* dirty_g,
                    int nsub, int cap_log2, int ring, int64_t p_lo, int np, int64_t cutoff,
                    const CompactOut& out, uint32_t* occupancy, intptr_t stream);
// The compaction's first min(*n_dev, cap) evicted rows grouped by pane (panes [p_lo, p_lo + np),
// np <= 64) into okey / oacc / ocnt / odirty; counts[j] = rows of pane p_lo + j (counts holds
// 128 words: [64, 128) are the scatter cursors).
void window_rows_pane_sort(const uint64_t* key, const int64_t* pane, const uint64_t* acc,
                           const uint32_t* cnt, const uint8_t* dirty, const uint32_t* n_dev,
                           uint32_t cap, int64_t p_lo, int np, uint64_t* okey, uint64_t* oacc,
                           uint32_t* ocnt, uint8_t* odirty, uint32_t* counts, intptr_t stream);
// (dacc/dcnt: the delta ring of local-global aggregation, zeroed for the same slots and panes.)
void dirty_clear(const uint32_t* list, const uint32_t* list_n, uint32_t list_cap, int ring,
                 int64_t nslots, uint8_t* dirty_g, uint32_t* slot_mark, int64_t p_lo, int np,
                 intptr_t stream, uint64_t* dacc = nullptr, uint32_t* dcnt = nullptr);
// Tiered firing (host-DRAM window tier): rows (key, raw accumulator, count) -- a window's device
// rows and the tier's rows of its panes -- combined per key into a global open-addressing table
// (tkeys = kEmptyKey, tacc = agg_identity, tcnt = 0 initially; mask + 1 slots). n_dev (optional):
// the device row count, read on the device (rows = min(n, *n_dev)). mode bit0: mark the row's
// key dirty (a re-firing's device rows); bit1: find only (rows of keys not in the table are
// skipped: a re-firing's tier rows). A full table sets flags[0] bit0.
void tier_merge(const uint64_t* keys, const uint64_t* acc, const uint32_t* cnt, int64_t n,
                const uint32_t* n_dev, int mode, int agg, uint64_t* tkeys, uint64_t* tacc,
                uint32_t* tcnt, uint8_t* tdirty, uint32_t mask, uint32_t* flags, intptr_t stream);
}  // namespace gpu

// ---- CPU twins (kernels_cpu.cpp) ------------------------------------------------------------
namespace cpu {
// C++ twins of the packed-row exchange (same layouts; counts then stable scatter, unpack).
void xrows_count(const int64_t* dest, int64_t n, int world, uint32_t* counts, uint32_t* bad);
void xrows_scatter(const int64_t* dest, int64_t n, int world, uint32_t cap, const XRowCols& c,
                   uint32_t* send, uint32_t* ovf);
void xrows_unpack(const uint32_t* recv, const uint32_t* rc, int world, uint32_t cap,
                  const XRowCols& c);
void format_rows_len(const FmtArgs& a, int64_t n, int64_t* len, uint32_t* bad);
void format_rows_write(const FmtArgs& a, int64_t n, const int64_t* end, char* out);
void set_threads(int n);  // worker threads of the parallel CPU twins (expr_filter, ...)
int get_threads();
void gen_events(uint64_t* keys, int64_t* ts, uint64_t* vals, int64_t n, uint64_t seed,
                uint64_t stream_id, uint64_t idx0, uint64_t nkeys, int64_t ts_base,
                int64_t ts_span, int64_t disorder, int64_t val_lo, int64_t val_span,
                int32_t val_f64, double zipf_s, uint64_t key_base = 0);
void partition(const uint64_t* keys, const int64_t* ts, const uint64_t* vals,
               const int32_t* jhash_tab, int64_t n, const PartPlan& plan, const int32_t* kg_dest,
               uint32_t* cursor, Rec* out, int64_t* stats, uint32_t* late_idx, uint32_t late_cap);
void window_agg(const Rec* recs, const uint32_t* counts, const AggPlan& plan, uint64_t* keys_g,
                uint64_t* acc_g, uint32_t* cnt_g, uint8_t* dirty_g, uint32_t* occupancy,
                uint32_t* flags);
void window_fire(const uint64_t* keys_g, const uint64_t* acc_g, const uint32_t* cnt_g,
                 const uint8_t* dirty_g, const FirePlan& plan, uint64_t* out_keys,
                 double* out_vals, uint64_t* out_raw, uint32_t* out_cnt, uint32_t* out_n);
void rolling(const Rec* recs, const uint32_t* counts, const RollPlan& plan, uint64_t* keys_g,
             uint64_t* acc_g, uint32_t* cnt_g, uint32_t* occupancy, uint32_t* flags,
             uint64_t* out_vals);
void expr_filter(const double* x, int64_t n, const ExprProg& prog, uint8_t* keep);
void expr_filter_compact(const double* x, int64_t n, const ExprProg& prog, int64_t* idx,
                         int64_t* total);
void step_begin(uint32_t* cursor, int nb, int64_t* stats);
// C++ twins of the device text ingest (csrc/ingest_cpu.cpp): identical outputs and ids.
void line_starts(const uint8_t* buf, int64_t n, int64_t* idx, int64_t* total);
void ingest_parse(const char* text, int64_t text_len, const int64_t* starts, int64_t n,
                  const IngestSpec& sp, const IngestOut& o, const DictState& d);
void dict_assign_new(const char* text, int64_t n, int32_t nstr, const IngestOut& o,
                     const DictState& d, int64_t* newpos);
void dict_rehash(const uint64_t* old_h, const int32_t* old_id, int64_t old_cap, const DictState& d);
void dict_find_new(int64_t n, int32_t nstr, const IngestOut& o, const DictState& d,
                   int64_t* newpos);
void dict_insert_ids(const uint8_t* buf, const int64_t* offs, const int32_t* lens, int64_t k,
                     int64_t id0, const DictState& d);
void dict_resolve(const char* text, int64_t n, int32_t nstr, const IngestOut& o,
                  const DictState& d);
void ingest_filter_compact(const int64_t* cols, int64_t n, int32_t nf, int32_t dbl_mask,
                           const ExprProg& prog, int64_t* idx, int64_t* total);
void ingest_gather(const int64_t* cols, int64_t n, int32_t nf, const int32_t* ids, int32_t nstr,
                   const int64_t* idx, const int64_t* total, int64_t* out_cols, int32_t* out_ids,
                   int64_t out_stride);
void rolling_rows(const Rec* recs, const uint32_t* counts, int nsrc, int nsub, uint32_t bucket_cap,
                  int cap_log2, int agg, uint64_t* keys_g, uint64_t* acc_g, uint32_t* cnt_g,
                  uint32_t* flags, const ExprProg& filt, uint64_t* out_key, uint64_t* out_val,
                  int64_t* out_tag, uint32_t* out_n, uint32_t out_cap, uint32_t count_n = 0);
void step_finish(const int64_t* stats, int64_t* local_maxts, int64_t bound, int32_t event_mode,
                 int64_t proc_now, int64_t* red, const uint32_t* flags, int32_t idle = 0,
                 int32_t fill_word = 0, const uint32_t* cursor = nullptr, int nb = 0);
void bucket_repack(const uint64_t* src, const uint32_t* counts, int nb, uint32_t src_cap,
                   uint32_t dst_cap, int words, uint64_t* dst, uint64_t* xstat);
void keygroups(const uint64_t* keys, int64_t n, int hash_mode, const int32_t* jhash, int max_par,
               int32_t* kg);
void table_insert(const uint64_t* keys, int64_t n, int nsub_log2, int cap_log2, uint64_t* keys_g,
                  int64_t* slots);
void window_combine(const Rec* recs, const uint32_t* counts, int nbuckets, const AggPlan& plan,
                    Rec* out, uint32_t ccap, uint32_t* out_counts, uint32_t* flags);
void f64_order_bits(const uint64_t* v, int64_t n, uint64_t* o);
void segment_median(const int64_t* heads, int64_t nseg, int64_t total, const uint64_t* ord,
                    double* out);
void segment_median_select(const int64_t* heads, int64_t nseg, int64_t total,
                           const uint64_t* ord, double* out);
void scatter_partials(const uint64_t* keys, const uint64_t* acc, const uint32_t* cnt,
                      const uint32_t* n_in, const ScatPlan& plan, const int32_t* jhash,
                      const int32_t* kg_dest, uint32_t* cursor, Rec* out, uint32_t* flags);
// Per sub-table: drop keys without live data, move keys whose newest data pane <= cutoff out
// (rows), rehash the kept keys into a tombstone-free table carrying their pane state along
// (live panes [p_lo, p_lo + np) of the ring). occupancy[sub] = kept keys.
void window_compact(uint64_t* keys_g, uint64_t* acc_g, uint32_t* cnt_g, uint8_t* dirty_g,
                    int nsub, int cap_log2, int ring, int64_t p_lo, int np, int64_t cutoff,
                    const CompactOut& out, uint32_t* occupancy);
void dirty_clear(const uint32_t* list, const uint32_t* list_n, uint32_t list_cap, int ring,
                 int64_t nslots, uint8_t* dirty_g, uint32_t* slot_mark, int64_t p_lo, int np,
                 uint64_t* dacc = nullptr, uint32_t* dcnt = nullptr);
void tier_merge(const uint64_t* keys, const uint64_t* acc, const uint32_t* cnt, int64_t n,
                const uint32_t* n_dev, int mode, int agg, uint64_t* tkeys, uint64_t* tacc,
                uint32_t* tcnt, uint8_t* tdirty, uint32_t mask, uint32_t* flags);
}  // namespace cpu

}  // namespace mxs
