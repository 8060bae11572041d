"""Validated launch wrappers around the native kernels.

Every wrapper checks dtype, device, contiguity and the sizes the kernel's grid assumes BEFORE
launching (a mis-shaped operand must never reach a hand-written kernel), then dispatches to the
gfx950 kernel for CUDA(HIP) tensors or to the C++ twin for CPU tensors. There is no Python
fallback: a missing extension raises.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch

from . import expr as _expr
from .native import load

REC_WORDS = 3  # 24-byte record = 3 x int64 words
STAT_COUNT = 8
STAT_MAXTS, STAT_MINPANE, STAT_MAXPANE, STAT_LATE, STAT_OVERFLOW, STAT_ACCEPTED, STAT_MAXBUCKET = range(7)
AGG_SLICE = 131072  # records per workgroup of a split sub-table (csrc kAggSliceMin)

I64_MIN = -(1 << 63)
I64_MAX = (1 << 63) - 1

# AggKind (csrc/mxs_common.h)
AGG_SUM_I64, AGG_SUM_F64, AGG_MIN_I64, AGG_MAX_I64, AGG_MIN_F64, AGG_MAX_F64, AGG_COUNT, \
    AGG_AVG_F64, AGG_AVG_I64 = range(9)
AGG_IS_F64 = {AGG_SUM_F64, AGG_MIN_F64, AGG_MAX_F64, AGG_AVG_F64}


def _is_gpu(t: torch.Tensor) -> bool:
    return t.device.type == "cuda"


def _stream(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


def _p(t: torch.Tensor | None) -> int:
    return 0 if t is None else t.data_ptr()


def resolve_device(d) -> torch.device:
    """torch.device with an explicit index: a bare 'cuda' means the current device (operators
    compare tensor devices against theirs, and tensors always carry the index)."""
    d = torch.device(d)
    if d.type == "cuda" and d.index is None:
        return torch.device("cuda", torch.cuda.current_device())
    return d


def _check(t: torch.Tensor, dtype: torch.dtype, numel_min: int, name: str, dev: torch.device):
    if t.dtype != dtype:
        raise TypeError(f"{name}: expected {dtype}, got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{name}: must be contiguous")
    if t.numel() < numel_min:
        raise ValueError(f"{name}: needs >= {numel_min} elements, has {t.numel()}")
    if t.device != dev and t.device != resolve_device(dev):
        raise ValueError(f"{name}: on {t.device}, expected {dev}")


def new_stats(device) -> torch.Tensor:
    s = torch.zeros(STAT_COUNT, dtype=torch.int64, device=device)
    s[STAT_MAXTS] = I64_MIN
    s[STAT_MINPANE] = I64_MAX
    s[STAT_MAXPANE] = I64_MIN
    return s


def reset_stats(s: torch.Tensor) -> None:
    init = torch.tensor([I64_MIN, I64_MAX, I64_MIN, 0, 0, 0, 0, 0], dtype=torch.int64)
    s.copy_(init, non_blocking=False)


def gen_events(keys, ts, vals, *, seed: int, stream_id: int, idx0: int, nkeys: int,
               ts_base: int, ts_span: int, disorder: int, val_lo: int, val_span: int,
               val_f64: bool = False, zipf: float = 0.0, key_base: int = 0) -> None:
    """keys: int64, or int32 (dictionary ids, nkeys < 2^31). zipf > 0: power-law skewed keys
    with that exponent (key 0 hottest; csrc/mxs_common.h zipf_key), 0: uniform. key_base: added
    to every key (a drifting key window without a separate pass)."""
    n = keys.numel()
    dev = keys.device
    key32 = keys.dtype == torch.int32
    _check(keys, torch.int32 if key32 else torch.int64, n, "keys", dev)
    _check(ts, torch.int64, n, "ts", dev)
    _check(vals, torch.int64, n, "vals", dev)
    if nkeys <= 0 or nkeys >= (1 << (31 if key32 else 63)):
        raise ValueError("nkeys out of range")
    m = load()
    args = (_p(keys), _p(ts), _p(vals), n, seed & (2**64 - 1), stream_id & (2**64 - 1), idx0,
            nkeys, ts_base, ts_span, disorder, val_lo, val_span, int(val_f64) | (2 if key32 else 0),
            float(zipf))
    if zipf < 0:
        raise ValueError("zipf exponent must be >= 0")
    if key_base < 0:
        raise ValueError("key_base must be >= 0")
    if _is_gpu(keys):
        m.gpu_gen_events(*args, _stream(keys), key_base)
    else:
        m.cpu_gen_events(*args, key_base)


@dataclass
class PartitionPlan:
    """keyBy + window assignment plan of one step (csrc/mxs_common.h PartPlan)."""

    max_parallelism: int
    nsub_log2: int
    nranks: int
    window_mode: int
    drop_late: int
    hash_mode: int
    bucket_cap: int
    late_ts: int = I64_MIN   # elements with ts < late_ts are late (all windows cleaned)
    tbase: int = 0           # start of the step's base pane
    pane: int = 1            # pane length (ms)
    ablate: int = 0          # profiling-only ablation bits
    rec_words: int = 3       # 3: 24-byte records; 2: 16-byte records (int32 values, window path)
    dense_bits: int = 0      # > 0: dense key ids < 2^dense_bits, directly addressed
    dense_mul: int = 0       # odd multiplier of the dense slot bijection
    key32: int = 0           # 1: int32 key column (compact-record GPU partition only)
    scratch: int = 0         # GPU two-level partition (> 512 buckets): coarse staging buffer
    scratch_cursor: int = 0  # ... and its 512 coarse cursors (data pointers; 0 = plain scatter)

    @property
    def nbuckets(self) -> int:
        return self.nranks << self.nsub_log2

    def as_dict(self) -> dict:
        return dict(self.__dict__)


def partition(keys, ts, vals, plan: PartitionPlan, kg_dest, cursor, out, stats,
              jhash=None, late_idx=None) -> None:
    n = keys.numel()
    dev = keys.device
    nb = plan.nbuckets
    _check(keys, torch.int64, n, "keys", dev)
    _check(ts, torch.int64, n, "ts", dev)
    _check(vals, torch.int64, n, "vals", dev)
    _check(kg_dest, torch.int32, plan.max_parallelism, "kg_dest", dev)
    _check(cursor, torch.int32, nb, "cursor", dev)
    _check(out, torch.int64, nb * plan.bucket_cap * REC_WORDS, "out", dev)
    _check(stats, torch.int64, STAT_COUNT, "stats", dev)
    if plan.hash_mode:
        if jhash is None:
            raise ValueError("hash_mode=1 needs the dictionary jhash table")
        _check(jhash, torch.int32, 1, "jhash", dev)
    if nb > 16384:
        raise ValueError("too many buckets (ranks x sub-tables > 16384)")
    if n >= (1 << 32):
        raise ValueError("batch too large (2^32 events)")
    late_cap = 0 if late_idx is None else late_idx.numel()
    if late_idx is not None:
        _check(late_idx, torch.int32, 0, "late_idx", dev)
    m = load()
    args = (_p(keys), _p(ts), _p(vals), _p(jhash), n, plan.as_dict(), _p(kg_dest), _p(cursor),
            _p(out), _p(stats), _p(late_idx), late_cap)
    if _is_gpu(keys):
        m.gpu_partition(*args, _stream(keys))
    else:
        m.cpu_partition(*args)


@dataclass
class AggPlan:
    cap_log2: int
    nsub: int
    ring: int
    agg: int
    nsrc: int
    bucket_cap: int
    np_step: int
    pg: int
    pane_base: int
    p_lo: int
    fired_hi: int
    combined: int = 0    # records are pre-aggregated by window_combine (aux = element count)
    rec_words: int = 3   # layout of the input records (3: Rec, 2: RecC)
    dlist: int = 0       # touched-slot list (data pointers, 0 = off): slot ids ...
    dlist_n: int = 0     # ... its length ...
    slot_mark: int = 0   # ... and the per-slot listed marks
    dense_bits: int = 0  # > 0: directly addressed dense key ids (see PartitionPlan)
    dense_mul: int = 0
    split: int = 1       # workgroups sharing an oversized sub-table (hot keys; GPU, see AGG_SLICE)
    det: int = 0         # 1: deterministic f64 sums (128-bit fixed-point per-step slot sums)
    dacc: int = 0        # local-global delta ring of late data (data pointers, 0 = off) ...
    dcnt: int = 0        # ... and its counts
    skip: int = 0        # device int64: non-zero -> leave the state untouched (incomplete exchange)
    pmask: int = 0       # GPU: relative panes with records (sparse pane rows; np_step = popcount)

    def as_dict(self) -> dict:
        return dict(self.__dict__)


def window_combine(recs, counts, plan: AggPlan, out, ccap: int, out_counts, flags) -> None:
    """Sender-side combiner: one pre-aggregated record per (key, pane) of every send bucket.
    `plan.nsub` here is the number of send buckets (ranks x sub-tables)."""
    dev = recs.device
    nb = plan.nsub
    _check(recs, torch.int64, nb * plan.bucket_cap * REC_WORDS, "recs", dev)
    _check(counts, torch.int32, nb, "counts", dev)
    _check(out, torch.int64, nb * ccap * REC_WORDS, "out", dev)
    _check(out_counts, torch.int32, nb, "out_counts", dev)
    _check(flags, torch.int32, 1, "flags", dev)
    if (1 << plan.cap_log2) * 8 + plan.pg * (1 << plan.cap_log2) * 12 + 16 > 160 * 1024:
        raise ValueError("window_combine: LDS plan too large")
    m = load()
    args = (_p(recs), _p(counts), nb, plan.as_dict(), _p(out), int(ccap), _p(out_counts), _p(flags))
    if _is_gpu(recs):
        m.gpu_window_combine(*args, _stream(recs))
    else:
        m.cpu_window_combine(*args)


def window_agg(recs, counts, plan: AggPlan, keys_g, acc_g, cnt_g, dirty_g, occ, flags) -> None:
    dev = keys_g.device
    nslots = plan.nsub << plan.cap_log2
    _check(recs, torch.int64, plan.nsrc * plan.nsub * plan.bucket_cap * REC_WORDS, "recs", dev)
    _check(counts, torch.int32, plan.nsrc * plan.nsub, "counts", dev)
    _check(keys_g, torch.int64, nslots, "keys_g", dev)
    _check(acc_g, torch.int64, plan.ring * nslots, "acc_g", dev)
    _check(cnt_g, torch.int32, plan.ring * nslots, "cnt_g", dev)
    _check(dirty_g, torch.uint8, plan.ring * nslots, "dirty_g", dev)
    _check(occ, torch.int32, plan.nsub, "occupancy", dev)
    _check(flags, torch.int32, 1, "flags", dev)
    if plan.np_step > plan.ring:
        raise ValueError("step touches more panes than the ring holds")
    m = load()
    args = (_p(recs), _p(counts), plan.as_dict(), _p(keys_g), _p(acc_g), _p(cnt_g), _p(dirty_g),
            _p(occ), _p(flags))
    if _is_gpu(keys_g):
        m.gpu_window_agg(*args, _stream(keys_g))
    else:
        m.cpu_window_agg(*args)


def window_fire(keys_g, acc_g, cnt_g, dirty_g, *, agg: int, npanes: int, ring: int, p0: int,
                wstart: int, wend: int, only_dirty: bool, map_prog: _expr.Program,
                filt_prog: _expr.Program, out_keys, out_vals, out_raw, out_cnt, out_n,
                ablate: int = 0, slot_list=None, slot_list_n=None, key32: bool = False) -> None:
    """slot_list/slot_list_n (int32 device tensors): visit only the listed slots (re-firings of
    late-but-allowed data) instead of sweeping the table. Compact rows: out_raw / out_cnt None
    (not written) and key32 (keys < 2^32 written as uint32 into out_keys' first 4*n bytes)."""
    dev = keys_g.device
    nslots = keys_g.numel()
    cap = out_keys.numel()
    _check(acc_g, torch.int64, ring * nslots, "acc_g", dev)
    _check(cnt_g, torch.int32, ring * nslots, "cnt_g", dev)
    _check(dirty_g, torch.uint8, ring * nslots, "dirty_g", dev)
    _check(out_vals, torch.float64, cap, "out_vals", dev)
    if out_raw is not None:
        _check(out_raw, torch.int64, cap, "out_raw", dev)
    if out_cnt is not None:
        _check(out_cnt, torch.int32, cap, "out_cnt", dev)
    _check(out_n, torch.int32, 1, "out_n", dev)
    if npanes > ring:
        raise ValueError("window spans more panes than the ring")
    plan = dict(agg=agg, npanes=npanes, ring=ring, only_dirty=int(only_dirty), nslots=nslots,
                p0=p0, wstart=float(wstart), wend=float(wend), out_cap=cap,
                map=tuple(map_prog.as_args()), filt=tuple(filt_prog.as_args()), ablate=ablate,
                key32=int(key32))
    if slot_list is not None:
        _check(slot_list, torch.int32, 0, "slot_list", dev)
        _check(slot_list_n, torch.int32, 1, "slot_list_n", dev)
        plan.update(list=_p(slot_list), list_n=_p(slot_list_n))
    m = load()
    args = (_p(keys_g), _p(acc_g), _p(cnt_g), _p(dirty_g), plan, _p(out_keys), _p(out_vals),
            0 if out_raw is None else _p(out_raw), 0 if out_cnt is None else _p(out_cnt),
            _p(out_n))
    if _is_gpu(keys_g):
        m.gpu_window_fire(*args, _stream(keys_g))
    else:
        m.cpu_window_fire(*args)


def scatter_partials(keys, acc, cnt, n_dev, *, n_cap: int, max_parallelism: int, nranks: int,
                     nsub_log2: int, hash_mode: int, jhash, kg_dest, bucket_cap: int, cursor, out,
                     flags) -> None:
    """Local-global window aggregation: the first min(n_dev[0], n_cap) rows of a local fire
    (key, partial accumulator, count) -> combined records in their owner's (rank, sub-table)
    bucket of `out` (bucket_cap records each; cursor counts). A bucket overflow sets flags bit0
    (the owner's sub-table cannot hold that many keys)."""
    dev = keys.device
    nb = nranks << nsub_log2
    _check(keys, torch.int64, n_cap, "keys", dev)
    _check(acc, torch.int64, n_cap, "acc", dev)
    _check(cnt, torch.int32, n_cap, "cnt", dev)
    _check(n_dev, torch.int32, 1, "n", dev)
    _check(kg_dest, torch.int32, max_parallelism, "kg_dest", dev)
    _check(cursor, torch.int32, nb, "cursor", dev)
    _check(out, torch.int64, nb * bucket_cap * REC_WORDS, "out", dev)
    _check(flags, torch.int32, 1, "flags", dev)
    if hash_mode:
        if jhash is None:
            raise ValueError("hash_mode=1 needs the dictionary jhash table")
        _check(jhash, torch.int32, 1, "jhash", dev)
    if n_cap >= (1 << 32):
        raise ValueError("too many rows")
    plan = dict(max_parallelism=max_parallelism, nranks=nranks, nsub_log2=nsub_log2,
                hash_mode=hash_mode, bucket_cap=bucket_cap, n_cap=n_cap)
    m = load()
    args = (_p(keys), _p(acc), _p(cnt), _p(n_dev), plan, _p(jhash), _p(kg_dest), _p(cursor),
            _p(out), _p(flags))
    if _is_gpu(keys):
        m.gpu_scatter_partials(*args, _stream(keys))
    else:
        m.cpu_scatter_partials(*args)


def dirty_clear(slot_list, slot_list_n, *, ring: int, nslots: int, dirty_g, slot_mark,
                p_lo: int = 0, np_: int | None = None, dacc=None, dcnt=None) -> None:
    """Reset the touched-slot list's dirty bytes (panes p_lo .. p_lo + np_ - 1; default every
    ring pane) and marks -- and the delta ring (dacc/dcnt) of the same slots and panes; the
    caller zeroes the list length afterwards."""
    dev = dirty_g.device
    _check(slot_list, torch.int32, 0, "slot_list", dev)
    _check(slot_list_n, torch.int32, 1, "slot_list_n", dev)
    _check(dirty_g, torch.uint8, ring * nslots, "dirty_g", dev)
    _check(slot_mark, torch.int32, nslots, "slot_mark", dev)
    if dacc is not None:
        _check(dacc, torch.int64, ring * nslots, "dacc", dev)
        _check(dcnt, torch.int32, ring * nslots, "dcnt", dev)
    m = load()
    np_ = ring if np_ is None else max(0, min(int(np_), ring))
    args = (_p(slot_list), _p(slot_list_n), slot_list.numel(), ring, nslots, _p(dirty_g),
            _p(slot_mark), int(p_lo), np_)
    extra = (0, 0) if dacc is None else (_p(dacc), _p(dcnt))
    if _is_gpu(dirty_g):
        m.gpu_dirty_clear(*args, _stream(dirty_g), *extra)
    else:
        m.cpu_dirty_clear(*args, *extra)


def rolling(recs, counts, *, cap_log2: int, nsub: int, agg: int, nsrc: int, bucket_cap: int,
            emit: bool, keys_g, acc_g, cnt_g, occ, flags, out_vals=None) -> None:
    dev = keys_g.device
    nslots = nsub << cap_log2
    _check(recs, torch.int64, nsrc * nsub * bucket_cap * REC_WORDS, "recs", dev)
    _check(counts, torch.int32, nsrc * nsub, "counts", dev)
    _check(keys_g, torch.int64, nslots, "keys_g", dev)
    _check(acc_g, torch.int64, nslots, "acc_g", dev)
    _check(cnt_g, torch.int32, nslots, "cnt_g", dev)
    _check(occ, torch.int32, nsub, "occupancy", dev)
    if emit and out_vals is None:
        raise ValueError("emit needs out_vals")
    plan = dict(cap_log2=cap_log2, nsub=nsub, agg=agg, nsrc=nsrc, bucket_cap=bucket_cap,
                emit=int(emit))
    m = load()
    args = (_p(recs), _p(counts), plan, _p(keys_g), _p(acc_g), _p(cnt_g), _p(occ), _p(flags),
            _p(out_vals))
    if _is_gpu(keys_g):
        m.gpu_rolling(*args, _stream(keys_g))
    else:
        m.cpu_rolling(*args)


def step_begin(cursor: torch.Tensor, stats: torch.Tensor) -> None:
    _check(stats, torch.int64, STAT_COUNT, "stats", cursor.device)
    _check(cursor, torch.int32, cursor.numel(), "cursor", cursor.device)
    m = load()
    if _is_gpu(cursor):
        m.gpu_step_begin(_p(cursor), cursor.numel(), _p(stats), _stream(cursor))
    else:
        m.cpu_step_begin(_p(cursor), cursor.numel(), _p(stats))


RED_WORDS = 16  # [-qmax, qmin, wm, -bucket_ovf, -pane_ovf, -compact_ovf, -table_full, 0, stats[8]]


def step_finish(stats: torch.Tensor, local_maxts: torch.Tensor, red: torch.Tensor, *,
                bound: int, event_mode: bool, proc_now: int,
                flags: torch.Tensor | None = None) -> None:
    """Reduce the partition stats into the step's all-reduce vector (RED_WORDS). With the
    operator's `flags`, red[6] = -(table full): a key that found no slot in a previous
    aggregation surfaces in the step's one host sync."""
    dev = stats.device
    _check(stats, torch.int64, STAT_COUNT, "stats", dev)
    _check(local_maxts, torch.int64, 1, "local_maxts", dev)
    _check(red, torch.int64, RED_WORDS, "red", dev)
    if flags is not None:
        _check(flags, torch.int32, 1, "flags", dev)
    m = load()
    args = (_p(stats), _p(local_maxts), int(bound), int(event_mode), int(proc_now), _p(red),
            _p(flags))
    if _is_gpu(stats):
        m.gpu_step_finish(*args, _stream(stats))
    else:
        m.cpu_step_finish(*args)


def expr_filter_compact(x: torch.Tensor, prog: _expr.Program) -> tuple[torch.Tensor, torch.Tensor]:
    """Indices (int64, input order) of the rows of one f64 column that pass a traced predicate,
    and their number as a 1-element device tensor (the index buffer has x.numel() entries;
    entries past the count are unspecified). No host sync."""
    _check(x, torch.float64, x.numel(), "x", x.device)
    n = x.numel()
    idx = torch.empty(max(n, 1), dtype=torch.int64, device=x.device)
    total = torch.zeros(1, dtype=torch.int64, device=x.device)
    m = load()
    code, consts = prog.as_args()
    if _is_gpu(x):
        scratch = torch.empty(max(1, m.gpu_filter_compact_scratch_bytes(n)), dtype=torch.uint8,
                              device=x.device)
        m.gpu_expr_filter_compact(_p(x), n, code, consts, _p(scratch), _p(idx), _p(total),
                                  _stream(x))
    else:
        m.cpu_expr_filter_compact(_p(x), n, code, consts, _p(idx), _p(total))
    return idx, total


def expr_filter(x: torch.Tensor, prog: _expr.Program) -> torch.Tensor:
    """Evaluate a traced predicate over one f64 column; returns a bool mask."""
    _check(x, torch.float64, x.numel(), "x", x.device)
    keep = torch.empty(x.numel(), dtype=torch.uint8, device=x.device)
    m = load()
    code, consts = prog.as_args()
    if _is_gpu(x):
        m.gpu_expr_filter(_p(x), x.numel(), code, consts, _p(keep), _stream(x))
    else:
        m.cpu_expr_filter(_p(x), x.numel(), code, consts, _p(keep))
    return keep.bool()


def keygroups(keys: torch.Tensor, *, max_parallelism: int, hash_mode: int = 0,
              jhash: torch.Tensor | None = None) -> torch.Tensor:
    """Flink key group of every key (murmur(javaHash) % maxParallelism), int32."""
    dev = keys.device
    _check(keys, torch.int64, keys.numel(), "keys", dev)
    if hash_mode:
        if jhash is None:
            raise ValueError("hash_mode=1 needs the dictionary jhash table")
        _check(jhash, torch.int32, 1, "jhash", dev)
        if keys.numel() and int(keys.max().item()) >= jhash.numel():
            raise ValueError("dictionary id outside the jhash table")
    kg = torch.empty(keys.numel(), dtype=torch.int32, device=dev)
    m = load()
    args = (_p(keys), keys.numel(), int(hash_mode), _p(jhash), int(max_parallelism), _p(kg))
    if _is_gpu(keys):
        m.gpu_keygroups(*args, _stream(keys))
    else:
        m.cpu_keygroups(*args)
    return kg


def table_insert(keys: torch.Tensor, keys_g: torch.Tensor, *, nsub_log2: int,
                 cap_log2: int) -> torch.Tensor:
    """Insert keys into the sub-table hash layout; returns their global slots (-1: table full)."""
    dev = keys.device
    _check(keys, torch.int64, keys.numel(), "keys", dev)
    _check(keys_g, torch.int64, (1 << nsub_log2) << cap_log2, "keys_g", dev)
    if bool(((keys == -1) | (keys == -2)).any()):
        raise ValueError("keys -1 / -2 are reserved (empty / tombstone)")
    slots = torch.empty(keys.numel(), dtype=torch.int64, device=dev)
    m = load()
    args = (_p(keys), keys.numel(), int(nsub_log2), int(cap_log2), _p(keys_g), _p(slots))
    if _is_gpu(keys):
        m.gpu_table_insert(*args, _stream(keys))
    else:
        m.cpu_table_insert(*args)
    return slots


def sort_pairs(keys: torch.Tensor, vals: torch.Tensor, *, bits: int = 64):
    """Stable ascending sort of (uint64 key bits, int64 value) pairs over the low `bits` key bits.
    GPU: the hand-written LSD radix sort (csrc/sort_hip.hip); CPU: torch stable sort."""
    n = keys.numel()
    dev = keys.device
    _check(keys, torch.int64, n, "keys", dev)
    _check(vals, torch.int64, n, "vals", dev)
    if not 1 <= bits <= 64:
        raise ValueError("bits must be in [1, 64]")
    if _is_gpu(keys):
        m = load()
        ko = torch.empty_like(keys)
        vo = torch.empty_like(vals)
        if n:
            need = m.gpu_sort_pairs_temp_bytes(n, 0, bits)
            tmp = torch.empty(max(1, need), dtype=torch.uint8, device=dev)
            m.gpu_sort_pairs(tmp.data_ptr(), tmp.numel(), keys.data_ptr(), ko.data_ptr(),
                             vals.data_ptr(), vo.data_ptr(), n, 0, bits, _stream(keys))
        return ko, vo
    k = keys if bits == 64 else keys & ((1 << bits) - 1)
    # Unsigned order of the 64-bit patterns: flip the sign bit for a signed sort.
    ks = k ^ I64_MIN if bits == 64 else k
    order = torch.sort(ks, stable=True).indices
    return keys[order], vals[order]


def f64_order_bits(v: torch.Tensor) -> torch.Tensor:
    """f64 bit patterns (int64 view) -> u64 bits whose unsigned order is Double.compareTo order."""
    _check(v, torch.int64, v.numel(), "v", v.device)
    o = torch.empty_like(v)
    m = load()
    if _is_gpu(v):
        m.gpu_f64_order_bits(v.data_ptr(), v.numel(), o.data_ptr(), _stream(v))
    else:
        m.cpu_f64_order_bits(v.data_ptr(), v.numel(), o.data_ptr())
    return o


def segment_median(heads: torch.Tensor, ord_bits: torch.Tensor, *, sorted_values: bool = True
                   ) -> torch.Tensor:
    """Median (Java ComputeCpuMiddle semantics) of every segment starting at `heads`.
    sorted_values=False: the values inside a segment are in any order (per-segment selection:
    LDS bitonic sort or radix select, csrc segment_median_select)."""
    dev = ord_bits.device
    _check(heads, torch.int64, heads.numel(), "heads", dev)
    _check(ord_bits, torch.int64, ord_bits.numel(), "ord", dev)
    if heads.numel() and (int(heads[0]) != 0 or int(heads[-1]) >= max(1, ord_bits.numel())):
        raise ValueError("segment heads out of range")
    out = torch.empty(heads.numel(), dtype=torch.float64, device=dev)
    m = load()
    args = (heads.data_ptr(), heads.numel(), ord_bits.numel(), ord_bits.data_ptr(), out.data_ptr())
    name = "segment_median" if sorted_values else "segment_median_select"
    if _is_gpu(ord_bits):
        getattr(m, "gpu_" + name)(*args, _stream(ord_bits))
    else:
        getattr(m, "cpu_" + name)(*args)
    return out
