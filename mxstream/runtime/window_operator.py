"""Keyed window operator: keyBy shuffle + pane-ring window state + watermark-driven firing.

One instance runs per rank (one process per GPU). Per micro-batch (``process``):

 1. ``partition`` kernel: key group -> destination rank (Flink's
    ``murmur(hash) % maxParallelism * P / maxParallelism``), sub-table, pane id, late drop —
    records land in fixed-capacity (dest, sub-table) buckets;
 2. one MIN all-reduce of [-max pane, min pane, local watermark, -overflow] (the watermark valve)
    and the equal-split all-to-all of the bucket ranges + counts (RCCL over xGMI); ONE host sync;
 3. ``window_agg`` kernel: one workgroup per LDS-resident hash sub-table folds the step's
    records into the pane ring (pane = gcd(size, slide); a sliding window is a run of panes);
 4. late-but-allowed data re-fires the touched windows (``only_dirty``); the advanced watermark
    fires every window with ``end - 1 <= wm`` (fused map/filter epilogue + compaction);
 5. panes whose every window passed its cleanup time (``maxTs + allowedLateness <= wm``) are
    zeroed for reuse.

Flink semantics reproduced (reference: ``BandwidthMonitorWithEventTime.java:30-55``,
``BandwidthMonitor.java:32-40``, ``ComputeCpuAvg.java:27-59``):
window assignment, lateness test, per-key emission only for windows that hold data, watermark =
min over source partitions of (max ts - bound), processing-time windows never fire at end of
input. Micro-batch deviation (documented): several late elements of one (key, window) in the same
micro-batch produce one re-firing carrying their combined effect (Flink fires once per element).
"""
from __future__ import annotations

import math
import os as _os
from dataclasses import dataclass, field
from typing import Callable

import numpy as np
import torch

from ..ops import expr as E
from ..ops import kernels as K
from ..parallel.comm import Comm, LocalComm

I64_MIN = K.I64_MIN
I64_MAX = K.I64_MAX


class PinnedSlabPool:
    """Pinned host slabs for fired rows, reused once every array handed out of a slab is gone.

    `torch.empty(..., pin_memory=True)` per fire cost ~1.5 ms of host time per firing in the
    rocprofv3 timeline of the headline bench (profiles/r1_fire_pinned_pool.md): the GPU idled
    between the fire kernel and the D2H copies. A slab is one pinned byte tensor plus its numpy
    view; every column handed out is a numpy view of that array, so the array's refcount says
    whether any caller still holds rows of the slab."""

    def __init__(self, pin: bool = True, max_slabs: int = 8):
        self.pin = pin
        self.max_slabs = max_slabs
        self.slabs: list[tuple[torch.Tensor, np.ndarray]] = []
        self.allocs = 0

    def _free(self, i: int) -> bool:
        # References to a free slab's array: the pool's tuple + getrefcount's own argument.
        import sys

        return sys.getrefcount(self.slabs[i][1]) <= 2

    def reserve_async(self, nbytes: int) -> None:
        """Allocate a slab of `nbytes` (rounded up) on a background thread, for a later take():
        a growing caller (the host tier's firing export) asks ahead of need, so the page-locking
        of a large slab (~25 ms at 512 MB on the box; torch releases the GIL inside it) runs
        beside the step instead of inside it."""
        if not self.pin or getattr(self, "_reserving", None) is not None:
            return
        size = _next_pow2(max(nbytes, 1 << 16))
        if any(s[0].numel() >= size for s in self.slabs):
            return
        import threading

        box = {}

        def work():
            try:
                box["t"] = torch.empty(size, dtype=torch.uint8, pin_memory=True)
            except BaseException as e:  # surfaced by the next take()
                box["err"] = e

        th = threading.Thread(target=work, name="mxs-pin-reserve", daemon=True)
        th.start()
        self._reserving = (th, box)

    def _land_reserve(self, block: bool) -> None:
        r = getattr(self, "_reserving", None)
        if r is None or (not block and r[0].is_alive()):
            return
        r[0].join()
        self._reserving = None
        if "err" in r[1]:
            raise r[1]["err"]
        t = r[1]["t"]
        if len(self.slabs) >= self.max_slabs:
            free = [i for i in range(len(self.slabs)) if self._free(i)]
            if not free:
                return  # every slab is in use: the reserve is dropped
            self.slabs.pop(min(free, key=lambda i: self.slabs[i][0].numel()))
        self.allocs += 1
        self.slabs.append((t, t.numpy()))

    def take(self, nbytes: int) -> tuple[torch.Tensor, np.ndarray]:
        if getattr(self, "_reserving", None) is not None:
            # a reserve in flight that this take needs is waited for (not allocated twice)
            self._land_reserve(block=not any(s[0].numel() >= nbytes and self._free(i)
                                             for i, s in enumerate(self.slabs)))
        for i in range(len(self.slabs)):
            if self.slabs[i][0].numel() >= nbytes and self._free(i):
                return self.slabs[i]
        if len(self.slabs) >= self.max_slabs:
            # Drop the smallest free slab so a long-lived caller cannot grow the pool unbounded.
            free = [i for i in range(len(self.slabs)) if self._free(i)]
            if free:
                self.slabs.pop(min(free, key=lambda i: self.slabs[i][0].numel()))
        t = torch.empty(_next_pow2(max(nbytes, 1 << 16)), dtype=torch.uint8, pin_memory=self.pin)
        self.allocs += 1
        slab = (t, t.numpy())
        self.slabs.append(slab)
        return slab


_TLS = __import__("threading").local()


def _thread_pool() -> PinnedSlabPool:
    """One pool per host thread: virtual ranks of a LoopbackGroup (threads) must never be handed
    the same free slab at once."""
    pool = getattr(_TLS, "pool", None)
    if pool is None:
        pool = _TLS.pool = PinnedSlabPool()
    return pool


def to_host_arrays(cols: list[torch.Tensor], n: int, pool: PinnedSlabPool | None = None) -> list[np.ndarray]:
    """The first n rows of each output column as host arrays. On a GPU: non-blocking copies into
    one pinned slab (reused from `pool` once the caller dropped the previous arrays) and one
    stream sync — a pageable .cpu() stages every column through a bounce buffer at a fraction of
    the PCIe rate. On the CPU: copies (the device buffers are reused by the next fire)."""
    if not cols or cols[0].device.type != "cuda":
        return [c[:n].numpy().copy() for c in cols]
    pool = _thread_pool() if pool is None else pool
    offs, nbytes = [], 0
    for c in cols:
        offs.append(nbytes)
        nbytes += (n * c.element_size() + 255) & ~255
    t, arr = pool.take(nbytes)
    out, copies = [], []
    kernel_ok = _D2H != "dma"
    for o, c in zip(offs, cols):
        nb = n * c.element_size()
        if not c.is_contiguous() or n > c.numel():
            raise ValueError("to_host_arrays: columns must be contiguous with at least n rows")
        nb16 = (nb + 15) & ~15
        kernel_ok = kernel_ok and nb16 <= c.numel() * c.element_size() and c.data_ptr() % 16 == 0
        copies.append((c.data_ptr(), nb16, o))
        out.append(arr[o:o + nb].view(_NP_DTYPE[c.dtype]))
    # The DMA path (hipMemcpyAsync, and torch's copy_ before it) stalled the host for 7-9 ms at
    # one firing in some runs (profiles/r2_fire_d2h.md): a copy kernel storing into the mapped
    # pinned slab by default, one native call either way.
    from ..ops.native import load

    stream = torch.cuda.current_stream(cols[0].device)
    m = load()
    if not kernel_ok or m.gpu_d2h_kernel(t.data_ptr(), copies, stream.cuda_stream) != 0:
        m.gpu_d2h_many(t.data_ptr(), [(p, min(b, n * c.element_size()), o)
                                      for (p, b, o), c in zip(copies, cols)], stream.cuda_stream)
    stream.synchronize()
    return out


_D2H = _os.environ.get("MXS_D2H", "kernel")  # "dma": hipMemcpyAsync (A/B)
# Tiered firings (host-DRAM window tier): "device" (default) combines the tier's rows with the
# device's on the GPU; "host": the C++ host merge (A/B, the round-3 path).
_TIER_MERGE = _os.environ.get("MXS_TIER_MERGE", "device")
# Evicted rows grouped by pane on the GPU before their D2H (window_rows_pane_sort); "0": the
# tier's host counting sort (A/B).
_EVICT_PANE_SORT = _os.environ.get("MXS_EVICT_PANE_SORT", "1") != "0"
# The presorted eviction's copy into the tier on a background thread ("1"; off by default: a
# re-firing over tier panes joins it within the step, config 4-spill 1.44 vs 1.60 G events/s,
# profiles/r4s_cfg4spill_bg_absorb.json).
_TIER_BG_ABSORB = _os.environ.get("MXS_TIER_BG_ABSORB", "0") == "1"


def _agg_identity(agg: int) -> int:
    """agg_identity (csrc/mxs_common.h) as an int64 bit pattern."""
    if agg == K.AGG_MIN_I64:
        return I64_MAX
    if agg == K.AGG_MAX_I64:
        return I64_MIN
    if agg == K.AGG_MIN_F64:
        return 0x7FF0000000000000
    if agg == K.AGG_MAX_F64:
        return 0xFFF0000000000000 - (1 << 64)
    return 0


class CountedHostRows:
    """Columns whose row count is still on the device, copied to one pinned slab WITHOUT a host
    round trip: the copy kernel reads the uint32 count (`n_dev`) itself and moves only that many
    rows (gpu_d2h_counted); small `fixed` device tensors (flags, per-window bounds) ride along
    whole. The host reads the slab once `ready()` -- nothing blocks at launch, so a firing no
    longer drains the stream twice (once for its count, once for its rows).

    Layout: fixed tensors first (16-byte granules), then each column at its capacity."""

    def __init__(self, pool: PinnedSlabPool, cols: list[torch.Tensor], n_dev: torch.Tensor,
                 fixed: list[torch.Tensor] = (), copy_stream=None):
        """copy_stream: run the copy there, after the producer's work on the current stream
        (it overlaps the compute that follows; ``done`` is the event the producer must wait for
        before it overwrites the columns)."""
        from ..ops.native import load

        self.cols_meta, self.fixed_meta, copies, off = [], [], [], 0
        for t in fixed:
            nb = t.numel() * t.element_size()
            if nb % 16 or not t.is_contiguous() or t.data_ptr() % 16:
                raise ValueError("CountedHostRows: fixed tensors must be 16-byte granules")
            copies.append((t.data_ptr(), nb, off, 0))
            self.fixed_meta.append((off, nb, t.dtype))
            off += (nb + 255) & ~255
        self.cap = min(c.numel() for c in cols)
        for c in cols:
            nb = self.cap * c.element_size()
            if not c.is_contiguous() or c.data_ptr() % 16 or nb % 16:
                raise ValueError("CountedHostRows: columns must be contiguous, 16-byte aligned "
                                 "and a 16-byte multiple long")
            copies.append((c.data_ptr(), nb, off, c.element_size()))
            self.cols_meta.append((off, c.dtype))
            off += (nb + 255) & ~255
        t0 = __import__("time").perf_counter()
        self.t, self.arr = pool.take(off)
        t1 = __import__("time").perf_counter()
        dev = cols[0].device
        cur = torch.cuda.current_stream(dev)
        st = cur
        if copy_stream is not None:
            ready = torch.cuda.Event()
            ready.record(cur)
            copy_stream.wait_event(ready)
            st = copy_stream
        e = load().gpu_d2h_counted(self.t.data_ptr(), copies, n_dev.data_ptr(), st.cuda_stream,
                                   64 if copy_stream is not None else 1024)
        if e != 0:
            raise RuntimeError(f"gpu_d2h_counted failed (hipError {e})")
        self.ev = torch.cuda.Event()
        self.ev.record(st)
        self.done = self.ev
        # host seconds: slab take, the rest of the launch (phase timers of the callers)
        self.t_take, self.t_launch = t1 - t0, __import__("time").perf_counter() - t1

    def ready(self) -> bool:
        return self.ev.query()

    def wait(self) -> None:
        _event_spin(self.ev)

    def fixed(self, i: int) -> np.ndarray:
        off, nb, dt = self.fixed_meta[i]
        return self.arr[off:off + nb].view(_NP_DTYPE[dt])

    def columns(self, n: int) -> list[np.ndarray]:
        """The first n rows of every column (views of the slab); n is capped at the capacity."""
        n = min(n, self.cap)
        out = []
        for off, dt in self.cols_meta:
            es = torch.empty((), dtype=dt).element_size()
            out.append(self.arr[off:off + n * es].view(_NP_DTYPE[dt]))
        return out


_NP_DTYPE = {torch.int64: np.int64, torch.int32: np.int32, torch.float64: np.float64,
             torch.float32: np.float32, torch.uint8: np.uint8, torch.int16: np.int16,
             torch.bfloat16: np.uint16, torch.float16: np.float16}


# How the step's host sync waits for the GPU (MXS_SYNC, measured in profiles/r2_host_sync.md):
#   "query" (default): poll hipEventQuery on the step's event -- the host resumes within a
#     microsecond of the partition finishing, where a blocking wait (hipEventSynchronize /
#     hipStreamSynchronize) sleeps in the driver and wakes tens of microseconds late, time
#     the pipelined step cannot hide; "event": hipEventSynchronize; "stream":
#     hipStreamSynchronize (unpipelined only).
_SYNC = __import__("os").environ.get("MXS_SYNC", "query")


def _event_spin(ev) -> None:
    """Poll the event in C++ with the GIL released (csrc/bindings.cpp gpu_event_spin)."""
    from ..ops.native import load

    e = load().gpu_event_spin(ev.cuda_event)
    if e != 0:
        raise RuntimeError(f"hipEventQuery failed (hipError {e})")


def _host_wait(ev, device, pipelined: bool) -> None:
    if _SYNC == "query":
        _event_spin(ev)
    elif _SYNC == "event" or pipelined:
        ev.synchronize()
    else:
        torch.cuda.current_stream(device).synchronize()


def _next_pow2(x: int) -> int:
    return 1 << max(0, int(x - 1).bit_length())


def combine_partials(agg: int, acc: torch.Tensor, inv: torch.Tensor, n: int) -> torch.Tensor:
    """Fold rows of exported accumulators (int64 bit patterns) into n groups (`inv`: group of
    each row) with the aggregate's combine: sum / min / max over int64 or float64 values."""
    f64 = agg in (K.AGG_SUM_F64, K.AGG_AVG_F64, K.AGG_MIN_F64, K.AGG_MAX_F64)
    x = acc.view(torch.float64) if f64 else acc
    if agg in (K.AGG_MIN_I64, K.AGG_MIN_F64, K.AGG_MAX_I64, K.AGG_MAX_F64):
        is_min = agg in (K.AGG_MIN_I64, K.AGG_MIN_F64)
        init = (float("inf") if is_min else float("-inf")) if f64 else (I64_MAX if is_min else I64_MIN)
        out = torch.full((n,), init, dtype=x.dtype, device=x.device)
        out.scatter_reduce_(0, inv, x, "amin" if is_min else "amax")
    else:
        out = torch.zeros(n, dtype=x.dtype, device=x.device).index_add_(0, inv, x)
    return out.view(torch.int64) if f64 else out


@dataclass
class FireResult:
    window_start: int
    window_end: int
    keys: np.ndarray        # uint64 key ids (dictionary ids for string keys; uint32 ids for
                            # emit="key_value")
    values: np.ndarray      # float64 (result after the fused map epilogue)
    raw: np.ndarray | None  # int64 raw accumulator (exact integer sums / f64 bit pattern)
    counts: np.ndarray | None  # int32 element counts (raw / counts: None for emit="key_value")
    refire: bool = False
    seq: int = 0            # the operator's batch count when the firing was triggered (1-based
                            # process() call; latency accounting of deferred results)


@dataclass
class _PendingFire:
    """A firing whose rows are on their way to the host (CountedHostRows): stands in the output
    list at its place until resolved (KeyedWindowOperator._resolve)."""
    rows: "CountedHostRows"
    wins: list              # window starts of the group, in firing order
    kv: bool                # compact (key id, value) rows
    only_dirty: bool
    bounds: bool            # per-window cumulative counts in fixed(1); else the count is flags[2]
    seq: int = 0


@dataclass
class _Front:
    """One batch whose partition has been enqueued (S0) and whose reduced vector is on its way
    to pinned host memory."""
    keys: torch.Tensor
    ts: torch.Tensor
    vals: torch.Tensor
    n: int
    par: int
    old_wm: int
    pane_base: int
    proc_now: int
    rw: int = 3
    ev: object = None
    idle: bool = False


@dataclass
class _Back:
    """The state half of one step, planned on the host after its sync."""
    par: int
    n: int
    old_wm: int
    rw: int
    pane_base: int
    has_data: bool = False
    qmin: int = 0
    np_step: int = 0
    pg: int = 1
    gmin: int = 0
    gmax: int = -1
    fired_hi: int = I64_MIN
    new_wm: int | None = None
    ccap: int = 0
    hard: int = 0
    chk_ev: object = None
    chk_dev: object = None  # all-reduced combiner check on the device (AggPlan.skip)
    aplan: object = None    # the step's aggregation plan (redo after a combiner overflow)
    maxb: int = 0  # largest bucket fill of the step's partition (0: not reported)
    pmask: int = 0  # relative panes with records (GPU partition, one rank's own records)
    np_act: int = 0  # panes the aggregation visits (popcount(pmask), else np_step)
    seq: int = 0   # metrics.steps after this batch (FireResult.seq of what it fires)


@dataclass
class OperatorMetrics:
    num_records_in: int = 0
    num_late_records_dropped: int = 0
    num_records_out: int = 0
    num_fires: int = 0
    current_watermark: int = I64_MIN
    steps: int = 0
    bucket_regrows: int = 0
    ring_regrows: int = 0
    extra: dict = field(default_factory=dict)


class KeyedWindowOperator:
    """Per-rank keyed tumbling/sliding window aggregation on GPU (or the CPU twin)."""

    _geometry = None  # subclasses: (max_keys, cap_log2) -> (nsub, cap_log2)

    def __init__(self, *, size: int, slide: int | None = None, offset: int = 0,
                 lateness: int = 0, agg: int = K.AGG_SUM_I64, device="cpu",
                 comm: Comm | None = None, max_keys: int = 1 << 20,
                 parallelism: int | None = None, max_parallelism: int = 128,
                 hash_mode: int = 0, jhash_table: torch.Tensor | None = None,
                 map_prog: E.Program = E.EMPTY, filter_prog: E.Program = E.EMPTY,
                 batch_capacity: int = 1 << 20, bucket_slack: float = 1.5,
                 cap_log2: int | None = None, time_mode: str = "event", ooo_bound: int = 0,
                 side_output_late: bool = False, late_capacity: int = 1 << 16,
                 clock: Callable[[], int] | None = None, external_watermark: bool = False,
                 combine: bool | None = None, compact: bool | None = None,
                 narrow: bool | None = None, dense_keys: bool = False,
                 pipeline: bool | str | None = None, exchange: str = "auto",
                 idle_timeout_steps: int | None = None, deterministic: bool = False,
                 spill: bool = False, spill_load: float = 0.8, spill_check_steps: int = 8,
                 spill_keep_panes: int | None = None, emit: str = "full",
                 latency_fire: int = 0, window_keys: int | None = None):
        """deterministic: f64 sums/averages accumulate each step's per-slot sum in 128-bit fixed
        point (order-independent integer adds, one rounding per slot and step), so results are
        bit-identical between runs, between the GPU and the C++ twin, and independent of the
        number of virtual ranks' exchange order; values must satisfy |x| < 2^63 and are
        truncated to multiples of 2^-64. The sender-side combiner is off in
        this mode (raw records are exchanged). Integer aggregates are always exact.

        emit: "full" fired rows carry (key, mapped value, raw accumulator, count); "key_value"
        only (key id, mapped value) -- 12 bytes a row instead of 28 from the fire kernel to the
        host (dense keys; FireResult.raw / counts are None) for sinks that read nothing else.

        latency_fire = N > 0 (pipelined mode): a step whose watermark makes at most N windows due
        (first firings and late-data re-firings) runs its state half right away instead of one
        call later, and its firings are resolved before the call returns -- the alert leaves in
        the call of the batch that triggered it (one step of latency, not two or three), at the
        cost of that step's overlap with the next partition. Steps firing more windows (a
        watermark jump) keep the pipelined, batched path."""
        self.device = K.resolve_device(device)
        if emit not in ("full", "key_value"):
            raise ValueError("emit must be 'full' or 'key_value'")
        self.emit = emit
        self.latency_fire = max(0, int(latency_fire))
        self.deterministic = bool(deterministic) and agg in (K.AGG_SUM_F64, K.AGG_AVG_F64)
        # spill: host-DRAM tier for hashed keys (runtime/window_spill.py). Every
        # `spill_check_steps` steps, a sub-table above `spill_load` of its slots triggers
        # window_compact: keys without live data are dropped, keys whose newest data pane is
        # older than the newest `spill_keep_panes` panes (default: one window) move to the tier.
        self.comm = comm or LocalComm()
        self.world = self.comm.world
        self.rank = self.comm.rank
        slide = size if slide is None else slide
        if size <= 0 or slide <= 0:
            raise ValueError("window size and slide must be positive")
        self.size, self.slide, self.offset, self.lateness = int(size), int(slide), int(offset), int(lateness)
        # Window arithmetic and the firing / re-firing / purge bookkeeping: the C++ state machine
        # the C ABI pipeline runs too (csrc/window_control.h).
        from ..ops.native import load as _load_native

        self._ctl = _load_native().WindowControl(self.size, self.slide, self.offset, self.lateness)
        self.pane = self._ctl.pane
        self.panes_per_window = self._ctl.panes_per_window
        self.agg = agg
        self.time_mode = time_mode
        if time_mode not in ("event", "processing"):
            raise ValueError("time_mode must be 'event' or 'processing'")
        self.ooo_bound = int(ooo_bound)
        self.clock = clock
        # external_watermark: the caller drives time with advance_watermark() (DataStream API:
        # watermarks come from the upstream assigner); process() then never advances it.
        self.external_watermark = external_watermark
        # Idle source partitions (Flink StreamStatus IDLE, StatusWatermarkValve): a rank whose
        # source is idle -- marked with mark_idle(), or empty for `idle_timeout_steps`
        # consecutive batches -- sends +inf as its watermark, so the MIN over ranks is taken over
        # the active partitions only; if every partition is idle the watermark holds.
        self.idle_timeout_steps = idle_timeout_steps
        self._idle_marked = False
        self._empty_steps = 0
        self.parallelism = parallelism or self.world
        self.max_parallelism = max_parallelism
        self.hash_mode = hash_mode
        self.jhash = jhash_table
        self.map_prog, self.filter_prog = map_prog, filter_prog
        self.side_output_late = side_output_late
        self.metrics = OperatorMetrics()

        # ---- keyBy exchange strategy (G > 1) ----
        # "records": per step, every event (pre-aggregated per (key, pane) by the sender-side
        #   combiner) crosses the all-to-all to the key's owner, whose table holds its key share.
        # "partials" (local-global aggregation): per step, every rank folds its own events into a
        #   local table of the whole key space -- no per-event exchange; when a window fires, the
        #   local fire's rows (key, partial accumulator, count) cross ONE all-to-all to the owner,
        #   which merges them and evaluates the window (epilogue, filter, emit). Every aggregate
        #   here is associative, so the emitted rows are identical; the exchange shrinks from
        #   ~#distinct (key, pane) per step to #keys per window, and the per-step work of a rank
        #   is the G = 1 step. HBM (288 GB) holds the whole key space per rank many times over.
        #   With allowed lateness the owner keeps every fired window's merged value until its
        #   cleanup time, each rank accumulates its late-but-allowed data into a delta ring as
        #   well, and a re-firing ships only those deltas (every aggregate merges deltas exactly).
        if exchange not in ("auto", "records", "partials"):
            raise ValueError("exchange must be 'auto', 'records' or 'partials'")
        # Deterministic f64 sums keep records exchange: a rank's partial would be rounded to a
        # double before the merge, so the result would depend on G.
        lg_ok = self.world > 1 and self._local_global_ok and not self.deterministic
        if exchange == "partials" and self.world > 1 and not lg_ok:
            raise ValueError("exchange='partials' needs deterministic=False and a plain reduce")
        self.local_global = lg_ok and exchange != "records"
        self._exchanging = self.world > 1 and not self.local_global
        self._part_ranks = self.world if self._exchanging else 1

        # ---- state geometry ----
        from .geometry import state_geometry

        # Dense keys: ids < max_keys (dictionary ids of string keys) are directly addressed --
        # 2^bits slots, slot = id * mul mod 2^bits (a bijection), no hash-table probe, no LDS key
        # table. Needs one destination per event (G = 1 or local-global aggregation).
        self.dense_bits = self.dense_mul = 0
        if dense_keys:
            if self._exchanging or not self._dense_ok:
                raise ValueError("dense_keys needs one destination (G = 1 or exchange='partials')")
            bits = max(4, int(max_keys - 1).bit_length())
            if bits > 32:
                raise ValueError("dense_keys: ids must fit 32 bits")
            cl = min(12, bits) if cap_log2 is None else min(int(cap_log2), bits)
            # Small dense key spaces (a thousand channels) still get ~256 sub-tables: one
            # aggregation workgroup each, instead of 4 workgroups over the whole batch (>= 32
            # slots: the touched-slot bitmap of late data needs a word per 32).
            cl = min(cl, max(5, bits - 8))
            self.nsub, self.cap_log2 = 1 << (bits - cl), cl
            self.dense_bits = bits
            self.dense_mul = (0x9E3779B1 & ((1 << bits) - 1)) | 1
        else:
            self.nsub, self.cap_log2 = (self._geometry(max_keys, cap_log2) if self._geometry
                                        else state_geometry(max_keys, self._part_ranks, cap_log2))
        cap_log2 = self.cap_log2
        self.nsub_log2 = self.nsub.bit_length() - 1
        if self.nsub * self._part_ranks > 16384:
            raise ValueError("key space too large for the bucket histogram; raise cap_log2")
        self.nslots = self.nsub << cap_log2
        self.ring = max(4, _next_pow2(self.panes_per_window + 2 + math.ceil(self.lateness / self.pane)
                                     + math.ceil(max(self.ooo_bound, self.slide) / self.pane)))
        dev = self.device
        if self.dense_bits:
            # The key of every slot: the inverse bijection (slots are never "inserted").
            inv = pow(self.dense_mul, -1, 1 << self.dense_bits)
            self.keys_g = (torch.arange(self.nslots, dtype=torch.int64, device=dev) * inv) & \
                ((1 << self.dense_bits) - 1)
        else:
            self.keys_g = torch.full((self.nslots,), -1, dtype=torch.int64, device=dev)
        self.acc_g = torch.zeros(self.ring * self.nslots, dtype=torch.int64, device=dev)
        self.cnt_g = torch.zeros(self.ring * self.nslots, dtype=torch.int32, device=dev)
        self.dirty_g = torch.zeros(self.ring * self.nslots, dtype=torch.uint8, device=dev)
        # Local-global with allowed lateness: the delta ring of late-but-allowed data.
        self.dacc_g = self.dcnt_g = None
        if self.local_global and self.lateness > 0:
            self.dacc_g = torch.zeros(self.ring * self.nslots, dtype=torch.int64, device=dev)
            self.dcnt_g = torch.zeros(self.ring * self.nslots, dtype=torch.int32, device=dev)
        self.occ = torch.zeros(self.nsub, dtype=torch.int32, device=dev)
        self.flags = torch.zeros(4, dtype=torch.int32, device=dev)

        # ---- key group -> rank map (subtasks laid out in contiguous blocks over ranks) ----
        kgd = [self._rank_of_kg(kg) for kg in range(max_parallelism)]
        self.kg_dest = torch.tensor(kgd, dtype=torch.int32, device=dev)

        # ---- per-step buffers ----
        self.nbuckets = self._part_ranks << self.nsub_log2
        # G > 1: sender-side combiner before the all-to-all (all aggregates are associative).
        self.combine = (self._exchanging if combine is None
                        else bool(combine and self._exchanging)) and not self.deterministic
        # Pipelining: the partition of batch i+1 is enqueued before the state half of batch i
        # (process() then returns the windows fired by the previous batch; flush() drains).
        #   True:     the state half runs on a second stream, overlapping the partition (hides
        #             the per-step exchange at G > 1);
        #   "stream": one stream, deferred order  partition(i+1) | state half(i): the step's host
        #             sync waits on partition(i+1)'s reduced vector while the GPU still works on
        #             the state half of batch i, so the host's planning and launches never leave
        #             the GPU idle (no second stream: no HBM contention between the halves).
        # Opt-in: the engine's hot loops (bench, configs) enable it; callers that need each
        # batch's fires from its own call (DataStream API, external watermarks) keep the default.
        stream_mode = pipeline == "stream"
        self.pipeline = (bool(pipeline) and not external_watermark
                         and (stream_mode or not self.local_global))
        self.s1 = (torch.cuda.Stream(dev) if self.pipeline and not stream_mode
                   and self.device.type == "cuda" else None)
        self._par = 0
        self._pending: _Back | None = None
        self._carry: list[FireResult] = []  # fired by a flush a state reader forced
        nbuf = 2 if self.pipeline else 1
        self._ev_consumed: list = [None] * nbuf
        self._ev_part: list = [None] * nbuf
        self._alloc_buckets(batch_capacity, bucket_slack)
        self._stats = [K.new_stats(dev) for _ in range(nbuf)]
        self._red = [torch.zeros(K.RED_WORDS, dtype=torch.int64, device=dev) for _ in range(nbuf)]
        pin = self.device.type == "cuda"
        self._hred = [torch.zeros(K.RED_WORDS, dtype=torch.int64, pin_memory=pin)
                      for _ in range(nbuf)]
        self._hchk = torch.zeros(2, dtype=torch.int64, pin_memory=pin)
        self._hflags = torch.zeros(4, dtype=torch.int32, pin_memory=pin)
        self.stats, self.red = self._stats[0], self._red[0]
        self.local_maxts = torch.full((1,), I64_MIN, dtype=torch.int64, device=dev)
        if self.local_global:
            # window_keys: keys one window can hold over all ranks -- with the spill tier a window
            # holds keys evicted from the table, so the owners' merge tables are sized for more
            self._init_owner_tables(int(window_keys or (4 * max_keys if spill else max_keys)),
                                    cap_log2)
        # Batched firing: up to `_fire_group` due windows per native call and host sync (one
        # window's rows never exceed nslots, so the output holds the group's rows).
        self._fire_group = (max(1, min(64, (1 << 21) // self.nslots))
                            if type(self)._fire_window is KeyedWindowOperator._fire_window else 1)
        orows = self.nslots * self._fire_group
        if self.local_global:  # the owner's merge table fires into the same columns
            orows = max(orows, self.nslots_o)
        self.out_keys = torch.empty(orows, dtype=torch.int64, device=dev)
        self.out_vals = torch.empty(orows, dtype=torch.float64, device=dev)
        self.out_raw = torch.empty(orows, dtype=torch.int64, device=dev)
        self.out_cnt = torch.empty(orows, dtype=torch.int32, device=dev)
        # (>= 32 entries: a fused re-firing reports up to 32 windows' bounds)
        self.fire_bounds = torch.zeros((max(self._fire_group, 32) + 3) & ~3, dtype=torch.int32,
                                       device=dev)
        self._hbounds = torch.zeros(self._fire_group, dtype=torch.int32,
                                    pin_memory=dev.type == "cuda")
        # flags: [0] table full (bit0) / [1] combiner overflow / [2] fired-row cursor (out_n), so
        # one 16-byte D2H after a fire returns the row count and the table-full bit together.
        self.out_n = self.flags[2:3]
        # Pinned slabs for fired rows, allocated here: a first-fire pinned allocation of the
        # whole-table slab costs milliseconds of host time inside a step.
        self._pool = None
        # Firings copy their rows with a device-counted kernel and resolve later (no host sync
        # per firing); MXS_ASYNC_FIRE=0 restores the synchronous count -> copy path (A/B).
        self._async_fire = dev.type == "cuda" and _os.environ.get("MXS_ASYNC_FIRE", "1") != "0"
        # Fired-row copies run on a side stream, overlapping the next step's kernels; a firing
        # that reuses an output buffer first waits for the copy still reading it (_claim).
        self._copy_stream = (torch.cuda.Stream(dev) if self._async_fire
                             and _os.environ.get("MXS_COPY_STREAM", "1") != "0" else None)
        self._out_busy = None    # copy of out_* in flight (event)
        self._rout_busy = None   # copy of the re-firing rows in flight (event)
        self._rout = None        # re-firing output columns (keys, vals[, raw, cnt])
        if dev.type == "cuda":
            self._pool = PinnedSlabPool()
            self._pool.take(orows * 28 + 4 * 256)
        self.late_idx = (torch.empty(late_capacity, dtype=torch.int32, device=dev)
                         if side_output_late else None)
        # Touched-slot list (allowed lateness): window_agg appends every slot that receives
        # late-but-allowed data, re-firings visit only those slots (not the whole table).
        self.dlist = self.dlist_n = self.slot_mark = None
        if self.lateness > 0 and self._use_dlist:
            self.dlist = torch.empty(self.nslots, dtype=torch.int32, device=dev)
            self.dlist_n = torch.zeros(1, dtype=torch.int32, device=dev)
            self.slot_mark = torch.zeros(self.nslots, dtype=torch.int32, device=dev)
        self.comb_send = self.comb_recv = None
        self.comb_counts = torch.zeros(self.nbuckets, dtype=torch.int32, device=dev)
        self._ccap_hint = 1 << self.cap_log2
        self._unverified: _Back | None = None  # combined exchange whose check is unread
        # 16-byte records (int32 values) for integer aggregates on the GPU staged path; a value
        # outside int32 switches the operator to 24-byte records for good (step redone).
        int_agg = agg in (K.AGG_SUM_I64, K.AGG_MIN_I64, K.AGG_MAX_I64, K.AGG_COUNT, K.AGG_AVG_I64)
        if compact is None:
            compact = self.device.type == "cuda" and int_agg
        compact = bool(compact and int_agg)
        # 8-byte records (32-bit key id, 28-bit value, 4-bit pane) when one destination owns
        # every key (G = 1 or local-global) and the partition uses its LDS-sorted kernel; a
        # record that does not fit widens the format for good (step redone).
        if narrow is None:
            narrow = compact and self.device.type == "cuda"
        # The records exchange takes 8-byte records too when its buckets fit the compact
        # partition (<= 512 per rank): half the all-to-all and combiner read bytes of 16-byte
        # records. MXS_NARROW_EXCHANGE=0 keeps 16-byte records there (A/B).
        narrow_x = _os.environ.get("MXS_NARROW_EXCHANGE", "1") != "0"
        narrow = bool(narrow and compact and type(self)._narrow_ok
                      and (not self._exchanging
                           or (narrow_x and (self._part_ranks << self.nsub_log2) <= 512)))
        # Record words: 1 = 8-byte RecN, 2 = 16-byte RecC (int32 values), 3 = 24-byte Rec.
        self.rec_w = 1 if narrow else 2 if compact else 3
        self.timer = None  # utils.metrics.StageTimer: per-stage step_ms histograms when attached
        from ..ops.native import load as _load

        self._m = _load()
        self._pplan = self._aplan = None
        self._pplan_key = self._aplan_key = None
        from ..ops.debug import debug_enabled

        self._debug = debug_enabled()  # MXS_DEBUG: table invariant check after every step
        self.host_tier = None
        if spill:
            if self.dense_bits or not type(self)._spill_ok:
                raise ValueError("spill needs hashed keys and a plain reduce")
            if self.deterministic:
                # A tiered firing folds device and tier rows of a key with f64 atomics
                # (tier_merge), whose order varies between runs: the bit-identical promise of
                # deterministic=True cannot hold once a window has rows in the host tier.
                raise ValueError("deterministic=True does not combine with spill=True")
            from .window_spill import HostWindowTier

            self.host_tier = HostWindowTier(agg)
        self.spill_load, self.spill_check_steps = float(spill_load), max(1, int(spill_check_steps))
        self.spill_keep_panes = spill_keep_panes
        self._spill_out = None
        self._evict_pending = None   # asynchronous eviction rows on their way to host DRAM
        self._evict_busy = None      # event: the eviction copy stopped reading the device rows
        self._evict_pool = None
        self._tier_pool = None       # pinned slabs of the tier's rows for device-merged firings
        self._tier_h2d: list = []    # (event, slab) of tier rows still being copied H2D
        self._tier_tab = None        # the device-merged firing's combine table + outputs
        self._tout_busy = None

        # ---- watermark / firing bookkeeping (host, identical on every rank) ----
        self.wm = I64_MIN
        # next_fire_start / min_live_pane / max_seen_pane: properties over self._ctl (unset)
        self.late_side: list[np.ndarray] = []

    _local_global_ok = True  # subclasses whose fire is not a plain reduce opt out
    _spill_ok = True         # subclasses whose state is not (acc, cnt) per slot opt out
    _narrow_ok = True        # subclasses whose records carry more than (key, value) opt out
    _dense_ok = True         # subclasses with their own aggregation kernel opt out

    @property
    def compact(self) -> bool:
        """Records narrower than 24 bytes (integer values)."""
        return self.rec_w < 3
    _use_dlist = True        # subclasses with their own fire kernel opt out of slot lists

    def _init_owner_tables(self, max_keys: int, cap_log2: int | None) -> None:
        """Local-global mode: the owner side of a fire -- the merge table of this rank's key
        share (one pane: the window being fired) and the fire exchange buffers. A bucket
        (owner, owner sub-table) holds at most one row per key of that sub-table, so its
        capacity is the sub-table's: the fire exchange cannot overflow unless the owner's table
        is full (reported as such)."""
        from .geometry import state_geometry

        dev = self.device
        self.nsub_o, self.cap_log2_o = state_geometry(max_keys, self.world, cap_log2)
        self.nsub_o_log2 = self.nsub_o.bit_length() - 1
        if self.nsub_o * self.world > 16384:
            raise ValueError("key space too large for the fire exchange; raise cap_log2")
        nslots_o = self.nsub_o << self.cap_log2_o
        self.nslots_o = nslots_o
        # One merge slice per window that fired but is not cleaned yet (allowed lateness), so a
        # re-firing adds the ranks' deltas to the window's merged value.
        self.ring_m = _next_pow2(math.ceil(self.lateness / self.slide) + 2)
        self.keys_m = torch.full((nslots_o,), -1, dtype=torch.int64, device=dev)
        self.acc_m = torch.zeros(self.ring_m * nslots_o, dtype=torch.int64, device=dev)
        self.cnt_m = torch.zeros(self.ring_m * nslots_o, dtype=torch.int32, device=dev)
        self.dirty_m = torch.zeros(self.ring_m * nslots_o, dtype=torch.uint8, device=dev)
        self.occ_m = torch.zeros(self.nsub_o, dtype=torch.int32, device=dev)
        self.fbcap = 1 << self.cap_log2_o
        nbf = self.world << self.nsub_o_log2
        self.fsend = torch.empty(nbf * self.fbcap * K.REC_WORDS, dtype=torch.int64, device=dev)
        self.frecv = torch.empty_like(self.fsend)
        self.fcursor = torch.zeros(nbf, dtype=torch.int32, device=dev)
        self.frecv_counts = torch.zeros(nbf, dtype=torch.int32, device=dev)
        self.part_n = torch.zeros(1, dtype=torch.int32, device=dev)

    # ------------------------------------------------------------------------------------
    def _rank_of_kg(self, kg: int) -> int:
        sub = kg * self.parallelism // self.max_parallelism
        return sub * self.world // self.parallelism

    def _alloc_buckets(self, batch_capacity: int, slack: float) -> None:
        self._drain()
        self.batch_capacity = int(batch_capacity)
        self.bucket_slack = slack
        per = self.batch_capacity / self.nbuckets
        # The GPU partition pads every workgroup's run to whole 8-record groups (<= 7 holes per
        # bucket and workgroup, <= 1024 workgroups): capacity is a multiple of 8 with that slack.
        nblk = min(1024, max(1, -(-self.batch_capacity // 65536)))
        cap = int(per * slack + 6 * math.sqrt(max(per, 1.0)) + 64) + 8 * nblk
        self.bucket_cap = (cap + 7) & ~7
        words = self.nbuckets * self.bucket_cap * K.REC_WORDS
        dev = self.device
        # Pipelined: step i+1's partition writes the other send buffer while step i's combiner /
        # all-to-all / aggregation still read theirs (double buffering).
        nbuf = 2 if self.pipeline else 1
        self._send_bufs = [torch.empty(words, dtype=torch.int64, device=dev) for _ in range(nbuf)]
        self._cursor_bufs = [torch.zeros(self.nbuckets, dtype=torch.int32, device=dev)
                             for _ in range(nbuf)]
        # The plain exchange lands in `recv`; with the combiner only combined records travel.
        self.recv = (torch.empty(words, dtype=torch.int64, device=dev)
                     if self._exchanging and not self.combine else None)
        self._recv_counts = (torch.zeros(self.nbuckets, dtype=torch.int32, device=dev)
                             if self._exchanging else None)
        # Two-level GPU partition (8-byte records, one destination, > 512 buckets): the coarse
        # staging buffer and its 512 cursors (csrc partition_split_kernel).
        self._scratch = self._scratch_cursor = None
        if self._two_level_ok():
            self._scratch = torch.empty(self.nbuckets * self.bucket_cap, dtype=torch.int64,
                                        device=dev)
            self._scratch_cursor = torch.zeros(512, dtype=torch.int32, device=dev)
        self._pplan_key = None  # bucket capacity / scratch changed: rebuild the plan object
        self._use_par(0)

    def _two_level_ok(self) -> bool:
        return (self.device.type == "cuda" and self._part_ranks == 1
                and 512 < self.nbuckets <= 512 * 32
                and _os.environ.get("MXS_TWO_LEVEL", "1") != "0")

    def _use_par(self, p: int) -> None:
        """Point send/cursor (and, at G = 1, recv/recv_counts) at buffer set `p`."""
        self.send, self.cursor = self._send_bufs[p], self._cursor_bufs[p]
        if not self._exchanging:
            self.recv, self.recv_counts = self.send, self.cursor
        else:
            self.recv_counts = self._recv_counts

    # ---- streams / host sync helpers (GPU pipelining) ----------------------------------------
    def _s1(self):
        """Context running the state half of a step (combiner, all-to-all, aggregation, firing,
        purge) on the operator's state stream; the partition of the next step keeps the
        caller's stream (S0)."""
        import contextlib

        return torch.cuda.stream(self.s1) if self.s1 is not None else contextlib.nullcontext()

    def _drain(self) -> None:
        """Wait for every queued kernel of this operator (before buffers are reallocated)."""
        if self.device.type == "cuda" and getattr(self, "s1", None) is not None:
            self.s1.synchronize()
            torch.cuda.current_stream(self.device).synchronize()

    def _event(self):
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.device))
        return ev

    def _combine_begin(self, b: "_Back") -> None:
        """G > 1: pre-aggregate every send bucket to one record per (key, pane); the global
        overflow flag and largest fill go through one small MIN all-reduce into pinned memory
        (read in _combine_finish, while the next step's partition runs on S0)."""
        cap = 1 << self.cap_log2
        nb = self.nbuckets
        hard = min(self.bucket_cap, cap * b.np_step)  # distinct (key, pane) per bucket bound
        ccap = min(hard, max(64, (self._ccap_hint + 7) & ~7))
        if self.comb_send is None or self.comb_send.numel() < nb * ccap * K.REC_WORDS:
            self._drain()
            words = nb * ccap * K.REC_WORDS
            self.comb_send = torch.empty(words, dtype=torch.int64, device=self.device)
            self.comb_recv = torch.empty(words, dtype=torch.int64, device=self.device)
        self.flags[1:2].zero_()
        cplan = K.AggPlan(cap_log2=self.cap_log2, nsub=nb, ring=self.ring, agg=self.agg,
                          nsrc=1, bucket_cap=self.bucket_cap, np_step=b.np_step, pg=b.pg,
                          pane_base=0, p_lo=b.qmin, fired_hi=0,
                          rec_words=b.rw)
        K.window_combine(self.send, self.cursor, cplan, self.comb_send, ccap,
                         self.comb_counts, self.flags[1:2])
        chk = torch.stack([-(self.flags[1].to(torch.int64) & 2),
                           -self.comb_counts.max().to(torch.int64)])
        self.comm.allreduce_min_(chk)
        b.ccap, b.hard, b.chk_dev = ccap, hard, chk
        if self.device.type == "cuda":
            self._hchk.copy_(chk, non_blocking=True)
            b.chk_ev = self._event()
        else:
            self._hchk.copy_(chk)
            b.chk_ev = None

    def _combine_finish(self, b: "_Back"):
        """The all-to-all of the combined buckets, without waiting for the overflow check: the
        step's aggregation skips itself on the device when the all-reduced check reports an
        overflow (AggPlan.skip), and _verify_combine reads the check later -- at the step's first
        host sync that needs the state (a firing) or at the next entry point -- and redoes the
        exchange with larger buckets then (the send buffers are still intact)."""
        ccap, nb = b.ccap, self.nbuckets
        send = self.comb_send[: nb * ccap * K.REC_WORDS]
        recv = self.comb_recv[: nb * ccap * K.REC_WORDS]
        self.comm.all_to_all(recv, send)
        self.comm.all_to_all(self.recv_counts, self.comb_counts)
        self.metrics.extra["a2a_bytes"] = self.metrics.extra.get("a2a_bytes", 0) + send.numel() * 8
        return recv, self.recv_counts, ccap

    def _verify_combine(self) -> None:
        """Read the overflow check of the last combined exchange (see _combine_finish); on
        overflow (every rank sees the same all-reduced check) recombine the step's send buckets
        with twice the capacity, exchange again and aggregate. Called before anything reads or
        replaces the state."""
        b, self._unverified = self._unverified, None
        if b is None:
            return
        with self._s1():
            redo = False
            while True:
                if b.chk_ev is not None:
                    _host_wait(b.chk_ev, self.device, self.pipeline)
                ovf, fill = (-int(x) for x in self._hchk.tolist())
                if not ovf:
                    break
                if b.ccap >= b.hard:
                    raise RuntimeError("window_combine: a send bucket exceeds its sub-table capacity")
                self._ccap_hint = b.ccap * 2
                self.metrics.extra["combine_regrows"] = self.metrics.extra.get("combine_regrows", 0) + 1
                self._use_par(b.par)
                self._combine_begin(b)
                redo = True
            self._ccap_hint = max(64, int(fill * 1.25) + 8)
            if redo:
                recs, counts, bcap = self._combine_finish(b)
                b.aplan.bucket_cap, b.aplan.skip = bcap, 0
                self._aggregate(recs, counts, b.aplan)

    def _grow_ring(self, need: int) -> None:
        """Re-lay the pane ring so `need` consecutive panes fit (rare; keeps absolute pane ids)."""
        new_ring = _next_pow2(need)
        old = self.ring
        acc = torch.zeros(new_ring * self.nslots, dtype=torch.int64, device=self.device)
        cnt = torch.zeros(new_ring * self.nslots, dtype=torch.int32, device=self.device)
        dirty = torch.zeros(new_ring * self.nslots, dtype=torch.uint8, device=self.device)
        if self.min_live_pane is not None and self.max_seen_pane is not None:
            for p in range(self.min_live_pane, self.max_seen_pane + 1):
                so = (p & (old - 1)) * self.nslots
                sn = (p & (new_ring - 1)) * self.nslots
                acc[sn:sn + self.nslots].copy_(self.acc_g[so:so + self.nslots])
                cnt[sn:sn + self.nslots].copy_(self.cnt_g[so:so + self.nslots])
                dirty[sn:sn + self.nslots].copy_(self.dirty_g[so:so + self.nslots])
        if self.dacc_g is not None:
            dacc = torch.zeros(new_ring * self.nslots, dtype=torch.int64, device=self.device)
            dcnt = torch.zeros(new_ring * self.nslots, dtype=torch.int32, device=self.device)
            if self.min_live_pane is not None and self.max_seen_pane is not None:
                for p in range(self.min_live_pane, self.max_seen_pane + 1):
                    so = (p & (old - 1)) * self.nslots
                    sn = (p & (new_ring - 1)) * self.nslots
                    dacc[sn:sn + self.nslots].copy_(self.dacc_g[so:so + self.nslots])
                    dcnt[sn:sn + self.nslots].copy_(self.dcnt_g[so:so + self.nslots])
            self.dacc_g, self.dcnt_g = dacc, dcnt
        self.acc_g, self.cnt_g, self.dirty_g, self.ring = acc, cnt, dirty, new_ring
        self.metrics.ring_regrows += 1

    # ---- window arithmetic + bookkeeping (csrc/window_control.h) ---------------------------
    def pane_of(self, t: int) -> int:
        return self._ctl.pane_of(t)

    def pane_start(self, p: int) -> int:
        return self._ctl.pane_start(p)

    def last_start(self, t: int) -> int:
        return self._ctl.last_start(t)

    def first_start_containing(self, t: int) -> int:
        return self._ctl.first_start_containing(t)

    def _fired_hi(self) -> int:
        return self._ctl.fired_hi()

    @property
    def next_fire_start(self) -> int | None:
        """Smallest window start not yet evaluated (None: no data yet)."""
        return self._ctl.nfs() if self._ctl.has_nfs() else None

    @next_fire_start.setter
    def next_fire_start(self, v: int | None) -> None:
        self._ctl.set_nfs(v is not None, 0 if v is None else int(v))

    @property
    def min_live_pane(self) -> int | None:
        return self._ctl.min_live() if self._ctl.has_live() else None

    @min_live_pane.setter
    def min_live_pane(self, v: int | None) -> None:
        c = self._ctl
        if v is None:
            c.set_live(False, 0, 0)
        else:
            c.set_live(True, int(v), c.max_seen() if c.has_live() else int(v))

    @property
    def max_seen_pane(self) -> int | None:
        return self._ctl.max_seen() if self._ctl.has_live() else None

    @max_seen_pane.setter
    def max_seen_pane(self, v: int | None) -> None:
        c = self._ctl
        if v is None:
            c.set_live(False, 0, 0)
        else:
            c.set_live(True, c.min_live() if c.has_live() else int(v), int(v))

    # ---- main entry points ---------------------------------------------------------------
    def _pane_base(self, ts: torch.Tensor) -> int:
        """Base pane of the step, identical on every rank (records carry pane - base)."""
        if self.wm > I64_MIN:
            # Every non-late element has ts >= wm - size - lateness + 1.
            return self._ctl.pane_base_from_wm(self.wm)
        # No watermark yet: the global minimum timestamp (one MIN all-reduce, first steps only).
        t = ts.min().reshape(1) if ts.numel() else torch.full((1,), I64_MAX, dtype=torch.int64,
                                                                device=ts.device)
        self.comm.allreduce_min_(t)
        m = int(t.item())
        base = self.pane_of(m) if m != I64_MAX else 0
        if self.min_live_pane is not None:
            base = min(base, self.min_live_pane)
        return base

    def _late_ts(self, wm: int) -> int:
        """Smallest window start whose cleanup time (maxTs + lateness) is after `wm`."""
        return self._ctl.late_ts(wm, self.time_mode == "event")

    def current_processing_time(self) -> int:
        import time
        return int(self.clock() if self.clock else time.time() * 1000)

    def process(self, keys: torch.Tensor, ts: torch.Tensor, vals: torch.Tensor) -> list[FireResult]:
        """Fold one micro-batch of this rank's source partition and fire what the watermark allows.

        Unpipelined (CPU, DataStream API): partition -> one host sync -> aggregation -> fire, all
        for this batch. Pipelined (GPU default): the call enqueues this batch's partition on the
        caller's stream (S0) and the state half of the PREVIOUS batch (combiner, all-to-all,
        aggregation, firing, purge) on the state stream (S1), so the two overlap; it returns the
        windows fired by the previous batch (``flush()`` / ``finish()`` drain the last one). One
        host sync per step, on this batch's reduced vector, while S1 still works."""
        self._verify_combine()
        out, self._carry = self._carry, []
        if not self.pipeline:
            b = self._settle(self._front(keys, ts, vals))
            self._back_begin(b)
            return self._resolve(out + self._back_finish(b))
        prev, self._pending = self._pending, None
        if prev is not None:
            with self._s1():
                self._back_begin(prev)      # combiner + its tiny all-reduce, before S0's
        f = self._front(keys, ts, vals)     # partition of this batch (S0)
        if prev is not None:
            out += self._back_finish(prev)
        b = self._settle(f)                 # the step's one host sync (S1 keeps working)
        if self.latency_fire and 0 < self._due_windows(b) <= self.latency_fire:
            # Latency-bounded firing: this batch's firings leave in this call.
            with self._s1():
                self._back_begin(b)
            out += self._back_finish(b)
            self.metrics.extra["latency_fires"] = self.metrics.extra.get("latency_fires", 0) + 1
            return self._resolve(out, block=True)
        self._pending = b
        # Firings whose rows have reached the host are returned now; the others stay queued
        # (in order) for the next call -- the host never waits on a fire's copy here.
        return self._resolve(out, block=False)

    def _due_windows(self, b: "_Back") -> int:
        """Windows the state half of settled step `b` will fire or re-fire (host bookkeeping,
        an upper bound: windows without live panes are counted too)."""
        return self._ctl.due_count(bool(b.has_data), b.gmin if b.has_data else 0,
                                   b.gmax if b.has_data else 0, b.fired_hi,
                                   b.new_wm is not None, b.new_wm or 0)

    def flush(self) -> list[FireResult]:
        """Complete the pending state half of the last batch (pipelined mode); returns what it
        fired. Every entry point that reads or replaces state calls it first."""
        self._verify_combine()
        out, self._carry = self._carry, []
        prev, self._pending = self._pending, None
        if prev is None:
            return self._resolve(out)
        with self._s1():
            self._back_begin(prev)
        out += self._back_finish(prev)
        self._verify_combine()  # callers read or replace the state next
        return self._resolve(out)

    # ---- step phases ------------------------------------------------------------------------
    def _front(self, keys, ts, vals) -> "_Front":
        n = keys.numel()
        if n > self.batch_capacity:
            self.flush()
            self._alloc_buckets(n, self.bucket_slack)
        p = self._par
        if self.pipeline:
            self._par ^= 1
        event_mode = self.time_mode == "event"
        self._empty_steps = self._empty_steps + 1 if n == 0 else 0
        f = _Front(keys=keys, ts=ts, vals=vals, n=n, par=p, old_wm=self.wm, idle=self.idle,
                   pane_base=self._pane_base(ts),
                   proc_now=0 if event_mode else self.current_processing_time())
        self._launch_front(f)
        return f

    def mark_idle(self, idle: bool = True) -> None:
        """SourceContext.markAsTemporarilyIdle(): exclude this partition from the valve until it
        is marked active again (or sends data, with an idle timeout)."""
        self._idle_marked = bool(idle)

    @property
    def idle(self) -> bool:
        return self._idle_marked or (self.idle_timeout_steps is not None
                                     and self._empty_steps >= self.idle_timeout_steps)

    def _launch_front(self, f: "_Front") -> None:
        p = f.par
        self._use_par(p)
        cuda = self.device.type == "cuda"
        if cuda and self._ev_consumed[p] is not None:
            # send[p] / cursor[p] are still read by the state half of the step before last
            torch.cuda.current_stream(self.device).wait_event(self._ev_consumed[p])
        event_mode = self.time_mode == "event"
        stats, red = self._stats[p], self._red[p]
        f.rw = self.rec_w
        # Native plan object, rebuilt only when its structure changes; per step only the late
        # bound and the pane base move. One native call launches step_begin + partition +
        # step_finish (per-call dict parsing and argument checks cost ~100 us of host time per
        # step, which the pipelined step cannot always hide).
        # int32 key ids (the columnar sources' dictionary ids): read as they are by the compact
        # GPU partition (4 bytes less per event in both passes); widened for the other paths.
        key32 = f.keys.dtype == torch.int32
        two_level = self.rec_w == 1 and self._scratch is not None
        if key32 and cuda and not ((self.rec_w in (1, 2) and self.nbuckets <= 512 or two_level)
                                   and self.nbuckets * self.bucket_cap < (1 << 32)):
            f.keys = f.keys.to(torch.int64)
            key32 = False
        key = (self.bucket_cap, self.rec_w, int(event_mode), key32, two_level)
        if self._pplan_key != key:
            self._pplan = self._m.PartPlanObj(K.PartitionPlan(
                max_parallelism=self.max_parallelism, nsub_log2=self.nsub_log2,
                nranks=self._part_ranks, window_mode=1, drop_late=int(event_mode),
                hash_mode=self.hash_mode, bucket_cap=self.bucket_cap, pane=self.pane,
                rec_words=self.rec_w, dense_bits=self.dense_bits,
                dense_mul=self.dense_mul, key32=int(key32)).as_dict())
            if two_level:
                self._pplan.scratch = self._scratch.data_ptr()
                self._pplan.scratch_cursor = self._scratch_cursor.data_ptr()
            self._pplan_key = key
        pp = self._pplan
        pp.late_ts = self._late_ts(f.old_wm)
        pp.tbase = self.pane_start(f.pane_base)
        if f.n:
            for t, name in ((f.keys, "keys"), (f.ts, "ts"), (f.vals, "vals")):
                want = torch.int32 if t is f.keys and key32 else torch.int64
                if t.dtype != want or not t.is_contiguous() or t.numel() < f.n \
                        or t.device != self.device:
                    K._check(t, want, f.n, name, self.device)
            if f.n >= (1 << 32):
                raise ValueError("batch too large (2^32 events)")
        li = self.late_idx
        with self._stage("partition"):
            self._m.window_front(
                cuda, f.keys.data_ptr(), f.ts.data_ptr(), f.vals.data_ptr(),
                0 if self.jhash is None else self.jhash.data_ptr(), f.n, pp,
                self.kg_dest.data_ptr(), self.cursor.data_ptr(), self.send.data_ptr(),
                stats.data_ptr(), 0 if li is None else li.data_ptr(),
                0 if li is None else li.numel(), self.local_maxts.data_ptr(), self.ooo_bound,
                int(event_mode), f.proc_now, red.data_ptr(), self.flags.data_ptr(),
                torch.cuda.current_stream(self.device).cuda_stream if cuda else 0)
        if f.idle:
            red[2:3].fill_(I64_MAX)  # idle partition: no say in the MIN watermark
        # Watermark valve + pane range + every overflow flag: ONE MIN all-reduce per step.
        self.comm.allreduce_min_(red[:8])
        if cuda:
            self._hred[p].copy_(red, non_blocking=True)
            f.ev = self._event()
        else:
            self._hred[p].copy_(red)
            f.ev = None
        if cuda:
            self._ev_part[p] = f.ev

    def _settle(self, f: "_Front") -> "_Back":
        """The step's host sync: overflow handling (redo), watermark and pane bookkeeping."""
        while True:
            if f.ev is not None:
                _host_wait(f.ev, self.device, self.pipeline)
            host = self._hred[f.par].tolist()
            if host[4]:
                raise RuntimeError("event timestamp outside the representable pane range "
                                   "(more than 2^32 panes ahead of the watermark)")
            if host[6]:
                raise RuntimeError("keyed state table full: a key found no free slot "
                                   "(raise max_keys)")
            if host[7]:
                raise ValueError("key ids -1 and -2 are reserved (the state tables' markers)")
            need_rw = {1: 2, 2: 3}.get(-host[5], self.rec_w)
            if need_rw > self.rec_w:
                # A record does not fit the format: wider records from now on (2: a key or value
                # outside the 8-byte record, 3: a value outside int32).
                self.rec_w = need_rw
                self.metrics.extra["compact_fallbacks"] = self.metrics.extra.get("compact_fallbacks", 0) + 1
            elif host[3]:
                # A bucket overflowed somewhere: grow the fixed bucket capacity and redo the step.
                self.metrics.bucket_regrows += 1
                from ..utils.log import get_logger

                get_logger("runtime.window").warning(
                    "bucket capacity %d exceeded: regrowing and redoing the step", self.bucket_cap)
                self._alloc_buckets(self.batch_capacity, self.bucket_slack * 2)
            else:
                break
            self._drain()
            self._launch_front(f)
        qmax, qmin, wm_global = -host[0], host[1], host[2]
        if wm_global == I64_MAX:
            wm_global = f.old_wm  # every partition idle: the watermark holds
        st = host[8:]
        self.metrics.num_records_in += f.n
        self.metrics.num_late_records_dropped += int(st[K.STAT_LATE])
        if self.side_output_late and st[K.STAT_LATE]:
            nl = min(int(st[K.STAT_LATE]), self.late_idx.numel())
            self.late_side.append(self.late_idx[:nl].cpu().numpy().copy())
        b = _Back(par=f.par, n=f.n, old_wm=f.old_wm, rw=f.rw, pane_base=f.pane_base,
                  maxb=int(st[K.STAT_MAXBUCKET]), seq=self.metrics.steps + 1)
        if qmin <= qmax:
            gmin, gmax = f.pane_base + qmin, f.pane_base + qmax
            span = self._ctl.live_span_with(gmin, gmax)
            if span > self.ring:
                self._drain()
                self._grow_ring(span)
            # live range += [gmin, gmax]; the fire cursor moves back to the first not-yet-due
            # window holding new data (due windows receiving data re-fire: _refire)
            self._ctl.observe(gmin, gmax, f.old_wm)
            b.fired_hi = self._ctl.fired_hi()
            cap = 1 << self.cap_log2
            lds_budget = 150 * 1024 - cap * 8 - (cap * 4 + cap // 8 + 16
                                                 if self.dlist is not None else 0)
            b.has_data = True
            b.qmin, b.np_step = qmin, gmax - gmin + 1
            # Sparse pane rows: the aggregation visits only the panes that received records (a
            # late pane and the current ones, not the empty panes between them). Own records
            # only: the exchanged / combined paths keep the dense range.
            pm = int(st[7]) & 0xFFFFFFFF
            b.pmask = pm if (pm and not pm >> 31 and self.device.type == "cuda"
                             and not self._exchanging and not self.combine
                             and _os.environ.get("MXS_SPARSE_PANES", "1") != "0") else 0
            b.np_act = bin(b.pmask).count("1") if b.pmask else b.np_step
            if self.dense_bits:
                lds_budget += cap * 8  # no LDS key table for dense ids
            per_pane = 20 if self.deterministic else (8 if self._agg_pack_ok(b.rw) else 12)
            b.pg = max(1, min(b.np_act, lds_budget // (cap * per_pane)))
            b.gmin, b.gmax = gmin, gmax
        self.metrics.steps += 1
        if not self.external_watermark:
            b.new_wm = max(f.old_wm, wm_global)
            self.wm = b.new_wm
            self.metrics.current_watermark = b.new_wm
        return b

    def _back_begin(self, b: "_Back") -> None:
        if not b.has_data:
            return
        self._use_par(b.par)
        if self.device.type == "cuda" and self._ev_part[b.par] is not None:
            torch.cuda.current_stream(self.device).wait_event(self._ev_part[b.par])
        if self.combine:
            with self._stage("combine"):
                self._combine_begin(b)

    def _back_finish(self, b: "_Back") -> list[FireResult]:
        out: list[FireResult] = []
        cuda = self.device.type == "cuda"
        with self._s1():
            if b.has_data:
                self._use_par(b.par)
                recs, counts, bcap, combined = self.recv, self.recv_counts, self.bucket_cap, 0
                if self.combine:
                    with self._stage("all_to_all"):
                        recs, counts, bcap = self._combine_finish(b)
                    combined = 1
                elif self._exchanging:
                    with self._stage("all_to_all"):
                        self._exchange(b.rw)
                if cuda and self._exchanging:
                    self._ev_consumed[b.par] = self._event()
                sparse = bool(b.pmask) and not combined
                aplan = K.AggPlan(cap_log2=self.cap_log2, nsub=self.nsub, ring=self.ring,
                                  agg=self.agg, nsrc=self._part_ranks, bucket_cap=bcap,
                                  np_step=b.np_act if sparse else b.np_step, pg=b.pg,
                                  pane_base=b.pane_base,
                                  p_lo=b.qmin, fired_hi=b.fired_hi, combined=combined,
                                  rec_words=3 if combined else b.rw,
                                  pmask=b.pmask if sparse else 0)
                aplan.dense_bits, aplan.dense_mul = self.dense_bits, self.dense_mul
                aplan.det = int(self.deterministic)
                # Hot keys: a sub-table holding more than AGG_SLICE records is shared by several
                # workgroups (the launcher applies it where the atomic merge is exact).
                aplan.split = min(64, max(1, -(-b.maxb // K.AGG_SLICE))) if not combined else 1
                if self.dlist is not None:
                    aplan.dlist, aplan.dlist_n = self.dlist.data_ptr(), self.dlist_n.data_ptr()
                    aplan.slot_mark = self.slot_mark.data_ptr()
                if self.dacc_g is not None:
                    aplan.dacc, aplan.dcnt = self.dacc_g.data_ptr(), self.dcnt_g.data_ptr()
                if combined:
                    aplan.skip = b.chk_dev.data_ptr()
                with self._stage("window_agg"):
                    self._aggregate(recs, counts, aplan)
                if combined:
                    b.aplan, self._unverified = aplan, b
                if cuda and not self._exchanging:
                    self._ev_consumed[b.par] = self._event()
                if self._debug:
                    from ..ops.debug import assert_table_ok

                    assert_table_ok(self.keys_g, nsub=self.nsub, nsub_log2=self.nsub_log2,
                                    cap_log2=self.cap_log2, where=f"after step {self.metrics.steps}")
                # Late-but-allowed data: re-fire already-passed windows that are not cleaned yet.
                if b.gmin <= b.fired_hi:
                    # panes that can hold dirty bytes: this step's panes up to fired_hi
                    fr = b.fired_hi - b.pane_base
                    self._dirty_panes = ((b.pane_base, b.pmask & ((1 << (fr + 1)) - 1))
                                         if b.pmask and 0 <= fr < 31 else (0, 0))
                    out.extend(self._refire(b.gmin, min(b.gmax, b.fired_hi), b.old_wm))
                    self._dirty_panes = (0, 0)
            if b.new_wm is not None:
                with self._stage("fire"):
                    out.extend(self._fire_ready(b.new_wm))
                    self._purge(b.new_wm)
            if self.host_tier is not None and self.metrics.steps % self.spill_check_steps == 0:
                self._maybe_spill()
        if self.timer is not None:
            self.timer.flush()
        for r in out:
            r.seq = b.seq
        return out

    # ---- host-DRAM spill tier (runtime/window_spill.py) -----------------------------------
    def _maybe_spill(self) -> None:
        self._verify_combine()  # the occupancy must include a redone combined step's inserts
        cap = 1 << self.cap_log2
        occ = int(self.occ.max())
        # Compact above `spill_load`, or earlier when the fullest sub-table's growth since the
        # last check (twice over: checks are spill_check_steps apart) would fill it first --
        # small sub-tables (a few dozen slots) have little headroom above the load threshold.
        prev, self._occ_prev = getattr(self, "_occ_prev", None), occ
        growth = max(0, occ - prev) if prev is not None else 0
        if self.max_seen_pane is None or (occ <= self.spill_load * cap
                                          and occ + 2 * growth <= 0.95 * cap):
            return
        keep = self.spill_keep_panes or self.panes_per_window
        self.compact_state(self.max_seen_pane - keep, wait=False)
        self._occ_prev = None  # the compacted occupancy is not read back (asynchronous)

    def compact_state(self, cutoff_pane: int | None = None, wait: bool = True) -> dict:
        """Table maintenance at a step boundary: drop keys without live data and (with the spill
        tier) move keys whose newest data pane is <= cutoff_pane to host DRAM. Returns counts.

        wait=False (the spill check inside a step, GPU): the evicted rows go to a pinned slab by
        the counted copy kernel on the copy stream, with no host sync; the tier absorbs them at
        the next point that reads it (_land_evictions: a firing over tier panes, a purge, a
        snapshot, the next eviction) and the counts are returned as None."""
        self._verify_combine()  # a combined step skipped on the device is redone before this
        if self.dense_bits:
            return {"dropped": 0, "evicted": 0, "rows": 0}
        if cutoff_pane is not None and self.host_tier is None:
            raise ValueError("evicting keys needs the spill tier (spill=True)")
        self._land_evictions()
        self._drain()
        dev = self.device
        cuda = dev.type == "cuda"
        if self.min_live_pane is None:
            p_lo, np_ = 0, 0
        else:
            p_lo, np_ = self.min_live_pane, min(self.ring, self.max_seen_pane - self.min_live_pane + 1)
        cutoff = I64_MIN if cutoff_pane is None else int(cutoff_pane)
        asynchronous = cuda and not wait and self._copy_stream is not None and \
            self.host_tier is not None
        if cutoff == I64_MIN:
            rows_cap = 1
        elif asynchronous:
            # bound without a host read of the occupancy: every slot's live panes (x 16 rows)
            rows_cap = (self.nslots * max(np_, 1) + 15) & ~15
        else:
            rows_cap = max(1, int(self.occ.sum()) * max(np_, 1))
        o = self._spill_out
        if o is None or o["key"].numel() < rows_cap:
            o = self._spill_out = {
                "key": torch.empty(rows_cap, dtype=torch.int64, device=dev),
                "pane": torch.empty(rows_cap, dtype=torch.int64, device=dev),
                "acc": torch.empty(rows_cap, dtype=torch.int64, device=dev),
                "cnt": torch.empty(rows_cap, dtype=torch.int32, device=dev),
                "dirty": torch.empty(rows_cap, dtype=torch.uint8, device=dev),
                "ctr": torch.zeros(4, dtype=torch.int32, device=dev)}
        if asynchronous and self._evict_busy is not None:
            torch.cuda.current_stream(dev).wait_event(self._evict_busy)  # last copy read o[...]
            self._evict_busy = None
        o["ctr"].zero_()
        ptrs = [o["key"].data_ptr(), o["pane"].data_ptr(), o["acc"].data_ptr(),
                o["cnt"].data_ptr(), o["dirty"].data_ptr(), o["ctr"][3:4].data_ptr(),
                o["ctr"].data_ptr()]
        args = (self.keys_g.data_ptr(), self.acc_g.data_ptr(), self.cnt_g.data_ptr(),
                self.dirty_g.data_ptr(), self.nsub, self.cap_log2, self.ring, p_lo, np_, cutoff,
                ptrs, o["key"].numel(), self.occ.data_ptr())
        if cuda:
            self._m.gpu_window_compact(*args, torch.cuda.current_stream(dev).cuda_stream)
        else:
            self._m.cpu_window_compact(*args)
        if asynchronous:
            if self._evict_pool is None:
                self._evict_pool = PinnedSlabPool(max_slabs=2)
            n_cap = o["key"].numel()
            presorted = None
            if _EVICT_PANE_SORT and 0 < np_ <= 64:
                # Rows grouped by pane on the device: the tier takes them with memcpy instead
                # of a host counting sort (csrc/window_tier.h absorb_presorted).
                if "skey" not in o or o["skey"].numel() < n_cap:
                    o["skey"] = torch.empty(n_cap, dtype=torch.int64, device=dev)
                    o["sacc"] = torch.empty(n_cap, dtype=torch.int64, device=dev)
                    o["scnt"] = torch.empty(n_cap, dtype=torch.int32, device=dev)
                    o["sdirty"] = torch.empty(n_cap, dtype=torch.uint8, device=dev)
                    o["pcount"] = torch.zeros(128, dtype=torch.int32, device=dev)
                self._m.gpu_window_rows_pane_sort(
                    o["key"].data_ptr(), o["pane"].data_ptr(), o["acc"].data_ptr(),
                    o["cnt"].data_ptr(), o["dirty"].data_ptr(), o["ctr"][3:4].data_ptr(), n_cap,
                    p_lo, np_, o["skey"].data_ptr(), o["sacc"].data_ptr(), o["scnt"].data_ptr(),
                    o["sdirty"].data_ptr(), o["pcount"].data_ptr(),
                    torch.cuda.current_stream(dev).cuda_stream)
                cols = [o["skey"][:n_cap], o["sacc"][:n_cap], o["scnt"][:n_cap],
                        o["sdirty"][:n_cap]]
                fixed = [o["ctr"], o["pcount"]]
                presorted = (p_lo, np_)
            else:
                cols = [o["key"][:n_cap], o["pane"][:n_cap], o["acc"][:n_cap], o["cnt"][:n_cap],
                        o["dirty"][:n_cap]]
                fixed = [o["ctr"]]
            rows = CountedHostRows(self._evict_pool, cols, o["ctr"][3:4], fixed,
                                   copy_stream=self._copy_stream)
            rows.presorted = presorted
            self._evict_pending = rows
            self._evict_busy = rows.done
            self.metrics.extra["async_evictions"] = self.metrics.extra.get("async_evictions", 0) + 1
            return {"dropped": None, "evicted": None, "rows": None}
        return self._absorb_evicted(o["ctr"].tolist(), None, o)

    def _absorb_evicted(self, ctr, rows, o) -> dict:
        """Append evicted rows to the tier: from a landed asynchronous copy (`rows`) or, after a
        synchronous compaction, by one pinned copy of the device columns (`o`)."""
        if ctr[2]:
            raise RuntimeError("window_compact: eviction rows overflowed (internal error)")
        n = int(ctr[3])
        if n and self.host_tier is not None:
            if rows is not None and getattr(rows, "presorted", None):
                p_lo, np_ = rows.presorted
                counts = rows.fixed(1)[:np_]
                if int(counts.sum()) != n:
                    raise RuntimeError("window_rows_pane_sort: pane counts do not add up "
                                       "(internal error)")
                h = rows.columns(n)
                self.host_tier.absorb_presorted(h[0], h[1], h[2], h[3], p_lo, counts,
                                                background=_TIER_BG_ABSORB)
                h = None
            elif rows is not None:
                h = rows.columns(n)
            else:
                h = to_host_arrays([o["key"], o["pane"], o["acc"], o["cnt"], o["dirty"]], n,
                                   self._pool)
            if h is not None:
                self.host_tier.absorb(h[0].view(np.uint64), h[1], h[2], h[3], h[4])
        # (Touched-slot lists and dirty bytes are empty here: every step's re-firings cleared
        # them before this step boundary, so no slot id survives the rehash.)
        ex = self.metrics.extra
        ex["dropped_keys"] = ex.get("dropped_keys", 0) + int(ctr[0])
        ex["spilled_keys"] = ex.get("spilled_keys", 0) + int(ctr[1])
        ex["spilled_rows"] = ex.get("spilled_rows", 0) + n
        return {"dropped": int(ctr[0]), "evicted": int(ctr[1]), "rows": n}

    def _land_evictions(self) -> None:
        """Absorb an asynchronous eviction's rows into the tier (its copy has long completed when
        this runs: the next spill check, firing over tier panes or purge)."""
        rows, self._evict_pending = self._evict_pending, None
        if rows is None:
            return
        rows.wait()
        self._absorb_evicted(rows.fixed(0).tolist(), rows, None)

    # ---- hooks (overridden by the vector-metric operator) ---------------------------------
    def _exchange(self, rw: int) -> None:
        """G > 1 without the combiner: the equal-split all-to-all of the bucket ranges. The
        buckets are laid out in records of `rw` words (16-byte compact or 24-byte), so the
        per-rank chunks are nsub * bucket_cap records of that size: the prefix of the buffers."""
        words = self.nbuckets * self.bucket_cap * rw
        self.comm.all_to_all(self.recv[:words], self.send[:words])
        self.comm.all_to_all(self.recv_counts, self.cursor)

    def _aggregate(self, recs, counts, aplan: K.AggPlan) -> None:
        if aplan.np_step > aplan.ring:
            raise ValueError("step touches more panes than the ring holds")
        key = (aplan.bucket_cap, aplan.rec_words, aplan.ring, aplan.nsrc, aplan.combined,
               aplan.pg, aplan.dlist, aplan.det, aplan.dacc)
        if self._aplan_key != key:
            self._aplan = self._m.AggPlanObj(aplan.as_dict())
            self._aplan_key = key
        ap = self._aplan
        ap.np_step, ap.pane_base, ap.p_lo, ap.fired_hi = (aplan.np_step, aplan.pane_base,
                                                          aplan.p_lo, aplan.fired_hi)
        ap.split, ap.skip, ap.pmask = aplan.split, aplan.skip, aplan.pmask
        cuda = self.device.type == "cuda"
        self._m.window_agg_obj(cuda, recs.data_ptr(), counts.data_ptr(), ap,
                               self.keys_g.data_ptr(), self.acc_g.data_ptr(),
                               self.cnt_g.data_ptr(), self.dirty_g.data_ptr(),
                               self.occ.data_ptr(), self.flags.data_ptr(),
                               torch.cuda.current_stream(self.device).cuda_stream if cuda else 0)

    def _agg_pack_ok(self, rw: int) -> bool:
        """Mirror of the launcher's packed (sum, count) LDS accumulator condition (8 bytes per
        slot and pane instead of 12): integer sums of 8/16-byte own records, < 65536 records
        per sub-table."""
        return (self.agg in (K.AGG_SUM_I64, K.AGG_AVG_I64) and rw <= 2 and not self.combine
                and self._part_ranks * self.bucket_cap < 65536
                and _os.environ.get("MXS_AGG_PACK", "1") != "0")

    def _zero_pane(self, so: int, k: int = 1) -> None:
        """Reset k consecutive pane slabs starting at slot index `so` (pane-major state)."""
        e = so + k * self.nslots
        self.acc_g[so:e].zero_()
        self.cnt_g[so:e].zero_()
        self.dirty_g[so:e].zero_()

    def _stage(self, name: str):
        import contextlib

        return self.timer.stage(name) if self.timer is not None else contextlib.nullcontext()

    def advance_watermark(self, wm: int) -> list[FireResult]:
        """Advance the watermark without data (idle step / processing-time timer / end of input)."""
        wm = int(wm)
        out = self.flush()
        if wm <= self.wm:
            return out
        self.wm = wm
        self.metrics.current_watermark = wm
        with self._s1():
            fired = self._fire_ready(wm)
            self._purge(wm)
        for r in fired:
            r.seq = self.metrics.steps
        return out + self._resolve(fired)

    def finish(self) -> list[FireResult]:
        """End of input: event time emits Long.MAX_VALUE (fires everything); processing time does
        not fire pending windows (Flink 1.8 SocketTextStreamFunction end-of-stream behaviour)."""
        if self.time_mode == "event":
            return self.advance_watermark(I64_MAX)
        return self.flush()

    # ---- firing ---------------------------------------------------------------------------
    def _window_overlaps_live(self, s: int) -> bool:
        return self._ctl.overlaps_live(s)

    def _claim(self, which: str = "_out_busy") -> None:
        """Before a firing overwrites an output buffer: the current stream waits for the
        side-stream copy still reading it."""
        ev = getattr(self, which)
        if ev is not None:
            torch.cuda.current_stream(self.device).wait_event(ev)
            setattr(self, which, None)

    def _fire_window(self, s: int, only_dirty: bool) -> FireResult | None:
        # Only panes inside the live span exist in the ring; older/newer panes of the window
        # never held data and their ring slots belong to other panes (aliasing).
        if self.device.type == "cuda":
            self._claim()
        p0, p1 = self._ctl.window_panes(s)
        if p1 < p0:
            return None
        if self.local_global:
            return self._fire_window_partials(s, p0, p1, only_dirty)
        if self.host_tier is not None:
            self._land_evictions()
            if self.host_tier.overlaps(p0, p1):
                return self._fire_window_tiered(s, p0, p1, only_dirty)
        self.out_n.zero_()
        kv = self._key_value_rows()
        K.window_fire(self.keys_g, self.acc_g, self.cnt_g, self.dirty_g, agg=self.agg,
                      npanes=p1 - p0 + 1, ring=self.ring, p0=p0, wstart=s,
                      wend=s + self.size, only_dirty=only_dirty, map_prog=self.map_prog,
                      filt_prog=self.filter_prog, out_keys=self.out_keys, out_vals=self.out_vals,
                      out_raw=None if kv else self.out_raw, out_cnt=None if kv else self.out_cnt,
                      out_n=self.out_n, slot_list=self.dlist if only_dirty else None,
                      slot_list_n=self.dlist_n if only_dirty else None, key32=kv)
        self.metrics.num_fires += 1
        pend = self._fire_async([s], kv, only_dirty, bounds=False)
        if pend is not None:
            return pend
        n = self._fired_count()
        if n == 0:
            return None
        n = min(n, self.out_keys.numel())
        self.metrics.num_records_out += n
        host = self._rows_to_host(n, kv)
        return FireResult(s, s + self.size, host[0], host[1], host[2], host[3],
                          refire=only_dirty)

    def _fire_cols(self, kv: bool) -> list[torch.Tensor]:
        if kv:
            return [self.out_keys.view(torch.int32), self.out_vals]
        return [self.out_keys, self.out_vals, self.out_raw, self.out_cnt]

    def _fire_async(self, wins: list[int], kv: bool, only_dirty: bool,
                    bounds: bool) -> "_PendingFire | None":
        """The enqueued firing's rows -> pinned slab by the device-counted copy kernel, with the
        flags (and the group's bounds) alongside; no host sync. None: not available here (CPU,
        MXS_ASYNC_FIRE=0) -- the caller syncs as before."""
        if not self._async_fire:
            return None
        k = len(wins)
        n_dev = self.fire_bounds[k - 1:k] if bounds else self.out_n
        fixed = [self.flags, self.fire_bounds] if bounds else [self.flags]
        try:
            rows = CountedHostRows(self._pool, self._fire_cols(kv), n_dev, fixed,
                                   copy_stream=self._copy_stream)
        except ValueError:
            return None
        self._out_busy = rows.done
        return _PendingFire(rows, list(wins), kv, only_dirty, bounds)

    def _finish_pending(self, p: _PendingFire) -> list[FireResult]:
        """Rows of a resolved firing (its copy has completed) as FireResults, one per window."""
        hf = p.rows.fixed(0).tolist()
        n_single = self._check_fire_flags(hf)
        b = p.rows.fixed(1)[:len(p.wins)].tolist() if p.bounds else [n_single]
        n = min(b[-1], p.rows.cap)
        if n <= 0:
            return []
        self.metrics.num_records_out += n
        cols = p.rows.columns(n)
        keys = cols[0].view(np.uint32) if p.kv else cols[0].view(np.uint64)
        vals = cols[1]
        raw = None if p.kv else cols[2]
        cnt = None if p.kv else cols[3]
        out, lo = [], 0
        for s, hi in zip(p.wins, b):
            hi = min(hi, n)
            if hi > lo:
                out.append(FireResult(s, s + self.size, keys[lo:hi], vals[lo:hi],
                                      None if raw is None else raw[lo:hi],
                                      None if cnt is None else cnt[lo:hi],
                                      refire=p.only_dirty, seq=p.seq))
            lo = hi
        return out

    def _resolve(self, items: list, block: bool = True) -> list[FireResult]:
        """Replace pending firings by their rows, in order. block=False: stop at the first
        firing whose copy is still running and keep it and everything after it (in order) for
        the next call (self._carry)."""
        out = []
        for i, it in enumerate(items):
            if isinstance(it, _PendingFire):
                if not block and not it.rows.ready():
                    self._carry = items[i:] + self._carry
                    return out
                it.rows.wait()
                out.extend(self._finish_pending(it))
            else:
                out.append(it)
        return out

    def _key_value_rows(self) -> bool:
        """Compact fired rows (emit="key_value"): dense key ids fit 32 bits."""
        return self.emit == "key_value" and bool(self.dense_bits)

    def _rows_to_host(self, n: int, kv: bool) -> list:
        """First n fired rows as host arrays: keys (uint64, or uint32 ids for compact rows),
        values, raw, counts (None, None for compact rows)."""
        if kv:
            keys, vals = to_host_arrays([self.out_keys.view(torch.int32), self.out_vals], n,
                                        self._pool)
            return [keys.view(np.uint32), vals, None, None]
        host = to_host_arrays([self.out_keys, self.out_vals, self.out_raw, self.out_cnt], n,
                              self._pool)
        return [host[0].view(np.uint64), host[1], host[2], host[3]]

    def _fire_window_tiered(self, s: int, p0: int, p1: int, only_dirty: bool):
        """Window [s, s + size) with part of its state in the host tier, merged on the device:
        1. the device fires its rows of the window without the epilogue (key, raw accumulator,
           count; the count stays on the device);
        2. the tier's live rows of panes [p0, p1] are exported uncombined into a pinned slab
           (threaded C++) and copied H2D;
        3. tier_merge combines both per key into a transient table with atomics (a re-firing
           marks the device's dirty keys and folds tier rows of those keys only);
        4. window_fire over the table (one pane) with the fused map/filter epilogue: only the
           emitted rows leave the device, by the asynchronous counted copy of every firing.
        No host merge, no copy of the device's rows to the host."""
        from .window_spill import merge_fire

        dev = self.device
        cuda = dev.type == "cuda"
        m = self._m
        st = torch.cuda.current_stream(dev).cuda_stream if cuda else 0
        if cuda:
            self._claim()
        self.out_n.zero_()
        K.window_fire(self.keys_g, self.acc_g, self.cnt_g, self.dirty_g, agg=self.agg,
                      npanes=p1 - p0 + 1, ring=self.ring, p0=p0, wstart=s, wend=s + self.size,
                      only_dirty=only_dirty, map_prog=E.EMPTY, filt_prog=E.EMPTY,
                      out_keys=self.out_keys, out_vals=self.out_vals, out_raw=self.out_raw,
                      out_cnt=self.out_cnt, out_n=self.out_n,
                      slot_list=self.dlist if only_dirty else None,
                      slot_list_n=self.dlist_n if only_dirty else None)
        self.metrics.num_fires += 1
        if _TIER_MERGE == "host":  # A/B: the host merge (C++ radix-partitioned hash combine)
            n = min(self._fired_count(), self.out_keys.numel())
            dk, dr, dc = (t[:n].cpu().numpy() for t in (self.out_keys, self.out_raw, self.out_cnt))
            if only_dirty and n == 0:
                return None
            keys, vals, raw, cnt = merge_fire(self.agg, dk.view(np.uint64), dr, dc,
                                              self.host_tier, only_dirty, self.map_prog,
                                              self.filter_prog, s, s + self.size, panes=(p0, p1))
            if not keys.size:
                return None
            self.metrics.num_records_out += int(keys.size)
            return FireResult(s, s + self.size, keys, vals, raw, cnt, refire=only_dirty)
        # 2. the tier's rows of the window's panes (H2D on this stream)
        ex = self._tier_rows(p0, p1)
        # 3. per-key combine table of the device's rows (count on the device) + the tier's
        tkeys, tacc, tcnt, tdirty, ok_, ov_, or_, oc_ = self._tier_combine(
            ex, self.out_n, 1 if only_dirty else 0, 2 if only_dirty else 0)
        # 4. the fused epilogue over the combined table
        self.out_n.zero_()
        K.window_fire(tkeys, tacc, tcnt, tdirty, agg=self.agg, npanes=1, ring=1, p0=0,
                      wstart=s, wend=s + self.size, only_dirty=only_dirty,
                      map_prog=self.map_prog, filt_prog=self.filter_prog, out_keys=ok_,
                      out_vals=ov_, out_raw=or_, out_cnt=oc_, out_n=self.out_n)
        if cuda and self._async_fire:
            rows = CountedHostRows(self._pool, [ok_, ov_, or_, oc_], self.out_n, [self.flags],
                                   copy_stream=self._copy_stream)
            self._tout_busy = rows.done
            return _PendingFire(rows, [s], False, only_dirty, False)
        n = self._fired_count()
        if n == 0:
            return None
        n = min(n, ok_.numel())
        self.metrics.num_records_out += n
        host = to_host_arrays([ok_, ov_, or_, oc_], n, self._pool)
        return FireResult(s, s + self.size, host[0].view(np.uint64), host[1], host[2], host[3],
                          refire=only_dirty)

    def _tier_rows(self, p0: int, p1: int):
        """The tier's live rows of panes [p0, p1] on the device (window_spill.HostWindowTier
        .export; the pinned slab is held until its H2D copy has completed)."""
        dev = self.device
        cuda = dev.type == "cuda"
        for ev, _arr in self._tier_h2d:
            ev.synchronize()  # (long done: a previous firing's copy) -- the slab may be reused
        self._tier_h2d = []
        if self._tier_pool is None and cuda:
            self._tier_pool = PinnedSlabPool(max_slabs=2)
        ex = self.host_tier.export(p0, p1, dev, self._tier_pool)
        if cuda and ex is not None:
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(dev))
            self._tier_h2d.append((ev, ex[4]))
        return ex

    def _tier_combine(self, ex, n_dev, dev_mode: int, tier_mode: int):
        """tier_merge of the device rows in out_keys / out_raw / out_cnt (count n_dev on the
        device) and the tier rows `ex` into the transient combine table; returns the table and
        its output columns (keys, vals, raw, cnt), >= 2x the rows it can receive."""
        dev = self.device
        cuda = dev.type == "cuda"
        n_t = 0 if ex is None else ex[3]
        need = _next_pow2(max(1024, 2 * (self.out_keys.numel() + n_t)))
        tt = self._tier_tab
        if tt is None or tt[0].numel() < need:
            if cuda and self._tout_busy is not None:
                self._claim("_tout_busy")
            tt = self._tier_tab = (torch.empty(need, dtype=torch.int64, device=dev),
                                   torch.empty(need, dtype=torch.int64, device=dev),
                                   torch.empty(need, dtype=torch.int32, device=dev),
                                   torch.empty(need, dtype=torch.uint8, device=dev),
                                   torch.empty(need // 2, dtype=torch.int64, device=dev),
                                   torch.empty(need // 2, dtype=torch.float64, device=dev),
                                   torch.empty(need // 2, dtype=torch.int64, device=dev),
                                   torch.empty(need // 2, dtype=torch.int32, device=dev))
        tkeys, tacc, tcnt, tdirty = tt[:4]
        if cuda:
            self._claim("_tout_busy")  # the previous tiered firing's copy reads the outputs
        size = tkeys.numel()
        tkeys.fill_(-1)
        tacc.fill_(_agg_identity(self.agg))
        tcnt.zero_()
        tdirty.zero_()
        st = torch.cuda.current_stream(dev).cuda_stream if cuda else 0
        m = self._m
        m.tier_merge(cuda, self.out_keys.data_ptr(), self.out_raw.data_ptr(),
                     self.out_cnt.data_ptr(), self.out_keys.numel(), n_dev.data_ptr(), dev_mode,
                     self.agg, tkeys.data_ptr(), tacc.data_ptr(), tcnt.data_ptr(),
                     tdirty.data_ptr(), size - 1, self.flags.data_ptr(), st)
        if ex is not None:
            m.tier_merge(cuda, ex[0].data_ptr(), ex[1].data_ptr(), ex[2].data_ptr(), n_t, 0,
                         tier_mode, self.agg, tkeys.data_ptr(), tacc.data_ptr(),
                         tcnt.data_ptr(), tdirty.data_ptr(), size - 1, self.flags.data_ptr(), st)
        return tt

    def _merge_tier_partials(self, p0: int, p1: int):
        """Local-global with the spill tier: this rank's local partial rows of a window (count
        part_n) plus its tier rows of the window's panes, combined per key on the device and
        re-emitted as partial rows (no epilogue) -- the columns scatter_partials reads."""
        ex = self._tier_rows(p0, p1)
        tkeys, tacc, tcnt, tdirty, ok_, ov_, or_, oc_ = self._tier_combine(ex, self.part_n, 0, 0)
        self.part_n.zero_()
        K.window_fire(tkeys, tacc, tcnt, tdirty, agg=self.agg, npanes=1, ring=1, p0=0, wstart=0,
                      wend=self.size, only_dirty=False, map_prog=E.EMPTY, filt_prog=E.EMPTY,
                      out_keys=ok_, out_vals=ov_, out_raw=or_, out_cnt=oc_, out_n=self.part_n)
        return ok_, or_, oc_

    def _fire_window_partials(self, s: int, p0: int, p1: int, only_dirty: bool = False,
                              emit: bool = True) -> FireResult | None:
        """Local-global fire of window [s, s + size): local partials -> owner -> emit.

        1. local fire without epilogue: one row (key, partial acc, count) per local key with
           data in the window (all ranks, collectively identical decisions); a re-firing
           (allowed lateness) reads the delta ring of the late data instead, only the listed
           touched slots;
        2. scatter_partials: rows -> combined records in (owner rank, owner sub-table) buckets;
        3. ONE equal-split all-to-all of the buckets (+ their counts) over RCCL;
        4. the owner folds the G partials per key into the window's merge slice (window_agg,
           combined records; a first fire resets the slice, a re-firing adds the deltas to the
           merged value and marks the keys) and fires it with the fused map/filter epilogue
           (a re-firing: only the marked keys). The slice lives until the window is cleaned.
        The row count of step 1 stays on the device until the owner's fire is counted."""
        self.part_n.zero_()
        delta = only_dirty and self.dacc_g is not None
        K.window_fire(self.keys_g, self.dacc_g if delta else self.acc_g,
                      self.dcnt_g if delta else self.cnt_g, self.dirty_g, agg=self.agg,
                      npanes=p1 - p0 + 1, ring=self.ring, p0=p0, wstart=s, wend=s + self.size,
                      only_dirty=only_dirty, map_prog=E.EMPTY, filt_prog=E.EMPTY,
                      out_keys=self.out_keys, out_vals=self.out_vals, out_raw=self.out_raw,
                      out_cnt=self.out_cnt, out_n=self.part_n,
                      slot_list=self.dlist if only_dirty else None,
                      slot_list_n=self.dlist_n if only_dirty else None)
        pk, pa, pc = self.out_keys, self.out_raw, self.out_cnt
        if not delta and self.host_tier is not None:
            self._land_evictions()
            if self.host_tier.overlaps(p0, p1):
                # spilled keys: this rank's tier rows of the window join its local partials
                pk, pa, pc = self._merge_tier_partials(p0, p1)
        self.fcursor.zero_()
        K.scatter_partials(pk, pa, pc, self.part_n,
                           n_cap=pk.numel(), max_parallelism=self.max_parallelism,
                           nranks=self.world, nsub_log2=self.nsub_o_log2,
                           hash_mode=self.hash_mode, jhash=self.jhash, kg_dest=self.kg_dest,
                           bucket_cap=self.fbcap, cursor=self.fcursor, out=self.fsend,
                           flags=self.flags)
        with self._stage("all_to_all"):
            self.comm.all_to_all(self.frecv, self.fsend)
            self.comm.all_to_all(self.frecv_counts, self.fcursor)
        self.metrics.extra["a2a_bytes"] = self.metrics.extra.get("a2a_bytes", 0) + \
            self.fsend.numel() * 8
        widx = (s - self.offset) // self.slide
        so = (widx & (self.ring_m - 1)) * self.nslots_o
        if not only_dirty:  # the slice's previous window is cleaned: reuse it
            self.acc_m[so:so + self.nslots_o].zero_()
            self.cnt_m[so:so + self.nslots_o].zero_()
            self.dirty_m[so:so + self.nslots_o].zero_()
        mplan = K.AggPlan(cap_log2=self.cap_log2_o, nsub=self.nsub_o, ring=self.ring_m,
                          agg=self.agg, nsrc=self.world, bucket_cap=self.fbcap, np_step=1, pg=1,
                          pane_base=widx, p_lo=0, fired_hi=widx if only_dirty else I64_MIN,
                          combined=1, rec_words=3, det=int(self.deterministic))
        K.window_agg(self.frecv, self.frecv_counts, mplan, self.keys_m, self.acc_m, self.cnt_m,
                     self.dirty_m, self.occ_m, self.flags)
        if not emit:  # restore: rebuild the merged value of an already fired window
            return None
        self.out_n.zero_()
        K.window_fire(self.keys_m, self.acc_m, self.cnt_m, self.dirty_m, agg=self.agg, npanes=1,
                      ring=self.ring_m, p0=widx, wstart=s, wend=s + self.size,
                      only_dirty=only_dirty, map_prog=self.map_prog, filt_prog=self.filter_prog,
                      out_keys=self.out_keys, out_vals=self.out_vals, out_raw=self.out_raw,
                      out_cnt=self.out_cnt, out_n=self.out_n)
        if only_dirty:
            self.dirty_m[so:so + self.nslots_o].zero_()
        n = self._fired_count()
        self._maybe_compact_merge()
        self.metrics.num_fires += 1
        if n == 0:
            return None
        n = min(n, self.out_keys.numel())
        self.metrics.num_records_out += n
        host = to_host_arrays([self.out_keys, self.out_vals, self.out_raw, self.out_cnt], n,
                              self._pool)
        return FireResult(s, s + self.size, host[0].view(np.uint64), host[1], host[2], host[3],
                          refire=only_dirty)

    def _maybe_compact_merge(self) -> None:
        """The owner's merge table keeps a key while any merge slice (a fired window inside its
        allowed lateness) holds a value for it. Keys whose slices were all recycled are dead;
        with a drifting key space they would fill the table, so every 16 partial fires the
        fullest sub-table is checked (the fire has just synchronised) and, above 0.6 load, the
        live keys are rehashed into a cleared table with their slices."""
        self._mfires = getattr(self, "_mfires", 0) + 1
        if self._mfires % 16 or int(self.occ_m.max()) <= 0.6 * (1 << self.cap_log2_o):
            return
        R, N = self.ring_m, self.nslots_o
        cnt = self.cnt_m.view(R, N)
        live = torch.nonzero(((cnt != 0).any(0)) & (self.keys_m != -1)
                             & (self.keys_m != -2)).flatten()
        keys = self.keys_m[live]
        acc = self.acc_m.view(R, N)[:, live]
        cnt_l = cnt[:, live]
        dirty = self.dirty_m.view(R, N)[:, live]
        self.keys_m.fill_(-1)
        self.acc_m.zero_()
        self.cnt_m.zero_()
        self.dirty_m.zero_()
        self.occ_m.zero_()
        if live.numel():
            slots = K.table_insert(keys.contiguous(), self.keys_m, nsub_log2=self.nsub_o_log2,
                                   cap_log2=self.cap_log2_o)
            if bool((slots < 0).any()):
                raise RuntimeError("merge table compaction: live keys do not fit")
            self.acc_m.view(R, N)[:, slots] = acc
            self.cnt_m.view(R, N)[:, slots] = cnt_l
            self.dirty_m.view(R, N)[:, slots] = dirty
            self.occ_m.copy_(torch.bincount(slots >> self.cap_log2_o, minlength=self.nsub_o)
                             .to(torch.int32))
        self.metrics.extra["merge_compactions"] = self.metrics.extra.get("merge_compactions", 0) + 1

    def _fired_count(self) -> int:
        """Rows the last fire produced; raises if any aggregation found its table full (a key
        without a slot would otherwise be missing from the fired windows)."""
        if self.device.type == "cuda":
            self._hflags.copy_(self.flags, non_blocking=True)
            torch.cuda.current_stream(self.device).synchronize()
            hf = self._hflags.tolist()
        else:
            hf = self.flags.tolist()
        return self._check_fire_flags(hf)

    def _fired_bounds(self, k: int) -> list[int]:
        """Cumulative row counts of a batched firing's k windows (one host sync)."""
        if self.device.type == "cuda":
            self._hflags.copy_(self.flags, non_blocking=True)
            self._hbounds[:k].copy_(self.fire_bounds[:k], non_blocking=True)
            torch.cuda.current_stream(self.device).synchronize()
            hf = self._hflags.tolist()
            b = self._hbounds[:k].tolist()
        else:
            hf = self.flags.tolist()
            b = self.fire_bounds[:k].tolist()
        self._check_fire_flags(hf)
        return b

    def _check_fire_flags(self, hf) -> int:
        if hf[0] & 1:
            raise RuntimeError("keyed state table full: a key found no free slot (raise max_keys)")
        if hf[0] & 8:
            raise ValueError("deterministic f64 sum: a value is NaN, infinite or |x| >= 2^63")
        return hf[2]

    def _batched_fire_ok(self) -> bool:
        return (not self.local_global and self.host_tier is None
                and type(self)._fire_window is KeyedWindowOperator._fire_window)

    def _fire_list(self, starts: list[int], only_dirty: bool) -> list[FireResult]:
        """Fire the windows starting at `starts` (in order)."""
        if starts:
            self._verify_combine()
        if len(starts) > 1 and self._batched_fire_ok():
            return self._fire_many(starts, only_dirty)
        out = []
        for s in starts:
            r = self._fire_window(s, only_dirty)
            if r is not None:
                out.append(r)
        return out

    def _fire_many(self, starts: list[int], only_dirty: bool) -> list:
        """Batched firing: a group of due windows is evaluated by one native call (one fire
        launch per window, rows appended at a shared cursor, the cursor recorded after each
        window), then ONE host sync and ONE copy to the pinned slab for the whole group -- a
        watermark jump over many slides (5 min / 5 s windows: 60 per element) no longer costs two
        host round trips per window."""
        out: list[FireResult] = []
        cuda = self.device.type == "cuda"
        kv = self._key_value_rows()
        plan = dict(agg=self.agg, npanes=1, ring=self.ring, only_dirty=int(only_dirty),
                    nslots=self.nslots, p0=0, wstart=0.0, wend=0.0, out_cap=self.out_keys.numel(),
                    map=tuple(self.map_prog.as_args()), filt=tuple(self.filter_prog.as_args()),
                    key32=int(kv))
        if only_dirty and self.dlist is not None:
            plan.update(list=self.dlist.data_ptr(), list_n=self.dlist_n.data_ptr())
        wins = []
        for s in starts:
            p0, p1 = self._ctl.window_panes(s)
            if p1 >= p0:
                wins.append((s, (p0, p1 - p0 + 1, float(s), float(s + self.size))))
        stream = torch.cuda.current_stream(self.device).cuda_stream if cuda else 0
        if cuda and only_dirty and self.dlist is not None and 1 < len(wins) <= 32 \
                and _os.environ.get("MXS_FUSED_REFIRE", "1") != "0":
            res = self._refire_fused(wins, kv, plan, stream)
            if res is not None:
                return res
        if cuda:
            self._claim()
        stage = self._fire_stage(kv) if cuda else None
        g = self._fire_group
        for i in range(0, len(wins), g):
            chunk = wins[i:i + g]
            if cuda:
                self._claim()  # the previous chunk's copy may still read out_*
            else:
                self.out_n.zero_()
            self._m.window_fire_many(cuda, self.keys_g.data_ptr(), self.acc_g.data_ptr(),
                                     self.cnt_g.data_ptr(), self.dirty_g.data_ptr(), plan,
                                     [w for _, w in chunk], self.out_keys.data_ptr(),
                                     self.out_vals.data_ptr(),
                                     0 if kv else self.out_raw.data_ptr(),
                                     0 if kv else self.out_cnt.data_ptr(), self.out_n.data_ptr(),
                                     self.fire_bounds.data_ptr(), stream, stage)
            self.metrics.num_fires += len(chunk)
            pend = self._fire_async([s for s, _ in chunk], kv, only_dirty, bounds=True) \
                if cuda else None
            if pend is not None:
                out.append(pend)
                continue
            bounds = self._fired_bounds(len(chunk))
            n = min(bounds[-1], self.out_keys.numel())
            if n == 0:
                continue
            self.metrics.num_records_out += n
            host = self._rows_to_host(n, kv)
            lo = 0
            for (s, _), hi in zip(chunk, bounds):
                hi = min(hi, n)
                if hi > lo:
                    out.append(FireResult(s, s + self.size, host[0][lo:hi], host[1][lo:hi],
                                          None if kv else host[2][lo:hi],
                                          None if kv else host[3][lo:hi], refire=only_dirty))
                lo = hi
        return out

    def _refire_fused(self, wins: list, kv: bool, plan: dict, stream: int) -> list | None:
        """Every re-fired window of the step in ONE pass over the touched-slot list
        (gpu_window_refire_many: each listed slot's union of panes is loaded once), packed in
        window order into the re-firing's own output columns and copied on the side stream;
        resolved later (no wait here). The touched-slot count is read first (one small wait on
        the aggregation): each window's staging region is sized to it, so no window can
        outgrow its region. None: not fusable here."""
        k = len(wins)
        n_list = int(self.dlist_n[0])  # host wait: the step's aggregation has run
        if n_list == 0:
            self.metrics.num_fires += k
            return []
        region = (n_list + 3) & ~3
        rows_cap = k * region
        self._claim("_rout_busy")  # the previous re-firing's copy reads the staging / columns
        r = self._rout
        if r is None or r[0].numel() < rows_cap or (r[2] is None) != kv:
            cap = max(rows_cap, 1 << 16)
            dev = self.device
            r = self._rout = (torch.empty(cap, dtype=torch.int64, device=dev),
                              torch.empty(cap, dtype=torch.float64, device=dev),
                              None if kv else torch.empty(cap, dtype=torch.int64, device=dev),
                              None if kv else torch.empty(cap, dtype=torch.int32, device=dev),
                              torch.empty(cap, dtype=torch.int64, device=dev),
                              torch.empty(cap, dtype=torch.float64, device=dev),
                              None if kv else torch.empty(cap, dtype=torch.int64, device=dev),
                              None if kv else torch.empty(cap, dtype=torch.int32, device=dev),
                              torch.zeros(32, dtype=torch.int32, device=dev),
                              torch.zeros(36, dtype=torch.int32, device=dev))
        st_keys, st_vals, st_raw, st_cnt, o_keys, o_vals, o_raw, o_cnt, win_n, bnd = r
        stage = (st_keys.data_ptr(), st_vals.data_ptr(), 0 if kv else st_raw.data_ptr(),
                 0 if kv else st_cnt.data_ptr(), win_n.data_ptr(), region)
        self.flags[3:4].zero_()
        ok = self._m.gpu_window_refire_many(
            self.keys_g.data_ptr(), self.acc_g.data_ptr(), self.cnt_g.data_ptr(),
            self.dirty_g.data_ptr(), plan, [w for _, w in wins], o_keys.data_ptr(),
            o_vals.data_ptr(), 0 if kv else o_raw.data_ptr(), 0 if kv else o_cnt.data_ptr(),
            bnd[32:33].data_ptr(), bnd.data_ptr(), self.flags[3:4].data_ptr(), stream, stage,
            *getattr(self, "_dirty_panes", (0, 0)))
        if not ok:
            return None
        cols = [o_keys.view(torch.int32), o_vals] if kv else [o_keys, o_vals, o_raw, o_cnt]
        rows = CountedHostRows(self._pool, [c[:rows_cap] for c in cols], bnd[k - 1:k],
                               [self.flags, bnd], copy_stream=self._copy_stream)
        self._rout_busy = rows.done
        self.metrics.num_fires += k
        return [_PendingFire(rows, [s for s, _ in wins], kv, True, True)]

    def _fire_stage(self, kv: bool = False) -> tuple:
        """Per-window staging regions of the GPU batched firing (window_fire_many: window w of
        a group writes rows [w * nslots, (w + 1) * nslots) at its own counter, a pack kernel
        then lays the group out in window order into out_*). Allocated on first use; sized like
        out_* (nslots x fire group)."""
        st = getattr(self, "_stage_cols", None)
        if st is None or st[0].numel() != self.out_keys.numel():
            n, dev = self.out_keys.numel(), self.out_keys.device
            st = (torch.empty(n, dtype=torch.int64, device=dev),
                  torch.empty(n, dtype=torch.float64, device=dev),
                  torch.empty(n, dtype=torch.int64, device=dev),
                  torch.empty(n, dtype=torch.int32, device=dev),
                  torch.empty(max(self._fire_group, 32), dtype=torch.int32, device=dev))
            self._stage_cols = st
        ptrs = [t.data_ptr() for t in st]
        if kv:  # compact rows: no raw / count columns
            ptrs[2] = ptrs[3] = 0
        return tuple(ptrs) + (self.nslots,)

    def _fire_ready(self, wm: int) -> list[FireResult]:
        """Fire every window the watermark makes due (the cursor moves past them)."""
        return self._fire_list(self._ctl.take_due(wm), only_dirty=False)

    def _align_up(self, t: int) -> int:
        """Smallest window start >= t."""
        return self._ctl.align_up(t)

    def _refire(self, pmin: int, pmax: int, old_wm: int) -> list[FireResult]:
        self._verify_combine()
        out: list[FireResult] = []
        out.extend(self._fire_list(self._ctl.refire_windows(pmin, pmax, old_wm), only_dirty=True))
        if self.dlist is not None:
            K.dirty_clear(self.dlist, self.dlist_n, ring=self.ring, nslots=self.nslots,
                          dirty_g=self.dirty_g, slot_mark=self.slot_mark, p_lo=pmin,
                          np_=pmax - pmin + 1, dacc=self.dacc_g, dcnt=self.dcnt_g)
            self.dlist_n.zero_()
        else:
            for p in range(pmin, pmax + 1):
                so = (p & (self.ring - 1)) * self.nslots
                self.dirty_g[so:so + self.nslots].zero_()
        return out

    def _purge(self, wm: int) -> None:
        if self.min_live_pane is None:
            return
        # keep_from: first pane of the earliest window not cleaned (s + size - 1 + lateness > wm);
        # panes [p, stop) are zeroed (at most one ring of them)
        keep_from, p, stop = self._ctl.purge_range(wm, self.ring)
        if self.host_tier is not None:
            self._land_evictions()
            self.host_tier.purge(keep_from)
        if p < stop:
            self._verify_combine()  # a redo must not land in a zeroed pane
        while p < stop:  # at most two runs of consecutive ring positions (wrap-around)
            r = p & (self.ring - 1)
            k = min(stop - p, self.ring - r)
            self._zero_pane(r * self.nslots, k)
            p += k
        self._ctl.commit_purge(keep_from)

    # ---- introspection ---------------------------------------------------------------------
    def state_bytes(self) -> int:
        return sum(t.numel() * t.element_size() for t in (self.keys_g, self.acc_g, self.cnt_g,
                                                          self.dirty_g))

    def host_state_bytes(self) -> int:
        """Bytes of keyed state in the host-DRAM tier (0 without spill)."""
        if self.host_tier is None:
            return 0
        self._land_evictions()
        return self.host_tier.nbytes

    def num_keys(self) -> int:
        self._sync_state()
        if self.dense_bits:  # no insertion: keys with data in a live pane
            return int((self.cnt_g.view(self.ring, self.nslots) > 0).any(0).sum().item())
        return int(self.occ.sum().item())

    def _sync_state(self) -> None:
        """Make the state tables current for a host reader: the pending step must be applied
        (its fired rows are kept for the next process()/flush() caller) and S1 drained."""
        if self._pending is not None:
            self._carry.extend(self.flush())
        self._drain()
        self._land_evictions()  # evicted rows still in flight belong to the tier's state

    # ---- checkpoint / restore (runtime/checkpoint.py) --------------------------------------
    def owned_key_groups(self) -> tuple[int, int]:
        from .checkpoint import owned_key_groups

        return owned_key_groups(self.rank, self.world, self.parallelism, self.max_parallelism)

    def _check_ckpt_meta(self, meta: dict) -> None:
        for k in ("size", "slide", "offset", "agg", "time_mode"):
            if meta[k] != getattr(self, k):
                raise ValueError(f"checkpoint {k}={meta[k]!r} does not match operator "
                                 f"{getattr(self, k)!r}")

    _state_tensors = ("keys_g", "acc_g", "cnt_g", "dirty_g")

    def snapshot_state_async(self):
        """Freeze the state now (D2D copies), export it later: see checkpoint.freeze_operator."""
        from .checkpoint import freeze_operator

        self._sync_state()

        def private_tier(frozen):
            # The export reads the spill tier from a worker thread while the step loop keeps
            # absorbing / purging the live one: the frozen copy gets its own tier as of now, so
            # keys evicted after the freeze are neither lost nor exported twice.
            if self.host_tier is not None:
                frozen.host_tier = self.host_tier.copy()

        return freeze_operator(self, self._state_tensors, post=private_tier)

    def snapshot_state(self):
        """Live (key, pane) accumulators grouped by key group, plus the firing bookkeeping."""
        from .checkpoint import OperatorSnapshot

        self._sync_state()
        live = torch.nonzero(self.keys_g != -1).flatten()
        cols = {"key": np.zeros(0, np.int64), "pane": np.zeros(0, np.int64),
                "acc": np.zeros(0, np.int64), "cnt": np.zeros(0, np.int32),
                "dirty": np.zeros(0, np.uint8)}
        kg = np.zeros(0, np.int32)
        if self.min_live_pane is not None and live.numel():
            panes = torch.arange(self.min_live_pane, self.max_seen_pane + 1, device=self.device)
            idx = ((panes & (self.ring - 1)) * self.nslots)[:, None] + live[None, :]
            cnt = self.cnt_g[idx]
            sel = cnt > 0
            keys = self.keys_g[live][None, :].expand_as(idx)[sel].contiguous()
            kg = K.keygroups(keys, max_parallelism=self.max_parallelism, hash_mode=self.hash_mode,
                             jhash=self.jhash).cpu().numpy()
            cols = {"key": keys.cpu().numpy(),
                    "pane": panes[:, None].expand_as(idx)[sel].cpu().numpy(),
                    "acc": self.acc_g[idx][sel].cpu().numpy(),
                    "cnt": cnt[sel].cpu().numpy(),
                    "dirty": self.dirty_g[idx][sel].cpu().numpy()}
        if self.host_tier is not None and self.host_tier.nrows:
            # Spilled state travels in the same rows (restore folds duplicate (key, pane) rows).
            h = self.host_tier.rows()
            hk = torch.from_numpy(h["key"].view(np.int64))
            kg = np.concatenate([kg, K.keygroups(hk, max_parallelism=self.max_parallelism,
                                                 hash_mode=self.hash_mode,
                                                 jhash=None if self.jhash is None else self.jhash.cpu()
                                                 ).numpy()]).astype(np.int32)
            cols = {"key": np.concatenate([cols["key"], h["key"].view(np.int64)]),
                    "pane": np.concatenate([cols["pane"], h["pane"]]),
                    "acc": np.concatenate([cols["acc"], h["acc"]]),
                    "cnt": np.concatenate([cols["cnt"], h["cnt"].astype(np.int32)]),
                    "dirty": np.concatenate([cols["dirty"], h["dirty"]])}
        meta = {"kind": "window", "size": self.size, "slide": self.slide, "offset": self.offset,
                "lateness": self.lateness, "agg": self.agg, "time_mode": self.time_mode,
                "wm": self.wm, "next_fire_start": self.next_fire_start,
                "min_live_pane": self.min_live_pane, "max_seen_pane": self.max_seen_pane,
                "metrics": {"num_records_in": self.metrics.num_records_in,
                            "num_late_records_dropped": self.metrics.num_late_records_dropped,
                            "num_records_out": self.metrics.num_records_out,
                            "num_fires": self.metrics.num_fires, "steps": self.metrics.steps}}
        return OperatorSnapshot(kg, cols, meta)

    def restore_state(self, rows: dict, meta: dict) -> None:
        """Rebuild the tables from checkpoint rows (this rank's key groups only)."""
        self._check_ckpt_meta(meta)
        if self.host_tier is not None:
            self._evict_pending = None  # rows of the replaced state
            self.host_tier.clear()
        self._pending, self._carry = None, []
        self._drain()
        dev = self.device
        self.wm = meta["wm"]
        self.metrics.current_watermark = self.wm
        self.next_fire_start = meta["next_fire_start"]
        self.min_live_pane, self.max_seen_pane = meta["min_live_pane"], meta["max_seen_pane"]
        for k, v in meta.get("metrics", {}).items():
            setattr(self.metrics, k, v)
        if self.min_live_pane is not None and self.max_seen_pane - self.min_live_pane + 1 > self.ring:
            self.ring = _next_pow2(self.max_seen_pane - self.min_live_pane + 1)
            self.acc_g = torch.zeros(self.ring * self.nslots, dtype=torch.int64, device=dev)
            self.cnt_g = torch.zeros(self.ring * self.nslots, dtype=torch.int32, device=dev)
            self.dirty_g = torch.zeros(self.ring * self.nslots, dtype=torch.uint8, device=dev)
        if not self.dense_bits:
            self.keys_g.fill_(-1)
        if self.dlist is not None:
            self.dlist_n.zero_()
            self.slot_mark.zero_()
        self.acc_g.zero_()
        self.cnt_g.zero_()
        self.dirty_g.zero_()
        self.occ.zero_()
        if self.local_global and self.lateness > 0:
            self.dacc_g = torch.zeros(self.ring * self.nslots, dtype=torch.int64, device=dev)
            self.dcnt_g = torch.zeros(self.ring * self.nslots, dtype=torch.int32, device=dev)
        if not len(rows["key"]):
            if self.local_global:
                self._rebuild_merge_ring()
            return
        keys = torch.from_numpy(np.ascontiguousarray(rows["key"])).to(dev)
        pane = torch.from_numpy(np.ascontiguousarray(rows["pane"])).to(dev)
        acc = torch.from_numpy(np.ascontiguousarray(rows["acc"])).to(dev)
        cnt = torch.from_numpy(np.ascontiguousarray(rows["cnt"])).to(dev)
        dirty = torch.from_numpy(np.ascontiguousarray(rows["dirty"])).to(dev)
        uniq, inv = torch.unique(keys, return_inverse=True)
        occ_slots = None
        if self.dense_bits:
            if bool((uniq >> self.dense_bits).any()):
                raise RuntimeError("restore: key id outside the dense key space (raise max_keys)")
            slots_u = (uniq * self.dense_mul) & ((1 << self.dense_bits) - 1)
        elif self.host_tier is not None:
            # With the spill tier the checkpoint may hold more keys than the table: keys without
            # data in the newest spill_keep_panes panes go back to the tier (as compact_state
            # would have put them), the others are inserted; any that find no slot join the tier.
            to_tier = torch.zeros(uniq.numel(), dtype=torch.bool, device=dev)
            if self.max_seen_pane is not None:
                newest = torch.full((uniq.numel(),), I64_MIN, dtype=torch.int64, device=dev)
                newest.scatter_reduce_(0, inv, pane, "amax")
                keep = self.spill_keep_panes or self.panes_per_window
                to_tier = newest <= self.max_seen_pane - keep
            slots_u = torch.full((uniq.numel(),), -1, dtype=torch.int64, device=dev)
            hot = torch.nonzero(~to_tier).flatten()
            if hot.numel():
                slots_u[hot] = K.table_insert(uniq[hot].contiguous(), self.keys_g,
                                              nsub_log2=self.nsub_log2, cap_log2=self.cap_log2)
            row_tier = (slots_u < 0)[inv]
            occ_slots = slots_u[slots_u >= 0]
            if bool(row_tier.any()):
                sel = torch.nonzero(row_tier).flatten()
                self.host_tier.absorb(keys[sel].cpu().numpy().view(np.uint64),
                                      pane[sel].cpu().numpy(), acc[sel].cpu().numpy(),
                                      cnt[sel].cpu().numpy(), dirty[sel].cpu().numpy())
                sel = torch.nonzero(~row_tier).flatten()
                keys, pane, acc, cnt, dirty = keys[sel], pane[sel], acc[sel], cnt[sel], dirty[sel]
                inv = inv[sel]
                slots_u = torch.where(slots_u < 0, torch.zeros_like(slots_u), slots_u)
        else:
            slots_u = K.table_insert(uniq.contiguous(), self.keys_g, nsub_log2=self.nsub_log2,
                                     cap_log2=self.cap_log2)
        if bool((slots_u < 0).any()):
            raise RuntimeError("restore: keyed state does not fit the table (raise max_keys)")
        slot = slots_u[inv]
        idx = (pane & (self.ring - 1)) * self.nslots + slot
        u, inv = torch.unique(idx, return_inverse=True)
        if u.numel() == idx.numel():
            self.acc_g[idx], self.cnt_g[idx], self.dirty_g[idx] = acc, cnt, dirty
        else:
            # Several rows per (key, pane): partial accumulators of a local-global checkpoint
            # (every rank held a partial of every key) -- fold them with the aggregate.
            self.acc_g[u] = combine_partials(self.agg, acc, inv, u.numel())
            self.cnt_g[u] = torch.zeros(u.numel(), dtype=torch.int32, device=dev).index_add_(
                0, inv, cnt)
            self.dirty_g[u] = torch.zeros(u.numel(), dtype=torch.int32, device=dev).scatter_reduce_(
                0, inv, dirty.to(torch.int32), "amax").to(torch.uint8)
        if self.dlist is not None:
            # Rebuild the touched-slot list from the restored dirty bytes.
            self.slot_mark.zero_()
            ds = torch.unique(slot[dirty != 0]).to(torch.int32)
            self.dlist[:ds.numel()] = ds
            self.dlist_n.fill_(ds.numel())
            self.slot_mark[ds.long()] = 1
        occ_slots = slots_u if occ_slots is None else occ_slots
        self.occ.copy_(torch.bincount(occ_slots >> self.cap_log2, minlength=self.nsub)
                       .to(torch.int32))
        if self.local_global:
            self._rebuild_merge_ring()

    def _rebuild_merge_ring(self) -> None:
        """Local-global with allowed lateness, after a restore: the owners' merged values of the
        windows that fired but are not cleaned (a late re-firing adds deltas to them) are
        recomputed from the restored state -- the same collective exchange as a fire, without
        the emit. Every rank runs the same window sequence (identical restored bookkeeping)."""
        self.keys_m.fill_(-1)
        self.acc_m.zero_()
        self.cnt_m.zero_()
        self.dirty_m.zero_()
        self.occ_m.zero_()
        if (self.lateness <= 0 or self.next_fire_start is None or self.min_live_pane is None
                or self.wm == I64_MIN):
            return
        s = max(self._align_up(self.wm - self.size - self.lateness + 2),
                self.first_start_containing(self.pane_start(self.min_live_pane)))
        while s < self.next_fire_start:
            p0 = max(self.pane_of(s), self.min_live_pane)
            p1 = min(self.pane_of(s) + self.panes_per_window - 1, self.max_seen_pane)
            if p1 >= p0:
                self._fire_window_partials(s, p0, p1, only_dirty=False, emit=False)
            s += self.slide
