"""Keyed window operator: keyBy shuffle + pane-ring window state + watermark-driven firing.

One instance runs per rank (one process per GPU). The whole micro-batch loop is native -- ONE C++
implementation (``csrc/window_step.h`` WindowStep) that the C ABI pipeline (``csrc/pipeline.cpp``)
runs too; this class converts arguments, forwards the multi-rank collectives to the rank's
process group, and wraps the fired rows. Per micro-batch (``process``), inside one native call
with the GIL released:

 1. ``partition`` kernel: key group -> destination rank (Flink's
    ``murmur(hash) % maxParallelism * P / maxParallelism``), sub-table, pane id, late drop —
    records land in fixed-capacity (dest, sub-table) buckets;
 2. one MIN all-reduce of [-max pane, min pane, local watermark, overflow flags] (the watermark
    valve) and, for the records exchange, the all-to-all of the bucket ranges; ONE host sync;
 3. ``window_agg`` kernel: one workgroup per LDS-resident sub-table folds the step's records into
    the pane ring (pane = gcd(size, slide); a sliding window is a run of panes);
 4. late-but-allowed data re-fires the touched windows; the advanced watermark fires every window
    with ``end - 1 <= wm`` (fused map/filter epilogue), rows copied to pinned slabs on a side
    stream and resolved later;
 5. panes whose every window passed its cleanup time (``maxTs + allowedLateness <= wm``) are
    zeroed for reuse; with ``spill`` cold keys move to the host-DRAM tier.

Flink semantics reproduced (reference: ``BandwidthMonitorWithEventTime.java:30-55``,
``BandwidthMonitor.java:32-40``, ``ComputeCpuAvg.java:27-59``):
window assignment, lateness test, per-key emission only for windows that hold data, watermark =
min over source partitions of (max ts - bound), processing-time windows never fire at end of
input. Micro-batch deviation (documented): several late elements of one (key, window) in the same
micro-batch produce one re-firing carrying their combined effect (Flink fires once per element).
"""
from __future__ import annotations

import time
from typing import Callable

import numpy as np
import torch

from ..ops import expr as E
from ..ops import kernels as K
from ..parallel.comm import Comm, LocalComm
# Names other modules import from here.
from .host_rows import (CountedHostRows, PinnedSlabPool, _event_spin, _host_wait,  # noqa: F401
                        _next_pow2, to_host_arrays)
from .window_state import _StateMixin
from .window_types import FireResult, OperatorMetrics  # noqa: F401

I64_MIN = K.I64_MIN
I64_MAX = K.I64_MAX

_DTYPES = {"i8": torch.int64, "i4": torch.int32, "u1": torch.uint8}


class _StepCommAdapter:
    """The native step's collectives over the rank's comm (torch.distributed: RCCL over xGMI or
    gloo; a LoopbackComm of virtual ranks). Buffers are the step's own memory, wrapped as
    non-owning tensors; the collective runs on the step's stream."""

    def __init__(self, comm: Comm, device: torch.device):
        self.comm, self.device = comm, device
        self._views: dict = {}

    def _t(self, ptr: int, n: int, code: str) -> torch.Tensor:
        key = (ptr, n, code)
        t = self._views.get(key)
        if t is None:
            from ..ops.native import load

            cuda = self.device.type == "cuda"
            t = torch.from_dlpack(load().dl_view(ptr, n, code, cuda, self.device.index or 0))
            self._views[key] = t
        return t

    def _stream(self, stream: int):
        import contextlib

        if self.device.type != "cuda":
            return contextlib.nullcontext()
        if stream == 0:
            # The step runs on the legacy default stream (torch's default stream hands out
            # handle 0). ExternalStream(0) is NOT that stream here: torch maps a null handle to
            # some other stream, and the collective raced the step's kernels (loopback ranks
            # read each other's vectors before step_finish had written them).
            return torch.cuda.stream(torch.cuda.default_stream(self.device))
        return torch.cuda.stream(torch.cuda.ExternalStream(stream, device=self.device))

    def allreduce_min(self, ptr: int, n: int, stream: int) -> None:
        with self._stream(stream):
            self.comm.allreduce_min_(self._t(ptr, n, "i8"))

    def all_to_all(self, recv: int, send: int, nbytes: int, elem: int, stream: int) -> None:
        code = {8: "i8", 4: "i4"}.get(elem, "u1")
        n = nbytes // {8: 8, 4: 4}.get(elem, 1)
        with self._stream(stream):
            self.comm.all_to_all(self._t(recv, n, code), self._t(send, n, code))


def _state_prop(name: str) -> property:
    """A state buffer of the native step as a tensor (settable on a frozen snapshot copy)."""
    return property(lambda self: self._view(name), lambda self, t: self._set_view(name, t))


class _Metrics:
    """OperatorMetrics view of the native step's counters (Flink names; `extra`: the engine's
    own counters). Assignment writes through (restore)."""

    __slots__ = ("_s",)
    _FIELDS = ("num_records_in", "num_late_records_dropped", "num_records_out", "num_fires",
               "current_watermark", "steps", "bucket_regrows", "ring_regrows")

    def __init__(self, step):
        object.__setattr__(self, "_s", step)

    def __getattr__(self, k):
        if k.startswith("__"):
            raise AttributeError(k)
        d = self._s.metrics()
        if k in d:
            return d[k]
        raise AttributeError(k)

    def __setattr__(self, k, v):
        self._s.set_metric(k, int(v))

    def __copy__(self) -> OperatorMetrics:  # a frozen copy (checkpoint.freeze_operator)
        return self.snapshot()

    def snapshot(self) -> OperatorMetrics:
        d = self._s.metrics()
        return OperatorMetrics(**{k: d[k] for k in self._FIELDS}, extra=dict(d["extra"]))


class KeyedWindowOperator(_StateMixin):
    """Per-rank keyed tumbling/sliding window aggregation on GPU (or the CPU twin)."""

    _dim = 0  # vector windows (runtime/vector_window_operator.py): metrics per event

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
                 latency_fire: int = 0, window_keys: int | None = None, _vector: dict | None = None):
        """deterministic: f64 sums/averages accumulate each step's per-slot sum in 128-bit fixed
        point (order-independent integer adds, one rounding per slot and step), so results are
        bit-identical between runs, between the GPU and the C++ twin, and independent of the
        number of virtual ranks' exchange order; values must satisfy |x| < 2^63 and are
        truncated to multiples of 2^-64. Integer aggregates are always exact.

        exchange (G > 1): "partials" = local-global aggregation (every rank folds its own events
        into a table of the whole key space; when a window fires, the local fire's rows cross ONE
        all-to-all to the key's owner, which merges and emits them); "records" = every step's
        records (pre-aggregated per (key, pane) by the sender-side combiner) cross the all-to-all
        to the key's owner; "auto" = partials where the aggregate allows.

        pipeline: "stream" = the partition of batch i+1 is enqueued before the state half of
        batch i on one stream (process() then returns the windows fired by earlier batches;
        flush() drains); True = the state half on a second stream; None / False = off.

        emit: "full" fired rows carry (key, mapped value, raw accumulator, count); "key_value"
        only (key id, mapped value) -- 12 bytes a row instead of 28 from the fire kernel to the
        host (dense keys; FireResult.raw / counts are None).

        latency_fire = N > 0 (pipelined): a step whose watermark makes at most N windows due runs
        its state half right away and its firings leave in the same call.

        spill: host-DRAM tier for hashed keys. Every `spill_check_steps` steps, a sub-table above
        `spill_load` of its slots triggers window_compact: keys without live data are dropped,
        keys whose newest data pane is older than the newest `spill_keep_panes` panes (default:
        one window) move to the tier."""
        if emit not in ("full", "key_value"):
            raise ValueError("emit must be 'full' or 'key_value'")
        if time_mode not in ("event", "processing"):
            raise ValueError("time_mode must be 'event' or 'processing'")
        if exchange not in ("auto", "records", "partials"):
            raise ValueError("exchange must be 'auto', 'records' or 'partials'")
        slide = size if slide is None else slide
        if size <= 0 or slide <= 0:
            raise ValueError("window size and slide must be positive")
        self.device = K.resolve_device(device)
        self.comm = comm or LocalComm()
        self.world, self.rank = self.comm.world, self.comm.rank
        self.size, self.slide, self.offset, self.lateness = int(size), int(slide), int(offset), int(lateness)
        self.agg, self.time_mode, self.ooo_bound = agg, time_mode, int(ooo_bound)
        self.clock = clock
        self.external_watermark = external_watermark
        self.idle_timeout_steps = idle_timeout_steps
        self.parallelism = parallelism or self.world
        self.max_parallelism, self.hash_mode = max_parallelism, hash_mode
        self._jhash = jhash_table
        self.map_prog, self.filter_prog = map_prog, filter_prog
        self.side_output_late, self.emit = side_output_late, emit
        self.latency_fire = max(0, int(latency_fire))
        self.deterministic = bool(deterministic) and agg in (K.AGG_SUM_F64, K.AGG_AVG_F64)
        self.spill_keep_panes = spill_keep_panes
        vec = _vector or {}
        cuda = self.device.type == "cuda"
        cfg = dict(
            size=self.size, slide=self.slide, offset=self.offset, lateness=self.lateness, agg=agg,
            gpu=cuda, device_index=self.device.index or 0, parallelism=self.parallelism,
            max_parallelism=max_parallelism, hash_mode=hash_mode,
            jhash=0 if jhash_table is None else jhash_table.data_ptr(),
            map=tuple(map_prog.as_args()), filt=tuple(filter_prog.as_args()),
            max_keys=int(max_keys), batch_capacity=int(batch_capacity),
            bucket_slack=float(bucket_slack), cap_log2=-1 if cap_log2 is None else int(cap_log2),
            event_time=time_mode == "event", ooo_bound=self.ooo_bound,
            side_output_late=bool(side_output_late), late_capacity=int(late_capacity),
            external_watermark=bool(external_watermark),
            combine=-1 if combine is None else int(bool(combine)),
            compact=-1 if compact is None else int(bool(compact)),
            narrow=-1 if narrow is None else int(bool(narrow)), dense_keys=bool(dense_keys),
            pipeline=1 if pipeline == "stream" else (2 if pipeline else 0),
            exchange={"auto": 0, "records": 1, "partials": 2}[exchange],
            idle_timeout_steps=-1 if idle_timeout_steps is None else int(idle_timeout_steps),
            deterministic=self.deterministic, spill=bool(spill), spill_load=float(spill_load),
            spill_check_steps=int(spill_check_steps),
            spill_keep_panes=-1 if spill_keep_panes is None else int(spill_keep_panes),
            emit_kv=emit == "key_value", latency_fire=self.latency_fire,
            window_keys=-1 if window_keys is None else int(window_keys),
            dim=int(vec.get("dim", 0)), vec_avg=bool(vec.get("avg", True)),
            vec_threshold=vec.get("threshold"), vec_mode=int(vec.get("mode", 0)))
        from ..ops.native import load

        self._m = load()
        self._s = self._m.WindowStep(cfg, _StepCommAdapter(self.comm, self.device), self.world,
                                     self.rank)
        self._ctl = self._s.ctl
        self.pane, self.panes_per_window = self._ctl.pane, self._ctl.panes_per_window
        self.metrics = _Metrics(self._s)
        self.late_side: list[np.ndarray] = []
        self._timer = None
        self._host_tier = None

    # ---- geometry / configuration (the native step's) ---------------------------------------
    nsub = property(lambda self: self._s.nsub)
    nsub_log2 = property(lambda self: self._s.nsub_log2)
    cap_log2 = property(lambda self: self._s.cap_log2)
    nslots = property(lambda self: self._s.nslots)
    ring = property(lambda self: self._s.ring)
    rec_w = property(lambda self: self._s.rec_w)
    dense_bits = property(lambda self: self._s.dense_bits)
    dense_mul = property(lambda self: self._s.dense_mul)
    local_global = property(lambda self: self._s.local_global)
    combine = property(lambda self: self._s.combine)
    nbuckets = property(lambda self: self._s.nbuckets)
    bucket_cap = property(lambda self: self._s.bucket_cap)
    batch_capacity = property(lambda self: self._s.batch_capacity)
    pipeline = property(lambda self: self._s.pipeline)
    nsub_o = property(lambda self: self._s.nsub_o)
    cap_log2_o = property(lambda self: self._s.cap_log2_o)
    nslots_o = property(lambda self: self._s.nslots_o)
    ring_m = property(lambda self: self._s.ring_m)
    async_fire = property(lambda self: self._s.async_fire)
    two_level = property(lambda self: self._s.two_level)

    @property
    def jhash(self) -> torch.Tensor | None:
        """Key id -> Java String.hashCode table (hash_mode 1); replaced as the dictionary grows."""
        return self._jhash

    @jhash.setter
    def jhash(self, t: torch.Tensor | None) -> None:
        self._jhash = t
        self._s.set_jhash(0 if t is None else t.data_ptr())

    @property
    def compact(self) -> bool:
        """Records narrower than 24 bytes (integer values)."""
        return self.rec_w < 3

    def set_combine_hint(self, ccap: int) -> None:
        """Capacity of the next combined exchange's buckets (tests force overflows with it)."""
        self._s.set_ccap_hint(int(ccap))

    # ---- state buffers (DLPack views sharing the native memory) -------------------------------
    def _view(self, name: str):
        over = self.__dict__.get("_frozen")
        if over is not None and name in over:
            return over[name]
        cap = self._s.view(name)
        return None if cap is None else torch.from_dlpack(cap)

    def _set_view(self, name: str, t) -> None:
        # the frozen copy of an asynchronous snapshot (checkpoint.freeze_operator) holds clones
        self._frozen = {**self.__dict__.get("_frozen", {}), name: t}

    keys_g, acc_g, cnt_g, dirty_g = map(_state_prop, ("keys_g", "acc_g", "cnt_g", "dirty_g"))
    dacc_g, dcnt_g, vacc_g, occ = map(_state_prop, ("dacc_g", "dcnt_g", "vacc_g", "occ"))
    keys_m, acc_m, cnt_m, dirty_m = map(_state_prop, ("keys_m", "acc_m", "cnt_m", "dirty_m"))
    occ_m, dlist, dlist_n, slot_mark = map(_state_prop, ("occ_m", "dlist", "dlist_n", "slot_mark"))
    flags, kg_dest = _state_prop("flags"), _state_prop("kg_dest")

    @property
    def host_tier(self):
        """The host-DRAM tier (runtime/window_spill.HostWindowTier over the native tier)."""
        if not self._s.has_tier:
            return None
        if self._host_tier is None:
            from .window_spill import HostWindowTier

            self._host_tier = HostWindowTier(self.agg, _core=self._s.tier())
        return self._host_tier

    # ---- window arithmetic + bookkeeping (csrc/window_control.h) ------------------------------
    @property
    def wm(self) -> int:
        return self._s.wm

    @wm.setter
    def wm(self, v: int) -> None:
        self._s.wm = int(v)

    def pane_of(self, t: int) -> int:
        return self._ctl.pane_of(t)

    def pane_start(self, p: int) -> int:
        return self._ctl.pane_start(p)

    def last_start(self, t: int) -> int:
        return self._ctl.last_start(t)

    def first_start_containing(self, t: int) -> int:
        return self._ctl.first_start_containing(t)

    def _align_up(self, t: int) -> int:
        return self._ctl.align_up(t)

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

    @property
    def max_seen_pane(self) -> int | None:
        return self._ctl.max_seen() if self._ctl.has_live() else None

    def _set_live(self, lo: int | None, hi: int | None) -> None:
        self._ctl.set_live(lo is not None, 0 if lo is None else int(lo), 0 if hi is None else int(hi))

    def current_processing_time(self) -> int:
        return int(self.clock() if self.clock else time.time() * 1000)

    # ---- main entry points ---------------------------------------------------------------
    def _stream(self) -> int:
        return torch.cuda.current_stream(self.device).cuda_stream if self.device.type == "cuda" else 0

    def _check_batch(self, keys, ts, vals) -> bool:
        n = keys.numel()
        key32 = keys.dtype == torch.int32
        for t, name in ((keys, "keys"), (ts, "ts"), (vals, "vals")):
            want = torch.int32 if t is keys and key32 else torch.int64
            if t.dtype != want or not t.is_contiguous() or t.numel() < n or t.device != self.device:
                K._check(t, want, n, name, self.device)
        if n >= (1 << 32):
            raise ValueError("batch too large (2^32 events)")
        return key32

    @property
    def timer(self):
        """utils.metrics.StageTimer fed by the native step's per-stage clocks (None: off)."""
        return self._timer

    @timer.setter
    def timer(self, t) -> None:
        self._timer = t
        self._s.set_timing(t is not None)

    def _collect(self, block: bool = True) -> list[FireResult]:
        if self._timer is not None:
            for name, ms in self._s.take_stages():
                self._timer.add(name, ms)
        out = [FireResult(s, e, k, v, r, c, refire=rf, seq=sq)
               for s, e, k, v, r, c, rf, sq in self._s.take(block)]
        if self.side_output_late:
            self.late_side.extend(self._s.late_side())
        return out

    def process(self, keys: torch.Tensor, ts: torch.Tensor, vals: torch.Tensor,
                _vecs: torch.Tensor | None = None) -> list[FireResult]:
        """Fold one micro-batch of this rank's source partition and fire what the watermark allows.

        Unpipelined (CPU, DataStream API): partition -> one host sync -> aggregation -> fire, all
        for this batch. Pipelined (GPU hot loops): the call enqueues this batch's partition ahead
        of the state half of the PREVIOUS batch and returns the firings whose rows have reached
        the host (``flush()`` / ``finish()`` drain the rest)."""
        key32 = self._check_batch(keys, ts, vals)
        if self.time_mode == "processing":
            self._s.set_proc_time(self.current_processing_time())
        self._s.process(keys.data_ptr(), key32, ts.data_ptr(), vals.data_ptr(), keys.numel(),
                        self._stream(), 0 if _vecs is None else _vecs.data_ptr())
        return self._collect(block=self._s.block_hint)

    def flush(self) -> list[FireResult]:
        """Complete the pending state half of the last batch (pipelined mode); returns what it
        fired. Every entry point that reads or replaces state calls it first."""
        self._s.flush(self._stream())
        return self._collect()

    def advance_watermark(self, wm: int) -> list[FireResult]:
        """Advance the watermark without data (idle step / processing-time timer / end of input)."""
        self._s.advance_watermark(int(wm), self._stream())
        return self._collect()

    def finish(self) -> list[FireResult]:
        """End of input: event time emits Long.MAX_VALUE (fires everything); processing time does
        not fire pending windows (Flink 1.8 SocketTextStreamFunction end-of-stream behaviour)."""
        self._s.finish(self._stream())
        return self._collect()

    def mark_idle(self, idle: bool = True) -> None:
        """SourceContext.markAsTemporarilyIdle(): exclude this partition from the valve until it
        is marked active again (or sends data, with an idle timeout)."""
        self._s.mark_idle(bool(idle))

    @property
    def idle(self) -> bool:
        return self._s.idle

    def compact_state(self, cutoff_pane: int | None = None, wait: bool = True) -> dict:
        """Table maintenance at a step boundary: drop keys without live data and (with the spill
        tier) move keys whose newest data pane is <= cutoff_pane to host DRAM. Returns counts
        (None: an asynchronous eviction, absorbed at the next tier reader)."""
        d, e, r = self._s.compact_state(cutoff_pane, wait, self._stream())
        if d < 0:
            return {"dropped": None, "evicted": None, "rows": None}
        return {"dropped": d, "evicted": e, "rows": r}

    def _sync_state(self) -> None:
        """Make the state tables current for a host reader (the pending step applied -- its
        firings stay queued for the next call -- streams drained, evictions landed)."""
        self._s.sync_state(self._stream())

    def _drain(self) -> None:
        self._s.drain()

    _state_tensors = ("keys_g", "acc_g", "cnt_g", "dirty_g")
