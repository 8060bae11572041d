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
from typing import Callable

import numpy as np
import torch

from ..ops import expr as E
from ..ops import kernels as K
from ..parallel.comm import Comm, LocalComm
# The operator's halves (mixins) and the names other modules import from here.
from .host_rows import (CountedHostRows, PinnedSlabPool, _event_spin, _host_wait,  # noqa: F401
                        _next_pow2, to_host_arrays)
from . import window_agg as _wa
from .window_agg import _AggMixin
from .window_fire import _FireMixin
from .window_state import _StateMixin
from .window_tiering import _TierMixin
from .window_types import FireResult, OperatorMetrics, _Back, _Front  # noqa: F401

I64_MIN = K.I64_MIN
I64_MAX = K.I64_MAX


class KeyedWindowOperator(_AggMixin, _FireMixin, _TierMixin, _StateMixin):
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







    def _drain(self) -> None:
        """Wait for every queued kernel of this operator (before buffers are reallocated)."""
        if self.device.type == "cuda" and getattr(self, "s1", None) is not None:
            self.s1.synchronize()
            torch.cuda.current_stream(self.device).synchronize()

    def _event(self):
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.device))
        return ev





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
                if _wa._FORCE_SPLIT > 1 and aplan.split == 1 and not combined:
                    aplan.split = -_wa._FORCE_SPLIT  # every sub-table over n workgroups (A/B)
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


































    _state_tensors = ("keys_g", "acc_g", "cnt_g", "dirty_g")




