"""Keyed event-time session windows with a host-DRAM spill tier (BASELINE config 5).

Semantics follow ``EventTimeSessionWindows.withGap(gap)`` + ``allowedLateness`` + an
aggregate (chapter3/README.md:412-428, chapter2/README.md:145 for ``AggregateFunction.merge``):
each element opens ``[ts, ts + gap)``; intersecting (or touching) sessions merge; a session fires
when the watermark reaches ``end - 1``, stays until ``end - 1 + lateness`` and fires again when a
late element extends it. Micro-batch rule (shared by every tier): a batch's elements of one key
are folded in timestamp order, a run of elements closer than ``gap`` is one candidate session,
and a candidate is dropped as late only when it is late on its own and merges with no live
session (csrc/sessions.cpp).

Per step and rank:

1. the batch's global minimum timestamp (one MIN all-reduce) is the step's time base;
2. keyBy partition (pane = 1 ms, so records carry ``ts - tbase``) + RCCL all-to-all, watermark
   valve and overflow flags in the step's one MIN all-reduce (same pass as the window operator);
3. GPU: ``session_lookup`` (HBM open-addressing slot table, tombstone reuse; keys in the device
   spill set -- or hitting a full sub-table -- are diverted to a host staging buffer) -> one
   radix sort of ``slot << 32 | ts - tbase`` -> ``session_heads`` -> ``session_merge`` (one wave
   per key, run detection + segmented scan with shuffles, up to ``kSess`` = 4 resident sessions
   per key; keys with more overflow to the host tier);
4. diverted records and overflow runs are merged by the host ``SessionStore`` (C++);
5. the advanced watermark fires due sessions on both tiers (``session_fire``: fused map/filter
   epilogue, compacted rows) and purges cleaned ones;
6. spill: when the slot table passes its load budget, slots idle for ``idle_spill_ms`` are packed
   by ``session_evict`` into staging rows, copied to host DRAM and inserted into the store; their
   keys join the device spill set (rebuilt from the store as spilled keys expire).

On CPU (``device="cpu"``) the store is the whole engine.
"""
from __future__ import annotations

import contextlib
import math
import time
from collections import defaultdict
from dataclasses import dataclass, field

import numpy as np
import torch

from ..ops import expr as E
from ..ops import kernels as K
from ..ops.native import load
from ..parallel.comm import Comm, LocalComm
from .host_rows import _event_spin

I64_MIN, I64_MAX = K.I64_MIN, K.I64_MAX
K_SESS = 4                # resident sessions per key slot (csrc/kernels_hip.hip kSess)
EMPTY_KEY = -1            # ~0ull
TOMB_KEY = -2             # ~1ull


# Session fold ordering: "lds" = fused lookup + per-sub-table LDS segmented sort (default),
# "radix" = lookup + device-wide radix sort (A/B and the fallback when a sub-table's records
# cannot be staged in LDS).
_SESSION_SORT = __import__("os").environ.get("MXS_SESSION_SORT", "lds")
# The fused lookup-sort writes interleaved (key, value) pairs (one 16-byte store per record)
# instead of two scattered 8-byte stores; "0" keeps the two arrays.
_SESSION_PAIR = int(__import__("os").environ.get("MXS_SESSION_PAIR", "1"))
# Key shards of the host session store, worked in parallel by a persistent pool
# (csrc/session_shards.h). Off by default: on the MI355X box 16 shards made config 5's host
# insert and firing 3-6x slower than one store (profiles/r4_cfg5_shards.md).
_STORE_SHARDS = int(__import__("os").environ.get("MXS_SESSION_SHARDS", "1"))
# The idle eviction's counted D2H on a side stream ("1", default) or behind the eviction on the
# compute stream ("0", A/B: the side-stream launch cost the host 1.2 ms per step at config 5
# while the GPU was busy, against 26 us on an idle GPU -- scripts/d2h_launch_bench.py).
_SPILL_SIDE_STREAM = __import__("os").environ.get("MXS_SPILL_SIDE_STREAM", "1") != "0"
# GPU keyBy records: 16-byte (key, int32 value, ts - tbase) through the two-level compact
# partition ("1", default; a value outside int32 widens the step to 24-byte records and redoes
# it) or the 24-byte plain scatter ("0", A/B).
_REC16 = __import__("os").environ.get("MXS_SESSION_REC16", "1") != "0"
# Promotion of revisited spilled keys through promote rows (SessionStore.extract_rows_into +
# session_promote_rows); "0": the previous extract_packed path (A/B).
_PROMOTE_ROWS = __import__("os").environ.get("MXS_PROMOTE_ROWS", "1") != "0"
# Slot-table rehash trigger (drop tombstones): occupied fraction above _REHASH_OCC with at least
# _REHASH_TOMBS of the slots tombstoned (MXS_SESSION_REHASH="occ,tombs").
_REHASH_OCC, _REHASH_TOMBS = (float(x) for x in
                              __import__("os").environ.get("MXS_SESSION_REHASH", "0.8,0.08").split(","))


def _next_pow2(x: int) -> int:
    return 1 << max(0, int(x - 1).bit_length())


@dataclass
class SessionRows:
    keys: np.ndarray      # uint64
    start: np.ndarray     # int64 session start
    end: np.ndarray       # int64 session end (exclusive; window maxTimestamp = end - 1)
    values: np.ndarray    # float64 result after the map epilogue
    raw: np.ndarray       # int64 raw accumulator
    counts: np.ndarray    # int64 element counts

    def __len__(self) -> int:
        return len(self.keys)

    @staticmethod
    def concat(parts: list["SessionRows"]) -> "SessionRows":
        parts = [p for p in parts if len(p)]
        if not parts:
            return SessionRows(np.zeros(0, np.uint64), *(np.zeros(0, np.int64) for _ in range(2)),
                               np.zeros(0, np.float64), np.zeros(0, np.int64), np.zeros(0, np.int64))
        return SessionRows(*(np.concatenate([getattr(p, f) for p in parts])
                             for f in ("keys", "start", "end", "values", "raw", "counts")))


@dataclass
class SessionMetrics:
    num_records_in: int = 0
    num_late_records_dropped: int = 0
    num_records_out: int = 0
    records_to_host: int = 0
    overflow_keys: int = 0
    spilled_keys: int = 0
    freed_slots: int = 0
    rehashes: int = 0
    promoted_keys: int = 0      # spilled keys handed back to HBM (records arrived for them)
    records_promoted: int = 0   # records of those keys folded on the GPU instead of the host
    current_watermark: int = I64_MIN
    steps: int = 0
    extra: dict = field(default_factory=dict)


class KeyedSessionOperator:
    """Per-rank keyed session-window aggregation: HBM slot table + host-DRAM store."""

    def __init__(self, *, gap: int, lateness: int = 0, agg: int = K.AGG_SUM_I64, device="cpu",
                 comm: Comm | None = None, max_keys: int = 1 << 20,
                 parallelism: int | None = None, max_parallelism: int = 128,
                 batch_capacity: int = 1 << 20, cap_log2: int | None = None,
                 map_prog: E.Program = E.EMPTY, filter_prog: E.Program = E.EMPTY,
                 ooo_bound: int = 0, max_load: float = 0.7, idle_spill_ms: int | None = None,
                 spill_rows: int = 1 << 20, emit_capacity: int | None = None,
                 external_watermark: bool = False, host_budget_bytes: int | None = None,
                 idle_timeout_steps: int | None = None, spill_set_log2: int = 16,
                 sub_table_log2: int | None = None, pipeline: bool = False):
        """pipeline (GPU): the host half of step i -- the fold's counters, the host store's fire,
        the fired rows' collection, the spill -- runs while the GPU works on step i+1's
        partition and fold; process() then returns the sessions fired by the PREVIOUS batch
        (flush() / finish() drain). GPU order stays fold(i) -> fire(i) -> fold(i+1)."""
        if gap <= 0:
            raise ValueError("session gap must be positive")
        self.device = K.resolve_device(device)
        self.comm = comm or LocalComm()
        self.world, self.rank = self.comm.world, self.comm.rank
        self.gap, self.lateness, self.agg = int(gap), int(lateness), agg
        self.parallelism = parallelism or self.world
        self.max_parallelism = max_parallelism
        self.map_prog, self.filter_prog = map_prog, filter_prog
        self.ooo_bound = int(ooo_bound)
        self.external_watermark = external_watermark
        # Idle partitions are left out of the MIN watermark valve (see KeyedWindowOperator).
        self.idle_timeout_steps = idle_timeout_steps
        self._idle_marked = False
        self._empty_steps = 0
        self.max_load = max_load
        self.host_budget_bytes = host_budget_bytes
        self.idle_spill_ms = int(idle_spill_ms if idle_spill_ms is not None else 4 * gap)
        self.metrics = SessionMetrics()
        self.pipeline = bool(pipeline)
        self._pend: dict | None = None   # pipelined: the step whose host half is pending
        self._rehash_due = False
        self._carry: list = []           # rows a state reader's flush fired (returned next)
        self.late_side: list = []  # late records are dropped (no side output on this path)
        self.phase_s: dict[str, float] = defaultdict(float)  # host wall time per phase
        self.native = load()
        self.store = self.native.SessionStore(self.gap, self.lateness, agg, _STORE_SHARDS)
        self.wm = I64_MIN
        self.gpu = self.device.type == "cuda"

        from .geometry import fixed_geometry, state_geometry

        # sub_table_log2: a fixed sub-table size (smaller tables -> more, smaller fold
        # workgroups with less LDS each); default: the shared geometry.
        self.nsub, self.cap_log2 = (fixed_geometry(max_keys, self.world, sub_table_log2)
                                    if sub_table_log2 else
                                    state_geometry(max_keys, self.world, cap_log2))
        self.nsub_log2 = self.nsub.bit_length() - 1
        self.nslots = self.nsub << self.cap_log2
        dev = self.device
        kgd = [(kg * self.parallelism // max_parallelism) * self.world // self.parallelism
               for kg in range(max_parallelism)]
        self.kg_dest = torch.tensor(kgd, dtype=torch.int32, device=dev)
        self.nbuckets = self.world << self.nsub_log2
        self.stats = K.new_stats(dev)
        self.kg_zero = torch.zeros(max_parallelism, dtype=torch.int32, device=dev)  # refold: local
        # Spilled keys that receive records return to HBM (False: fold them in host DRAM).
        self.promote_spilled = True
        self.local_maxts = torch.full((1,), I64_MIN, dtype=torch.int64, device=dev)
        self.red = torch.zeros(K.RED_WORDS, dtype=torch.int64, device=dev)
        # keyBy record width of the GPU step (2: 16-byte records, 3: 24-byte; CPU: 3)
        self.rec_w = 2 if self.gpu and _REC16 else 3
        self._alloc(batch_capacity)
        if self.gpu:
            self._alloc_state()
            self.spill_rows = int(spill_rows)
            self.st_rows = torch.empty(6 * self.spill_rows, dtype=torch.int64, device=dev)
            self._pin_rows = torch.empty((6, self.spill_rows), dtype=torch.int64).pin_memory()
            # A fire can close every resident session of every slot (end of input: all kSess).
            self.ocap = (int(emit_capacity or max(self.nslots * K_SESS, 1 << 16)) + 3) & ~3
            self.out_key = torch.empty(self.ocap, dtype=torch.int64, device=dev)
            self.out_start = torch.empty(self.ocap, dtype=torch.int64, device=dev)
            self.out_end = torch.empty(self.ocap, dtype=torch.int64, device=dev)
            self.out_val = torch.empty(self.ocap, dtype=torch.float64, device=dev)
            self.out_raw = torch.empty(self.ocap, dtype=torch.int64, device=dev)
            self.out_cnt = torch.empty(self.ocap, dtype=torch.int32, device=dev)
            # counters: [0] n_out [1] n_heads [2] n_host [3] n_inserted(step) [4] n_ovf
            #           [5] n_ovf_runs [6] fire n_out [7] evict rows [8] evicted [9] rehash ins
            self.ctr = torch.zeros(16, dtype=torch.int32, device=dev)
            # The pinned slabs of the asynchronous eviction copy, at their final size now
            # (page-locking ~100 MB costs ~15 ms: never inside a step) -- a third one with the
            # pipelined step, whose evictions trail a fold, so the store worker may lag a step.
            nb = ((self.ctr.numel() * 4 + 255) & ~255) + 6 * ((self.spill_rows * 8 + 255) & ~255)
            self._spill_slabs = []
            for _ in range(3 if self.pipeline else 2):
                t = torch.empty(_next_pow2(nb), dtype=torch.uint8, pin_memory=True)
                self._spill_slabs.append([t, t.numpy(), 0])  # tensor, array, job id
            self._spill_turn = 0
            self._spill_allocs = 0
            self.late_cnt = torch.zeros(1, dtype=torch.int64, device=dev)
            self.spill_log2 = int(spill_set_log2)  # grows on the GPU (_rehash_spill_set)
            self.spill_set = torch.full((1 << self.spill_log2,), EMPTY_KEY, dtype=torch.int64,
                                        device=dev)
            self.set_used = 0  # occupied spill-set entries (keys + tombstones)
            self._live_estimate = 0
            # Occupancy bookkeeping from the kernels' own counters (no table scan per step):
            # live keys = inserted - evicted (exact); occupied = live + tombstones, where the
            # tombstone count is an upper bound (an insert may reuse one) -- a rehash decision
            # takes exact counts (launched without a host wait, read a step later). _occ_exact:
            # the next check scans the table.
            self._tombs_bound = 0
            self._occ_exact = True
            self._occ_pending = None  # event of an in-flight occupancy count (_occ_launch)
            # Fired rows: the device-counted copy into a pinned slab (one wait per firing);
            # more rows than the slab column holds take the synchronous copy.
            from .host_rows import PinnedSlabPool

            self._pool = PinnedSlabPool()
            self._fire_rows_async = min(self.ocap, 1 << 20)
            self._hctr = torch.zeros(16, dtype=torch.int32, pin_memory=True)
            self._hlate = torch.zeros(1, dtype=torch.int64, pin_memory=True)
            self._hred = torch.zeros(K.RED_WORDS, dtype=torch.int64, pin_memory=True)
            self.spill_any = False
            self._warm_promote_ops()

    def _warm_promote_ops(self) -> None:
        """The first launch of a PyTorch kernel in a process loads its code object (tens of ms
        on a fresh box, measured as a 60 ms stall inside the first promotion of config 5 with
        revisits, which the warm-up steps never reach): the promote path's own tensor ops run
        once here, on dummy rows, so no step pays it."""
        self._diverted_cols(1, 0)
        cur = torch.zeros(self.nsub, dtype=torch.int32, device=self.device)
        int(cur.max())
        torch.cuda.current_stream(self.device).synchronize()

    # ---- buffers ----------------------------------------------------------------------------
    def _alloc(self, batch_capacity: int, slack: float = 1.5) -> None:
        self.batch_capacity = int(batch_capacity)
        self.slack = slack
        per = self.batch_capacity / self.nbuckets
        nblk = min(1024, max(1, -(-self.batch_capacity // 65536)))
        cap = int(per * slack + 6 * math.sqrt(max(per, 1.0)) + 64) + 8 * nblk
        self.bucket_cap = (cap + 7) & ~7
        dev = self.device
        words = self.nbuckets * self.bucket_cap * K.REC_WORDS
        self.send = torch.empty(words, dtype=torch.int64, device=dev)
        self.recv = torch.empty(words, dtype=torch.int64, device=dev) if self.world > 1 else self.send
        self.cursor = torch.zeros(self.nbuckets, dtype=torch.int32, device=dev)
        self.recv_counts = (torch.zeros(self.nbuckets, dtype=torch.int32, device=dev)
                            if self.world > 1 else self.cursor)
        # Two-level GPU partition (> 512 buckets): write-combined staged kernel into 512 coarse
        # buckets, then the split kernel (csrc partition_split_kernel<24>). Opt-in: for config 5's
        # 24-byte records it measured 407 + 205 us against 464 us for the plain scatter
        # (profiles/r3_cfg5_two_level.md).
        self._scratch = self._scratch_cursor = None
        if self.gpu and 512 < self.nbuckets <= 512 * 32 and (
                _REC16 or __import__("os").environ.get("MXS_TWO_LEVEL24", "0") == "1"):
            # (sized for 24-byte records: a widened step may take the 24-byte two-level path)
            self._scratch = torch.empty(words, dtype=torch.int64, device=dev)
            self._scratch_cursor = torch.zeros(512, dtype=torch.int32, device=dev)
        self._two_level24 = __import__("os").environ.get("MXS_TWO_LEVEL24", "0") == "1"
        if self.gpu:
            total = self.nbuckets * self.bucket_cap
            self.sort_key = torch.empty(total, dtype=torch.int64, device=dev)
            self.vals_buf = torch.empty(total, dtype=torch.int64, device=dev)
            # One buffer: (sort_out | vals_out) for the radix path, or the interleaved
            # (key, value) pairs the fused lookup-sort writes with 16-byte stores.
            self._sv_out = torch.empty(2 * total, dtype=torch.int64, device=dev)
            self.sort_out, self.vals_out = self._sv_out[:total], self._sv_out[total:]
            self._sort_tmp = None
            self.heads = torch.empty(total, dtype=torch.int32, device=dev)
            # key segments of the fused lookup-sort (output position | length << 32)
            self.seg_heads = torch.empty(total, dtype=torch.int64, device=dev)
            self.host_cap = total
            self.host_recs = torch.empty(total * K.REC_WORDS, dtype=torch.int64, device=dev)
            # The merge folds runs into the state as it goes (no redo), so the overflow-run buffer
            # holds the worst case: every received record a run of its own.
            self.ovf_cap = max(1 << 12, total)
            self.ovf_rows = torch.empty(5 * self.ovf_cap, dtype=torch.int64, device=dev)
            self.ovf_slots = torch.empty(2 * total, dtype=torch.int64, device=dev)  # (slot, key)

    def _alloc_state(self) -> None:
        dev, n = self.device, self.nslots
        self.keys_g = torch.full((n,), EMPTY_KEY, dtype=torch.int64, device=dev)
        # [slot][kSess] x {start, end, acc, cnt | flags << 32}: one 128-byte record per slot.
        self.sess = torch.zeros(n * K_SESS * 4, dtype=torch.int64, device=dev)
        # (due, last) per slot in one 16-byte pair (the merge reads and writes both at once);
        # slot_due / slot_last are strided views of it (kSlotMeta in csrc/kernels_hip.hip)
        self._slot_meta = torch.empty((n, 2), dtype=torch.int64, device=dev)
        self.slot_due, self.slot_last = self._slot_meta[:, 0], self._slot_meta[:, 1]
        self.slot_due.fill_(I64_MAX)
        self.slot_last.fill_(I64_MIN)

    def state_bytes(self) -> int:
        self._sync_pending()
        if self.gpu:
            self._join_spill()
        hbm = 0
        if self.gpu:
            hbm = self.nslots * (8 + K_SESS * 32 + 16)
        return hbm + int(self.store.bytes())

    def host_bytes(self) -> int:
        if self.gpu:
            self._join_spill()
        return int(self.store.bytes())

    @contextlib.contextmanager
    def _phase(self, name: str):
        t0 = time.perf_counter()
        try:
            yield
        finally:
            self.phase_s[name] += time.perf_counter() - t0

    # ---- main entry -------------------------------------------------------------------------
    def process(self, keys: torch.Tensor, ts: torch.Tensor, vals: torch.Tensor) -> SessionRows:
        if (self.pipeline and self.gpu and self.wm != I64_MIN and _SESSION_SORT == "lds"
                and self.nslots.bit_length() + 32 <= 62 and keys.numel() <= self.batch_capacity):
            return self._process_pipelined(keys, ts, vals)
        pre = self.flush() if self._pend is not None or self._carry else None
        out = self._process_sync(keys, ts, vals)
        return out if pre is None else SessionRows.concat([pre, out])

    def _process_sync(self, keys: torch.Tensor, ts: torch.Tensor, vals: torch.Tensor,
                      fire: bool = True, exact: bool = False) -> SessionRows | None:
        """One unpipelined step. fire=False: the step stops before its fire (the watermark is
        set; the pipelined path fires it later); exact: start with the exact time base."""
        n = keys.numel()
        if n > self.batch_capacity:
            self._alloc(n, self.slack)
        old_wm = self.wm
        self._empty_steps = self._empty_steps + 1 if n == 0 else 0
        idle = self._idle_marked or (self.idle_timeout_steps is not None
                                     and self._empty_steps >= self.idle_timeout_steps)
        # Time base of the step's relative record times: after the first watermark a provisional
        # base 2^30 ms (12 days) below it -- identical on every rank, no MIN all-reduce and no
        # host sync -- and a step with an older record is redone with the exact minimum (the
        # partition flags it like an unrepresentable span).
        exact = exact or self.wm == I64_MIN
        if exact:
            tbase = self._exact_tbase(ts, n)
        else:
            tbase = self.wm - (1 << 30)
        # GPU, LDS fold: the fold is enqueued right behind the partition and skips itself on the
        # device when the step's reduced flags ask for a redo -- the partition's flags, the
        # fold's counters and its late count come back in ONE host wait (tbits fixed at 32).
        spec = (self.gpu and _SESSION_SORT == "lds"
                and self.nslots.bit_length() + 32 <= 62)
        while True:
            # (the per-rank chunks of the all-to-all are nsub * bucket_cap records of rec_w words:
            # the prefix of the buffers, sized for 24-byte records)
            self._launch_front(keys, ts, vals, n, tbase, idle)
            folded = None
            if spec:
                with self._phase("fold_gpu"):
                    self._fold_prepare()
                    if self._fold_launch(self.recv, self.recv_counts, self.world, tbase, old_wm,
                                         32, self.bucket_cap, skip=self.red, rw=self.rec_w):
                        folded = self._fold_counters(with_red=True)
                        host = self._hred.tolist()
            if folded is None:
                host = self.red.cpu().tolist()
            if host[4]:
                if not exact:  # a record older than the provisional base: exact base, redo
                    exact = True
                    tbase = self._exact_tbase(ts, n)
                    self.metrics.extra["tbase_redos"] = self.metrics.extra.get("tbase_redos", 0) + 1
                    continue
                raise RuntimeError("session batch spans more than 2^32 ms")
            if host[7]:
                raise ValueError("key ids -1 and -2 are reserved (the state tables' markers)")
            if host[5] and self.rec_w < 3:
                # a value outside int32: 24-byte records from now on, redo the step
                self.rec_w = 3
                self.metrics.extra["record_widenings"] = \
                    self.metrics.extra.get("record_widenings", 0) + 1
                continue
            if host[3]:
                self._alloc(self.batch_capacity, self.slack * 2)
                continue
            break
        wm_global = host[2]
        if wm_global == I64_MAX:
            wm_global = old_wm  # every partition idle: the watermark holds
        self.metrics.num_records_in += n
        self.metrics.steps += 1
        if folded is not None:
            with self._phase("fold_gpu"):
                self._fold_finish(folded, folded[0], tbase, old_wm, 32)
        elif self.gpu:
            with self._phase("fold_gpu"):
                self._fold_gpu(tbase, old_wm, max(0, -host[0]))
        else:
            self._fold_cpu(tbase, old_wm)
        # Sessions that late data re-opened fire even when the watermark did not move
        # (EventTimeTrigger.onElement: maxTimestamp <= currentWatermark -> FIRE).
        wm = old_wm if self.external_watermark else max(old_wm, wm_global)
        if not fire:
            self.wm = wm
            self.metrics.current_watermark = wm
            return None
        return self._fire_at(wm)

    def _launch_front(self, keys, ts, vals, n: int, tbase: int, idle: bool) -> None:
        """step_begin + partition + step_finish, the watermark valve's MIN all-reduce and (G > 1)
        the records all-to-all, all enqueued (no host wait)."""
        K.step_begin(self.cursor, self.stats)
        plan = K.PartitionPlan(max_parallelism=self.max_parallelism, nsub_log2=self.nsub_log2,
                               nranks=self.world, window_mode=1, drop_late=0, hash_mode=0,
                               bucket_cap=self.bucket_cap, late_ts=I64_MIN, tbase=tbase, pane=1,
                               rec_words=self.rec_w)
        if self._scratch is not None and (self.rec_w == 2 or self._two_level24):
            plan.scratch = self._scratch.data_ptr()
            plan.scratch_cursor = self._scratch_cursor.data_ptr()
        if n:
            K.partition(keys, ts, vals, plan, self.kg_dest, self.cursor, self.send, self.stats)
        K.step_finish(self.stats, self.local_maxts, self.red, bound=self.ooo_bound,
                      event_mode=True, proc_now=0)
        if idle:
            self.red[2:3].fill_(I64_MAX)
        self.comm.allreduce_min_(self.red[:8])
        if self.world > 1:
            words = self.nbuckets * self.bucket_cap * self.rec_w
            self.comm.all_to_all(self.recv[:words], self.send[:words])
            self.comm.all_to_all(self.recv_counts, self.cursor)

    def _counters_launch(self):
        """The fold's counters and late count on their way to pinned memory (an event, no wait)."""
        self._hctr.copy_(self.ctr, non_blocking=True)
        self._hlate.copy_(self.late_cnt, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.device))
        return ev

    def _counters_read(self, ev) -> list[int]:
        with self._phase("fold_gpu.sync"):
            _event_spin(ev)
            h = self._hctr[:6].tolist() + [int(self._hlate[0])]
        self._live_estimate += h[3]
        return h

    def _process_pipelined(self, keys, ts, vals) -> SessionRows:
        """One pipelined step (GPU, LDS fold): returns what the PREVIOUS batch fired.

        GPU stream:  ... fold(i-1) | partition(i) | fire(i-1) | fold(i) | evict(i-1) ...
        host:        wait fold(i-1)'s counters -> its host fold work -> launch fire(i-1) ->
                     launch fold(i) (skips itself on the device if step i must be redone) ->
                     spill check at fire(i-1)'s watermark -> host store fire(i-1) -> collect
                     fire(i-1)'s rows -> read step i's flags.
        Late data of batch i merges after fire(i-1) as unpipelined; the spill check and the host
        fire overlap fold(i). An eviction behind fold(i) moves that fold's merges with the
        sessions (the overflow list carries each slot's key, so an overflowed slot may be
        evicted before the host reads the list); a due rehash, which moves slots, waits for the
        next step's window with no fold in flight. The host fire waits only for evictions
        before fire(i-1) (later ones moved sessions the GPU fire saw). Keys the host fire or the
        spill worker release leave the device spill set behind fold(i), which still diverted
        their records to the host tier: _host_fold puts such keys back in the set."""
        n = keys.numel()
        old_wm = self.wm
        empty0 = self._empty_steps
        self._empty_steps = self._empty_steps + 1 if n == 0 else 0
        idle = self._idle_marked or (self.idle_timeout_steps is not None
                                     and self._empty_steps >= self.idle_timeout_steps)
        tbase = old_wm - (1 << 30)
        with self._phase("front"):
            self._launch_front(keys, ts, vals, n, tbase, idle)
            self._hred.copy_(self.red, non_blocking=True)
            ev_red = torch.cuda.Event()
            ev_red.record(torch.cuda.current_stream(self.device))
        P, self._pend = self._pend, None
        fire_rows = None
        if P is not None:
            if not P["done"]:
                h = self._counters_read(P["ev"])
                with self._phase("fold_gpu"):
                    self._fold_finish(h, h[0], P["tbase"], P["old_wm"], 32)
            self._rehash_if_due()
            with self._phase("fire_gpu"):
                fire_rows = self._fire_gpu_launch(P["wm"])
        with self._phase("fold_gpu"):
            self._fold_prepare()
            launched = self._fold_launch(self.recv, self.recv_counts, self.world, tbase, old_wm,
                                         32, self.bucket_cap, skip=self.red, rw=self.rec_w)
            ev_fold = self._counters_launch() if launched else None
        out = SessionRows.concat([])
        if P is not None:
            jobs = self.store.spill_submitted()
            with self._phase("spill"):
                self._maybe_spill(P["wm"], inflight=launched)
            with self._phase("fire_host"):
                host_rows = self._fire_host(P["wm"], jobs)
            out = self._fire_rows(P["wm"], fire_rows, host_rows)
        with self._phase("front.sync"):
            _event_spin(ev_red)
            host = self._hred.tolist()
        if host[7]:
            raise ValueError("key ids -1 and -2 are reserved (the state tables' markers)")
        redo = host[4] or host[3] or (host[5] and self.rec_w < 3)
        if redo or not launched:
            # The speculative fold skipped itself on the device (or the LDS fold does not apply):
            # this batch takes the synchronous path (cause fixed first), its fire stays pending.
            exact = bool(host[4])
            ex = self.metrics.extra
            if exact:
                ex["tbase_redos"] = ex.get("tbase_redos", 0) + 1
            if host[5] and self.rec_w < 3:
                self.rec_w = 3
                ex["record_widenings"] = ex.get("record_widenings", 0) + 1
            if host[3]:
                self._alloc(self.batch_capacity, self.slack * 2)
            self._rehash_if_due()
            self._empty_steps = empty0
            self._process_sync(keys, ts, vals, fire=False, exact=exact)
            self._pend = {"tbase": 0, "old_wm": old_wm, "wm": self.wm, "ev": None, "done": True}
            return out
        wm_global = host[2]
        if wm_global == I64_MAX:
            wm_global = old_wm
        self.metrics.num_records_in += n
        self.metrics.steps += 1
        wm = old_wm if self.external_watermark else max(old_wm, wm_global)
        self.wm = wm
        self.metrics.current_watermark = wm
        self._pend = {"tbase": tbase, "old_wm": old_wm, "wm": wm, "ev": ev_fold, "done": False}
        return out

    def flush(self) -> SessionRows:
        """Pipelined: the pending step's host half (counters, host fold work, fire, spill) and
        any rows a state reader's flush left behind."""
        out, self._carry = self._carry, []
        P, self._pend = self._pend, None
        if P is not None:
            if not P["done"]:
                h = self._counters_read(P["ev"])
                self._fold_finish(h, h[0], P["tbase"], P["old_wm"], 32)
            self._rehash_if_due()
            out.append(self._fire_at(P["wm"]))
        return SessionRows.concat(out)

    def _rehash_if_due(self) -> None:
        """A rehash the spill check deferred while a fold was in flight (it moves slots; the
        fold's overflow list and counters are read afterwards): done with no fold pending."""
        if self._rehash_due:
            self._rehash_due = False
            self._rehash()
            self._tombs_bound = 0

    def _sync_pending(self) -> None:
        """Before a state reader: apply the pending step; its rows wait for the next call."""
        if self._pend is not None:
            rows = self.flush()  # (flush swaps self._carry: read it after the call)
            self._carry.append(rows)

    def _exact_tbase(self, ts: torch.Tensor, n: int) -> int:
        """The step's minimum timestamp over all ranks (one MIN all-reduce + host read)."""
        t = ts.min().reshape(1) if n else torch.full((1,), I64_MAX, dtype=torch.int64,
                                                    device=ts.device)
        self.comm.allreduce_min_(t)
        tbase = int(t.item())
        return 0 if tbase == I64_MAX else tbase

    def mark_idle(self, idle: bool = True) -> None:
        self._idle_marked = bool(idle)

    def advance_watermark(self, wm: int) -> SessionRows:
        wm = int(wm)
        pre = self.flush()
        if wm <= self.wm:
            return pre
        return SessionRows.concat([pre, self._fire_at(wm)])

    def _fire_at(self, wm: int) -> SessionRows:
        self.wm = wm
        self.metrics.current_watermark = wm
        if wm == I64_MIN:
            return SessionRows.concat([])
        pending = None
        if self.gpu:
            # The GPU firing is launched first; the host store fires while it runs and its rows
            # come back.
            with self._phase("fire_gpu"):
                pending = self._fire_gpu_launch(wm)
        return self._fire_complete(wm, pending)

    def _fire_complete(self, wm: int, pending) -> SessionRows:
        """The host store's fire at `wm`, the launched GPU fire's rows, the spill check."""
        with self._phase("fire_host"):
            # (the store's fire waits for the hot phase of queued eviction jobs itself)
            host_rows = self._fire_host(wm)
        if self.gpu:
            with self._phase("spill"):
                self._maybe_spill(wm)
        return self._fire_rows(wm, pending, host_rows)

    def _fire_rows(self, wm: int, pending, host_rows: SessionRows) -> SessionRows:
        """The launched GPU fire's rows (the spill check's eviction kernel runs after the fire
        kernel: the rows are those of the table before it) with the host store's, and the
        host-DRAM budget check."""
        parts = []
        if pending is not None:
            with self._phase("fire_gpu"):
                parts.append(self._fire_gpu_collect(pending))
        parts.append(host_rows)
        out = SessionRows.concat(parts)
        self.metrics.num_records_out += len(out)
        if self.host_budget_bytes is not None and self.steps_since_budget_check() and \
                self.host_bytes() > self.host_budget_bytes:
            raise MemoryError(f"host-DRAM session state {self.host_bytes()} B exceeds the budget "
                              f"{self.host_budget_bytes} B")
        return out

    def steps_since_budget_check(self, every: int = 16) -> bool:
        """The store's byte count walks the hot map: check the budget every `every` steps."""
        return self.metrics.steps % every == 0

    def finish(self) -> SessionRows:
        return self.advance_watermark(I64_MAX)

    # ---- CPU tier ---------------------------------------------------------------------------
    def _received(self, tbase: int):
        """Decode the received bucket records (host arrays key, ts, val)."""
        recs = self.recv.view(-1, K.REC_WORDS).cpu().numpy()
        counts = self.recv_counts.cpu().numpy().astype(np.int64)
        idx = np.arange(self.bucket_cap, dtype=np.int64)
        valid = (idx[None, :] < counts[:, None]).reshape(-1)
        r = recs[: self.nbuckets * self.bucket_cap][valid]
        t = (r[:, 2] & 0xFFFFFFFF)
        keep = t != 0xFFFFFFFF
        r, t = r[keep], t[keep]
        return r[:, 0].copy(), t + tbase, r[:, 1].copy()

    def _fold_cpu(self, tbase: int, wm: int) -> None:
        k, t, v = self._received(tbase)
        if len(k):
            self.metrics.num_late_records_dropped += int(self.store.process(k, t, v, wm))

    def _fire_host(self, wm: int, hot_upto: int = -1) -> SessionRows:
        """hot_upto >= 0: wait only for eviction jobs up to that id (the pipelined step fires
        after the next spill check: its evictions were in HBM for the GPU fire)."""
        mc, mk = self.map_prog.as_args()
        fc, fk = self.filter_prog.as_args()
        # GPU: cold-chunk expiry (no rows, only released keys) runs on the spill worker after
        # its insert, except at end of input.
        defer = self.gpu and wm != I64_MAX
        d = self.store.fire(wm, mc, mk, fc, fk, not defer, hot_upto)
        if defer:
            self._expire_wm = wm
        rel = d["released"]
        if self.gpu and len(rel) and self.spill_any:
            # Keys that left the host store leave the device spill set (tombstoned).
            kt = self._keys_to_device(rel)
            self.native.gpu_set_erase(self.spill_set.data_ptr(), self.spill_set.numel() - 1,
                                      kt.data_ptr(), kt.numel(), self._st())
        return SessionRows(d["keys"].view(np.uint64), d["start"], d["end"], d["values"], d["raw"],
                           d["counts"])

    # ---- GPU tier ---------------------------------------------------------------------------
    def _st(self) -> int:
        return torch.cuda.current_stream(self.device).cuda_stream

    def _fold_gpu(self, tbase: int, wm: int, tspan: int) -> None:
        """tspan: the step's largest ts - tbase over all ranks (sizes the sort key's time bits)."""
        tbits = min(32, max(1, int(tspan).bit_length()))  # (no records: tspan is meaningless)
        self._fold_prepare()
        h, total = self._fold_recs(self.recv, self.recv_counts, self.world, tbase, wm, tbits,
                                   self.bucket_cap, rw=self.rec_w)
        self._fold_finish(h, total, tbase, wm, tbits)

    def _fold_prepare(self) -> None:
        if self._live_estimate > 0.9 * self.nslots:
            self._join_spill()
            # Sub-tables may fill up: room in the spill set for every key the lookup may divert.
            self._ensure_spill_capacity(self.batch_capacity)

    def _fold_finish(self, h: list[int], total: int, tbase: int, wm: int, tbits: int) -> None:
        """Host side of a fold whose counters are read: overflow runs, promotion or host fold
        of records diverted to spilled keys."""
        if h[2] > self.host_cap:
            raise RuntimeError("host diversion buffer overflow")
        if h[2] or h[4]:
            # Diverted records / overflow runs go to the host store, which must hold last step's
            # spilled rows; otherwise the spill worker keeps running until the host fire needs it.
            self._join_spill()
        late = h[6] if total else 0
        n_host = h[2]
        # Overflow runs first: the refold below reuses the overflow buffers.
        late += self._overflow_runs(h, wm)
        if n_host and self.promote_spilled:
            n_host, late2 = self._promote_and_refold(n_host, tbase, wm, tbits)
            late += late2
        if n_host:
            self._host_fold(n_host, tbase, wm)
        self.metrics.num_late_records_dropped += late

    def _fold_recs(self, recs, counts, nsrc: int, tbase: int, wm: int, tbits: int,
                   bucket_cap: int, rw: int = 3):
        """Lookup -> (slot | ts) radix sort -> ordered session merge of bucketed records
        (`rw`: their width, 2 = 16-byte, 3 = 24-byte). Returns the host counters c[:6] and the
        number of looked-up records."""
        m, st, c = self.native, self._st(), self.ctr
        sbits = self.nslots.bit_length()  # one spare bit: valid keys stay below the sentinel
        if self._fold_launch(recs, counts, nsrc, tbase, wm, tbits, bucket_cap, rw=rw):
            h = self._fold_counters()
            if h[2] > self.host_cap:
                raise RuntimeError("host diversion buffer overflow")
            return h, h[0]
        m.gpu_session_lookup(recs.data_ptr(), counts.data_ptr(), nsrc,
                             self.nsub, bucket_cap, self.cap_log2, self.keys_g.data_ptr(),
                             self.spill_set.data_ptr(), self.spill_set.numel() - 1,
                             int(self.spill_any), self.sort_key.data_ptr(), self.vals_buf.data_ptr(),
                             c[0:1].data_ptr(), self.host_recs.data_ptr(), c[2:3].data_ptr(),
                             self.host_cap, c[3:4].data_ptr(), tbits, st, rec_words=rw)
        total = int(c[0].item())
        if total:
            # Key-value radix sort over the used bits only (slot | ts - tbase); values ride along.
            nbits = tbits + sbits
            need = m.gpu_sort_pairs_temp_bytes(total, 0, nbits)
            if self._sort_tmp is None or self._sort_tmp.numel() < need:
                self._sort_tmp = torch.empty(need, dtype=torch.uint8, device=self.device)
            m.gpu_sort_pairs(self._sort_tmp.data_ptr(), self._sort_tmp.numel(),
                             self.sort_key.data_ptr(), self.sort_out.data_ptr(),
                             self.vals_buf.data_ptr(), self.vals_out.data_ptr(), total, 0, nbits, st)
            m.gpu_session_merge(self.sort_out.data_ptr(), self.vals_out.data_ptr(),
                                c[0:1].data_ptr(), self.heads.data_ptr(), c[1:2].data_ptr(),
                                total, tbits, self.gap, self.lateness, wm, tbase,
                                self.agg, self.cap_log2, self.nslots, self.sess.data_ptr(),
                                self.slot_due.data_ptr(),
                                self.slot_last.data_ptr(), self.late_cnt.data_ptr(),
                                self.keys_g.data_ptr(), self.ovf_slots.data_ptr(),
                                c[4:5].data_ptr(), self.ovf_rows.data_ptr(), c[5:6].data_ptr(),
                                self.ovf_cap, st)
        h = self._fold_counters()
        if h[2] > self.host_cap:
            raise RuntimeError("host diversion buffer overflow")
        return h, total

    # Reduced-vector words whose non-zero value makes a speculatively launched fold skip itself:
    # [3] bucket overflow (redo), [4] span > 2^32 ms, [7] reserved key id (and, with 16-byte
    # records, [5]: a value that needs 24-byte records).
    _SKIP_MASK = (1 << 3) | (1 << 4) | (1 << 7)

    def _fold_launch(self, recs, counts, nsrc: int, tbase: int, wm: int, tbits: int,
                     bucket_cap: int, skip: torch.Tensor | None = None, rw: int = 3) -> bool:
        """Lookup + per-sub-table LDS segmented sort in one kernel -- (slot, ts)-ordered records
        without holes, straight into the merge (no device-wide radix sort). The record count
        stays on the device (the merge reads it); the host learns it with the counters. False:
        the LDS path does not apply (nothing launched)."""
        m, st, c = self.native, self._st(), self.ctr
        c[:7].zero_()
        c[10:11].zero_()
        self.late_cnt.zero_()
        n_cap = nsrc * self.nsub * bucket_cap
        if _SESSION_SORT != "lds" or n_cap > self.sort_out.numel():
            return False
        if not m.gpu_session_lookup_sort(
                recs.data_ptr(), counts.data_ptr(), nsrc, self.nsub, bucket_cap,
                self.cap_log2, self.keys_g.data_ptr(), self.spill_set.data_ptr(),
                self.spill_set.numel() - 1, int(self.spill_any), self.sort_out.data_ptr(),
                self.vals_out.data_ptr(), c[0:1].data_ptr(), self.host_recs.data_ptr(),
                c[2:3].data_ptr(), self.host_cap, c[3:4].data_ptr(), tbits, st,
                skip.data_ptr() if skip is not None else 0,
                (self._SKIP_MASK | (1 << 5 if rw < 3 else 0)) if skip is not None else 0,
                self.seg_heads.data_ptr(), c[10:11].data_ptr(), _SESSION_PAIR, rec_words=rw):
            return False
        # One lane per key segment listed by the lookup-sort (c[10] segments on the device).
        m.gpu_session_merge_heads(self.sort_out.data_ptr(), self.vals_out.data_ptr(),
                                  c[0:1].data_ptr(), self.seg_heads.data_ptr(),
                                  c[10:11].data_ptr(), min(n_cap, self.nslots),
                                  self.heads.data_ptr(), c[1:2].data_ptr(), tbits, self.gap,
                                  self.lateness, wm, tbase, self.agg, self.cap_log2, self.nslots,
                                  self.sess.data_ptr(), self.slot_due.data_ptr(),
                                  self.slot_last.data_ptr(), self.late_cnt.data_ptr(),
                                  self.keys_g.data_ptr(), self.ovf_slots.data_ptr(),
                                  c[4:5].data_ptr(), self.ovf_rows.data_ptr(), c[5:6].data_ptr(),
                                  self.ovf_cap, st, _SESSION_PAIR)
        return True

    def _fold_counters(self, with_red: bool = False) -> list[int]:
        """The fold's counters and late count in one wait (two small copies into pinned memory,
        one stream sync); inserted keys go into the occupancy bookkeeping. Returns c[:6] with
        the late-dropped count of the fold appended (h[6])."""
        with self._phase("fold_gpu.sync"):
            if with_red:
                self._hred.copy_(self.red, non_blocking=True)
            self._hctr.copy_(self.ctr, non_blocking=True)
            self._hlate.copy_(self.late_cnt, non_blocking=True)
            torch.cuda.current_stream(self.device).synchronize()
            h = self._hctr[:6].tolist() + [int(self._hlate[0])]
        self._live_estimate += h[3]
        return h

    def _diverted(self, n_host: int, tbase: int):
        r = self.host_recs[: n_host * K.REC_WORDS].view(-1, K.REC_WORDS)
        return r[:, 0], (r[:, 2] & 0xFFFFFFFF) + tbase, r[:, 1]

    def _diverted_cols(self, n_host: int, tbase: int):
        """The diverted records as three contiguous columns in a reused device buffer."""
        buf = getattr(self, "_dv_buf", None)
        if buf is None or buf.shape[1] < n_host:
            buf = self._dv_buf = torch.empty((3, max(1 << 16, 1 << (n_host - 1).bit_length())),
                                             dtype=torch.int64, device=self.device)
        r = self.host_recs[: n_host * K.REC_WORDS].view(-1, K.REC_WORDS)
        dk, dt, dv = buf[0, :n_host], buf[1, :n_host], buf[2, :n_host]
        dk.copy_(r[:, 0])
        torch.bitwise_and(r[:, 2], 0xFFFFFFFF, out=dt)
        dt.add_(tbase)
        dv.copy_(r[:, 1])
        return dk, dt, dv

    def _host_fold(self, n_host: int, tbase: int, wm: int) -> None:
        """Records of keys that live in host DRAM: folded by the host store."""
        dk, t, v = self._diverted(n_host, tbase)
        if self.pipeline:
            # (pipelined: a key released by the host fire that ran behind this fold's launch was
            # erased from the set after its records were diverted -- it holds sessions again)
            dk = dk.contiguous()
            self.native.gpu_set_insert(self.spill_set.data_ptr(), self.spill_set.numel() - 1,
                                       dk.data_ptr(), dk.numel(), self._st())
        k, t, v = (x.cpu().numpy() for x in (dk, t, v))
        self.metrics.num_late_records_dropped += int(self.store.process(k.copy(), t, v.copy(), wm))
        self.metrics.records_to_host += n_host
        self.set_used += n_host  # upper bound on keys the lookup added (full sub-tables)
        self.spill_any = True
        self._ensure_spill_capacity(0)

    def _promote_and_refold(self, n_host: int, tbase: int, wm: int, tbits: int):
        """Spilled keys that received records come back to HBM: their sessions leave the host
        store (store.extract), are written into freshly inserted slots, the keys leave the
        device spill set, and their records are re-partitioned and folded by the same GPU
        lookup/sort/merge as resident keys (instead of a per-record host fold). Keys with more
        sessions than a slot holds, or whose sub-table is full, stay on the host path.
        Returns (records still for the host tier, late-dropped)."""
        with self._phase("promote"):
            with self._phase("promote.clone"):
                dk, dt, dv = self._diverted_cols(n_host, tbase)
            dev = self.device
            if _PROMOTE_ROWS:
                # the diverted keys as they are (repeats included): the store dedups them (a
                # bitmap over dense ids) -- no device unique and no second round trip
                with self._phase("promote.keys"):
                    if getattr(self, "_pk_host", None) is None or self._pk_host.numel() < n_host:
                        self._pk_host = torch.empty(max(1024, 1 << (n_host - 1).bit_length()),
                                                    dtype=torch.int64, pin_memory=True)
                    hk = self._pk_host[:n_host]
                    hk.copy_(dk, non_blocking=True)
                    torch.cuda.current_stream(dev).synchronize()
                n_moved = self._promote_rows(dk, hk.numpy(), wm)
            else:
                with self._phase("promote.unique"):
                    ukh = torch.unique(dk).cpu().numpy()
                n_moved = self._promote_packed(ukh, wm)
            self.metrics.promoted_keys += n_moved
            # Re-partition the diverted records (local sub-tables only) and fold them.
            # Private bucket buffers sized for these records (the exchange buffers must keep the
            # same size on every rank, so they are never regrown locally).
            per = n_host / self.nsub
            cap = (int(per * 1.5 + 6 * math.sqrt(max(per, 1.0)) + 64) + 8 * 16 + 7) & ~7
            t_part = time.perf_counter()
            while True:
                words = self.nsub * cap * K.REC_WORDS
                if getattr(self, "_rf_send", None) is None or self._rf_send.numel() < words:
                    self._rf_send = torch.empty(words, dtype=torch.int64, device=dev)
                    self._rf_cursor = torch.zeros(self.nsub, dtype=torch.int32, device=dev)
                K.step_begin(self._rf_cursor, self.stats)
                plan = K.PartitionPlan(max_parallelism=self.max_parallelism,
                                       nsub_log2=self.nsub_log2, nranks=1, window_mode=1,
                                       drop_late=0, hash_mode=0, bucket_cap=cap,
                                       late_ts=I64_MIN, tbase=tbase, pane=1)
                K.partition(dk, dt, dv, plan, self.kg_zero, self._rf_cursor, self._rf_send,
                            self.stats)
                if int(self._rf_cursor.max()) <= cap:
                    break
                cap *= 2  # a bucket overflowed (skewed keys): larger buckets, partition again
            self.phase_s["promote.partition"] += time.perf_counter() - t_part
            with self._phase("promote.fold"):
                h, total = self._fold_recs(self._rf_send, self._rf_cursor, 1, tbase, wm, tbits,
                                           cap)
            self.metrics.records_promoted += n_host - h[2]
            late = h[6] if total else 0
            with self._phase("promote.overflow"):
                late += self._overflow_runs(h, wm)
            return h[2], late

    def _promote_rows(self, dk, hk, wm: int) -> int:
        """The promote path's host side in one C++ call and one copy: the store writes the
        revisited keys' sessions as promote rows {key, start, end, acc, cnt | flags << 32, last
        activity, position, sessions of the key} straight into a reused pinned buffer
        (SessionStore.extract_rows_into: with the dense cold-row index, one lookup per key
        instead of a scan of every cold row; the general extract otherwise), plus the keys that
        left the store. ONE copy takes the rows to HBM and session_promote_rows (two launches:
        slot insert + record 0, then further positions) writes the slots. The keys leave the
        device spill set from the device copy of the diverted keys when all of them moved (no
        upload; repeats are harmless). dk / hk: the diverted keys on the device / in pinned
        memory. Returns the number of keys that left the store."""
        n = len(hk)
        if n == 0:
            return 0
        rows_cap = n * K_SESS
        if getattr(self, "_pd_host", None) is None or self._pd_host.shape[0] < rows_cap:
            cap = max(1024, 1 << (rows_cap - 1).bit_length())
            self._pd_host = torch.empty((cap, 8), dtype=torch.int64, pin_memory=True)
            self._pd_moved = torch.empty(cap, dtype=torch.int64, pin_memory=True)
            self._pd_dev = torch.empty((cap, 8), dtype=torch.int64, device=self.device)
            self._pd_slots = torch.empty(cap, dtype=torch.int64, device=self.device)
        if getattr(self, "_pd_copied", None) is not None:
            with self._phase("promote.wait_upload"):
                self._pd_copied.synchronize()  # the previous upload has left the pinned buffers
        hrows, hmoved = self._pd_host, self._pd_moved
        with self._phase("promote.extract"):
            nk, nm, nu = self.store.extract_rows_into(hk, wm, K_SESS, self.gap, hrows.data_ptr(),
                                                      hrows.shape[0], hmoved.data_ptr(),
                                                      hmoved.numel())
        st = self._st()
        with self._phase("promote.scatter"):
            if nm == nu:
                mt = dk  # every wanted key left the store
            else:
                mt = hmoved[:nm].to(self.device, non_blocking=True)
            if nm:
                self.native.gpu_set_erase(self.spill_set.data_ptr(), self.spill_set.numel() - 1,
                                          mt.data_ptr(), mt.numel(), st)
            if nk:
                self._pd_dev[:nk].copy_(hrows[:nk], non_blocking=True)
            if getattr(self, "_pd_copied", None) is None:
                self._pd_copied = torch.cuda.Event()
            self._pd_copied.record(torch.cuda.current_stream(self.device))
            if nk == 0:
                return nm
            self.ctr[3:5].zero_()
            self.native.gpu_session_promote_rows(self._pd_dev.data_ptr(), nk, self.nsub_log2,
                                                 self.cap_log2, self.keys_g.data_ptr(),
                                                 self._pd_slots.data_ptr(), self.sess.data_ptr(),
                                                 self.slot_due.data_ptr(),
                                                 self.slot_last.data_ptr(),
                                                 self.ctr[3:4].data_ptr(),
                                                 self.ctr[4:5].data_ptr(), st)
            ins, n_bad = self.ctr[3:5].tolist()
            self._live_estimate += ins
        if n_bad:  # sub-table full (rare): those keys' sessions go back to the store
            ex = self.metrics.extra
            ex["promote_bad_keys"] = ex.get("promote_bad_keys", 0) + n_bad
            bad = (self._pd_slots[:nk] < 0).cpu().numpy()
            r = hrows[:nk].numpy()[bad]
            self.store.insert(np.ascontiguousarray(r[:, 0]), np.ascontiguousarray(r[:, 1]),
                              np.ascontiguousarray(r[:, 2]), np.ascontiguousarray(r[:, 3]),
                              np.ascontiguousarray(r[:, 4] & 0xFFFFFFFF),
                              np.ascontiguousarray(r[:, 4] >> 32), False)
            bk = torch.from_numpy(np.unique(r[:, 0])).to(self.device)
            self.native.gpu_set_insert(self.spill_set.data_ptr(), self.spill_set.numel() - 1,
                                       bk.data_ptr(), bk.numel(), st)
            self.set_used += int(bk.numel())
            nm -= int(bk.numel())
        return nm

    def _promote_packed(self, ukh, wm: int) -> int:
        """The previous promote path (MXS_PROMOTE_ROWS=0, A/B): extract_packed's slot records
        ([key][kSess][4]) + last activity, three uploads, slot insert + promote kernels, the
        moved keys uploaded for the spill-set erase. Returns the number of keys that left."""
        dev = self.device
        with self._phase("promote.extract"):
            ex = self.store.extract_packed(ukh, wm, K_SESS, self.gap)
        moved = ex["moved"]
        nk = len(ex["key"])
        if nk:
            with self._phase("promote.scatter"):
                ukeys = torch.from_numpy(ex["key"]).to(dev, non_blocking=True)
                rec = torch.from_numpy(ex["rec"]).to(dev, non_blocking=True)
                last = torch.from_numpy(ex["last"]).to(dev, non_blocking=True)
                slots_t = torch.empty_like(ukeys)
                self.ctr[3:5].zero_()
                self.native.gpu_session_slot_insert(ukeys.data_ptr(), nk, self.nsub_log2,
                                                    self.cap_log2, self.keys_g.data_ptr(),
                                                    slots_t.data_ptr(),
                                                    self.ctr[3:4].data_ptr(), self._st())
                self.native.gpu_session_promote(slots_t.data_ptr(), rec.data_ptr(),
                                                last.data_ptr(), nk, self.sess.data_ptr(),
                                                self.slot_due.data_ptr(),
                                                self.slot_last.data_ptr(),
                                                self.ctr[4:5].data_ptr(), self._st())
                ins, n_bad = self.ctr[3:5].tolist()
                self._live_estimate += ins
            if n_bad:  # sub-table full (rare): those keys' sessions go back to the store
                bad = slots_t.cpu().numpy() < 0
                rr = ex["rec"].reshape(nk, K_SESS, 4)[bad].reshape(-1, 4)
                kk = np.repeat(ex["key"][bad], K_SESS)
                live = (rr[:, 3] & 0xFFFFFFFF) != 0
                self.store.insert(np.ascontiguousarray(kk[live]),
                                  np.ascontiguousarray(rr[live, 0]),
                                  np.ascontiguousarray(rr[live, 1]),
                                  np.ascontiguousarray(rr[live, 2]),
                                  np.ascontiguousarray(rr[live, 3] & 0xFFFFFFFF),
                                  np.ascontiguousarray(rr[live, 3] >> 32), False)
                moved = np.setdiff1d(moved, ex["key"][bad])
        if len(moved):
            mt = torch.from_numpy(np.ascontiguousarray(moved, dtype=np.int64)).to(dev)
            self.native.gpu_set_erase(self.spill_set.data_ptr(), self.spill_set.numel() - 1,
                                      mt.data_ptr(), mt.numel(), self._st())
        return len(moved)

    def _overflow_runs(self, h, wm: int) -> int:
        """Keys whose merge produced more than kSess sessions move to the host tier."""
        n_ovf, n_runs = h[4], h[5]
        if not n_ovf:
            return 0
        if n_runs > self.ovf_cap:
            raise RuntimeError("session overflow-run buffer too small")
        pairs = self.ovf_slots[:2 * n_ovf].view(n_ovf, 2)
        slots = pairs[:, 0].contiguous()
        # (the merge recorded each slot's key: a pipelined step's idle eviction may have
        # tombstoned the slot since -- _evict skips it, its sessions are in the store already)
        hp = pairs.cpu().numpy()
        sl, okeys = hp[:, 0].copy(), hp[:, 1].copy()
        self._evict(slots=slots)
        rows = self.ovf_rows.view(5, self.ovf_cap)[:, :n_runs].cpu().numpy()
        # key of every run's slot (vectorised: sorted slots + searchsorted)
        o = np.argsort(sl, kind="stable")
        pos = np.searchsorted(sl[o], rows[0])
        rk = okeys[o][np.minimum(pos, max(o.size - 1, 0))].astype(np.int64)
        self.metrics.overflow_keys += n_ovf
        return int(self.store.merge_runs(rk, rows[1].copy(), rows[2].copy(), rows[3].copy(),
                                         rows[4].copy(), wm))

    def _fire_gpu(self, wm: int) -> SessionRows:
        return self._fire_gpu_collect(self._fire_gpu_launch(wm))

    def _fire_gpu_launch(self, wm: int):
        m, st, c = self.native, self._st(), self.ctr
        mc, mk = self.map_prog.as_args()
        fc, fk = self.filter_prog.as_args()
        c[6:7].zero_()
        m.gpu_session_fire(self.gap, self.lateness, wm, self.agg, self.cap_log2, self.nslots,
                           self.keys_g.data_ptr(), self.sess.data_ptr(), self.slot_due.data_ptr(), mc, mk, fc, fk, self.out_key.data_ptr(),
                           self.out_start.data_ptr(), self.out_end.data_ptr(),
                           self.out_val.data_ptr(), self.out_raw.data_ptr(),
                           self.out_cnt.data_ptr(), c[6:7].data_ptr(), self.ocap, st)
        from .host_rows import CountedHostRows

        ka = self._fire_rows_async
        cols = [t[:ka] for t in (self.out_key, self.out_start, self.out_end, self.out_val,
                                 self.out_raw, self.out_cnt)]
        return CountedHostRows(self._pool, cols, c[6:7], [c])

    def _fire_gpu_collect(self, rows) -> SessionRows:
        ka = self._fire_rows_async
        rows.wait()
        k = int(rows.fixed(0)[6])
        if k > self.ocap:
            raise RuntimeError(f"session emit buffer overflow ({k} > {self.ocap})")
        if k <= ka:
            h = rows.columns(k)
            return SessionRows(h[0].view(np.uint64), h[1], h[2], h[3], h[4],
                               h[5].astype(np.int64))
        return SessionRows(self.out_key[:k].cpu().numpy().view(np.uint64),
                           self.out_start[:k].cpu().numpy(), self.out_end[:k].cpu().numpy(),
                           self.out_val[:k].cpu().numpy(), self.out_raw[:k].cpu().numpy(),
                           self.out_cnt[:k].cpu().numpy().astype(np.int64))

    # ---- spill tier -------------------------------------------------------------------------
    def _evict(self, *, slots: torch.Tensor | None = None, idle_before: int = I64_MIN) -> None:
        """Pack slots (listed, or idle since before `idle_before`) into staging rows and
        tombstone them; the rows go to the host store. For idle evictions the host-store insert
        runs on the store's C++ worker while the next step's kernels run."""
        if slots is not None or not self.gpu:
            self._join_spill()
        else:
            # Finished jobs' results (their released keys leave the device spill set) are applied
            # before this eviction adds keys to the set. A job still running cannot release a
            # key this eviction adds: a released key was in the store when that job expired it,
            # an evicted key is resident in HBM, and a key only moves from the store back to HBM
            # through a store call that joins every queued job first (extract for a promote,
            # process for a host fold) -- whose results the poll below then applies.
            self._poll_spill()
        prev = getattr(self, "_spill_copy_done", None)
        if prev is not None:
            # The staging rows and counters are rewritten below: after the previous eviction's
            # counted copy has read them (a stream wait, no host block).
            torch.cuda.current_stream(self.device).wait_event(prev)
            self._spill_copy_done = None
        m, st, c = self.native, self._st(), self.ctr
        with self._phase("spill.capacity"):
            self._ensure_spill_capacity(slots.numel() if slots is not None
                                        else self._live_estimate)
        R = self.spill_rows
        rows = self.st_rows.view(6, R)
        rows[4].zero_()
        c[7:9].zero_()
        m.gpu_session_evict(self.nslots, self.cap_log2, self.keys_g.data_ptr(),
                            self.sess.data_ptr(), self.slot_due.data_ptr(),
                            self.slot_last.data_ptr(), idle_before,
                            slots.data_ptr() if slots is not None else 0,
                            slots.numel() if slots is not None else 0,
                            self.spill_set.data_ptr(), self.spill_set.numel() - 1,
                            rows[0].data_ptr(), rows[1].data_ptr(), rows[2].data_ptr(),
                            rows[3].data_ptr(), rows[4].data_ptr(), rows[5].data_ptr(),
                            c[7:8].data_ptr(), R, c[8:9].data_ptr(), st)
        self.spill_any = True
        if slots is None and self.gpu:
            # Idle eviction without a host round trip: the rows' count stays on the device, a
            # counted copy on a side stream moves just those rows to pinned memory, and the
            # worker applies the counts when it is joined.
            with self._phase("spill.async_launch"):
                self._evict_async(rows, R, getattr(self, "_expire_wm", None))
            return
        with self._phase("spill.evict_kernel"):
            nr_all, ne = self.ctr[7:9].cpu().tolist()
        self._live_estimate -= ne
        self._tombs_bound += ne
        nr = min(nr_all, R)
        if not nr:
            self._apply_spill((0, ne))
            return
        t0 = time.perf_counter()
        # Six contiguous DMA copies into pinned host memory; the host store reads the pinned
        # rows in place (the buffer is reused only after the insert has been joined).
        for j in range(6):
            self._pin_rows[j, :nr].copy_(rows[j, :nr], non_blocking=True)

        def host_rows():
            pin = self._pin_rows.numpy()
            h = [pin[j, :nr] for j in range(6)]
            if nr_all > R:  # staging overflowed: rows of skipped slots stay zero (cnt == 0)
                ok = h[4] > 0
                h = [np.ascontiguousarray(x[ok]) for x in h]
            return h

        torch.cuda.current_stream(self.device).synchronize()
        self.phase_s["spill.d2h"] += time.perf_counter() - t0
        h = host_rows()
        nk = int(np.count_nonzero(h[0][1:] != h[0][:-1])) + 1 if len(h[0]) else 0
        self._apply_spill((nk, ne))
        if len(h[0]):
            self.store.insert(h[0], h[1], h[2], h[3], h[4], h[5], False)

    def _evict_async(self, rows: torch.Tensor, R: int, expire_wm: int | None = None) -> None:
        """The evicted rows' counted D2H into one of two pinned slabs on the copy stream, then
        a job for the store's persistent C++ worker (csrc/sessions.cpp SessionStore.spill_submit):
        it waits for the copy's HIP event, inserts the rows and expires dead cold chunks with no
        GIL and no Python thread. Its results are applied when polled (_apply_spill_results)."""
        from .host_rows import CountedHostRows

        if getattr(self, "_spill_stream", None) is None:
            self._spill_stream = torch.cuda.Stream(self.device)
        slab = self._spill_slabs[self._spill_turn]
        self._spill_turn = (self._spill_turn + 1) % len(self._spill_slabs)
        if slab[2] > self.store.spill_completed():
            self._join_spill()  # that slab's rows are still being read by the worker

        class _Slab:  # PinnedSlabPool interface over this one slab (grows when too small)
            def take(_, nbytes):
                if slab[0] is None or slab[0].numel() < nbytes:
                    t = torch.empty(_next_pow2(nbytes), dtype=torch.uint8, pin_memory=True)
                    slab[0], slab[1] = t, t.numpy()
                    self._spill_allocs += 1
                return slab[0], slab[1]

        with self._phase("spill.async_launch.copy"):
            hr = CountedHostRows(_Slab(), [rows[j] for j in range(6)], self.ctr[7:8], [self.ctr],
                                 copy_stream=self._spill_stream if _SPILL_SIDE_STREAM else None)
        self.phase_s["spill.async_launch.take"] += hr.t_take
        self.phase_s["spill.async_launch.kernel"] += hr.t_launch
        self.metrics.extra["spill_slab_allocs"] = self._spill_allocs
        self._spill_copy_done = hr.done
        st = self._spill_stream if _SPILL_SIDE_STREAM else torch.cuda.current_stream(self.device)
        slab[2] = self.store.spill_submit(st.cuda_stream, hr.t.data_ptr(), hr.fixed_meta[0][0],
                                          [off for off, _ in hr.cols_meta], R, expire_wm)
        self.metrics.extra["spill_jobs"] = self.metrics.extra.get("spill_jobs", 0) + 1

    def _apply_spill(self, res: tuple[int, int]) -> None:
        nk, ne = res
        self.set_used += nk
        self.metrics.spilled_keys += nk
        self.metrics.freed_slots += ne

    def _join_spill(self) -> None:
        """Wait for every queued eviction job of the store's worker and apply the results."""
        if not self.gpu or self.store.spill_submitted() == 0:
            return
        with self._phase("spill.join"):
            res = self.store.spill_join()
        self._apply_spill_results(res)

    def _poll_spill(self) -> None:
        """Apply the results of eviction jobs the worker has finished (no wait)."""
        if self.gpu and self.store.spill_submitted():
            self._apply_spill_results(self.store.spill_poll())

    def _keys_to_device(self, keys: np.ndarray) -> torch.Tensor:
        """Host key ids on the device for a kernel the caller enqueues next on the current stream
        (a pageable copy of the ~3 MB released per expired chunk cost ~0.9 ms per step).

        A ring of four pinned / device buffer pairs; the copy runs on a side stream and the
        current stream waits for it. The host reuses a pinned buffer after ITS copy (side stream,
        not queued behind the step's kernels) -- copying on the current stream made the second
        call of a pipelined step wait for the fold queued ahead of it. A device buffer is
        rewritten only after the current stream's use of it (an event recorded at the next call,
        once the caller's kernel is enqueued)."""
        n = len(keys)
        dev = self.device
        ring = getattr(self, "_kh_ring", None)
        if ring is None:
            ring = self._kh_ring = [{"cap": 0, "host": None, "dev": None, "copied": None,
                                     "used": None} for _ in range(4)]
            self._kh_i = 0
            self._kh_last = None
            self._kh_side = torch.cuda.Stream(dev)
        cur = torch.cuda.current_stream(dev)
        if self._kh_last is not None:  # the previous call's kernel is enqueued by now
            ev = torch.cuda.Event()
            ev.record(cur)
            self._kh_last["used"] = ev
        slot = ring[self._kh_i]
        self._kh_i = (self._kh_i + 1) % len(ring)
        if slot["cap"] < n:
            cap = max(1 << 16, 1 << (max(n, 1) - 1).bit_length())
            if slot["copied"] is not None:
                slot["copied"].synchronize()
            slot.update(cap=cap, host=torch.empty(cap, dtype=torch.int64, pin_memory=True),
                        dev=torch.empty(cap, dtype=torch.int64, device=dev), copied=None)
        elif slot["copied"] is not None:
            slot["copied"].synchronize()  # its last copy has left the pinned buffer
        slot["host"][:n].numpy()[:] = keys
        side = self._kh_side
        if slot["used"] is not None:
            side.wait_event(slot["used"])  # the device buffer's last reader is done
        with torch.cuda.stream(side):
            slot["dev"][:n].copy_(slot["host"][:n], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(side)
        slot["copied"] = ev
        cur.wait_event(ev)
        self._kh_last = slot
        return slot["dev"][:n]

    def _apply_spill_results(self, res: list) -> None:
        for r in res:
            rel = r["released"]
            if len(rel) and self.spill_any:
                # keys of expired cold chunks leave the device spill set
                kt = self._keys_to_device(rel)
                self.native.gpu_set_erase(self.spill_set.data_ptr(), self.spill_set.numel() - 1,
                                          kt.data_ptr(), kt.numel(), self._st())
            self._live_estimate -= r["ne"]
            self._tombs_bound += r["ne"]
            self.set_used += r["nr"]
            self.metrics.freed_slots += r["ne"]
            self.metrics.spilled_keys += r["nk"]
            for k in ("wait", "hot", "build", "index", "publish", "expire"):  # worker phase times
                self.phase_s[f"spill.worker.{k}"] += r[f"t_{k}"]
            self.phase_s["spill.worker.index.populate"] += r["t_populate"]
            ex = self.metrics.extra  # rows the worker could not take the all-cold path for
            ex["spill_hot_rows"] = ex.get("spill_hot_rows", 0) + r["n_hot"]
            ex["spill_jobs_with_hot_map"] = ex.get("spill_jobs_with_hot_map", 0) + r["hot_keys"]

    def _ensure_spill_capacity(self, extra: int) -> None:
        """Keep the device spill set (live keys + tombstones) at most half full after `extra`
        more insertions; otherwise rebuild it from the store's keys at a larger size."""
        cap = self.spill_set.numel()
        if self.set_used + extra <= cap // 2:
            return
        want = 4 * (self.store.num_keys() + extra)
        self._rehash_spill_set(max(16, _next_pow2(max(1, want)).bit_length() - 1))

    def _rehash_spill_set(self, log2: int) -> None:
        """Grow the device spill set (dropping its tombstones) on the GPU: the live keys of the
        old set are re-inserted into a fresh one (no host walk of the store, no H2D copy)."""
        t0 = time.perf_counter()
        old = self.spill_set
        self.spill_log2 = log2
        self.spill_set = torch.full((1 << log2,), EMPTY_KEY, dtype=torch.int64, device=self.device)
        self.native.gpu_set_rehash(old.data_ptr(), old.numel(), self.spill_set.data_ptr(),
                                   (1 << log2) - 1, self._st())
        # Live keys of the set = the store's keys (+ keys evicted by a still-queued insert,
        # which the worker adds to the store; num_keys() is an upper bound after the join).
        self.set_used = self.store.num_keys()
        self.spill_any = self.spill_any or self.set_used > 0
        self.phase_s["spill.set_rebuild"] += time.perf_counter() - t0

    def _rebuild_spill_set(self, log2: int) -> None:
        """Rebuild the device spill set from the host store's keys (restore)."""
        t0 = time.perf_counter()
        arr = self.store.spill_set(log2)
        self.spill_log2 = log2
        self.spill_set = torch.from_numpy(arr).to(self.device)
        self.set_used = self.store.num_keys()
        self.spill_any = self.set_used > 0
        self.phase_s["spill.set_rebuild"] += time.perf_counter() - t0

    def _rehash(self) -> None:
        self._occ_pending = None  # counts of the old table
        m, st = self.native, self._st()
        old = (self.keys_g, self.sess, self.slot_due, self.slot_last)
        self._alloc_state()
        self.ctr[9:10].zero_()
        m.gpu_session_rehash(self.nslots, self.cap_log2, *(t.data_ptr() for t in old),
                             self.keys_g.data_ptr(), self.sess.data_ptr(),
                             self.slot_due.data_ptr(), self.slot_last.data_ptr(),
                             self.ctr[9:10].data_ptr(), st)
        self.metrics.rehashes += 1

    def _count_occupancy(self) -> tuple[int, int]:
        """Exact (live, occupied) slot counts: a table scan and a host sync."""
        k = self.keys_g
        with self._phase("spill.occupancy"):
            live, occupied = torch.stack([((k != EMPTY_KEY) & (k != TOMB_KEY)).sum(),
                                          (k != EMPTY_KEY).sum()]).tolist()
        self._live_estimate, self._tombs_bound = int(live), int(occupied - live)
        self._occ_exact = False
        return int(live), int(occupied)

    def _occ_launch(self) -> None:
        k = self.keys_g
        if getattr(self, "_occ_pin", None) is None:
            self._occ_pin = torch.zeros(2, dtype=torch.int64, pin_memory=True)
        c = torch.stack([((k != EMPTY_KEY) & (k != TOMB_KEY)).sum(), (k != EMPTY_KEY).sum()])
        self._occ_pin.copy_(c, non_blocking=True)
        # estimates at the launch: the landed exact counts are corrected by what changed since
        self._occ_base = (self._live_estimate, self._tombs_bound)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.device))
        self._occ_pending = ev

    def _occ_poll(self):
        """(live, occupied) of a count launched earlier, once it has landed (else None)."""
        ev = self._occ_pending
        if ev is None or not ev.query():
            return None
        self._occ_pending = None
        live, occupied = self._occ_pin.tolist()
        return int(live), int(occupied)

    def _maybe_spill(self, wm: int, inflight: bool = False) -> None:
        """inflight: a fold is enqueued ahead of this check (pipelined step) -- a due rehash
        waits for the next step (_rehash_if_due)."""
        # Live keys come from the kernels' insert / evict counters; the table is scanned only
        # after a restore and when the tombstone bound suggests a rehash.
        # Rehash (drop tombstones) once live + tombstones pass 0.8 of the slots with at least 8 %
        # tombstones: evicted keys leave tombstones that new keys only partly reuse, and the
        # LDS probes of the fold (a missing key scans to the first empty slot) grow with the
        # occupied fraction, not with the live one.
        def due(live, occupied):
            return (occupied > _REHASH_OCC * self.nslots
                    and occupied - live > _REHASH_TOMBS * self.nslots)

        self._poll_spill()
        t_occ = time.perf_counter()

        def rehash():
            if inflight:
                self._rehash_due = True
            else:
                self._rehash()
                self._tombs_bound = 0

        if self._rehash_due:
            live = self._live_estimate  # a rehash is already queued for the next step
        elif self._occ_exact:
            live, occupied = self._count_occupancy()
            if due(live, occupied):
                rehash()
        else:
            # The tombstone bound only grows (new keys reuse tombstones unseen), so the exact
            # counts are taken without a host wait: launched when the bound suggests a rehash and
            # read at a later step once they have landed (a one-step-late rehash decision).
            live = self._live_estimate
            stale = self._occ_poll()
            if stale is not None and due(*stale):
                rehash()
            elif stale is not None:
                # Not due: tighten the estimates from the exact counts (plus the inserts and
                # evictions counted since the launch), so the bound stops re-launching the scan
                # every step until a rehash.
                live0, tombs0 = self._occ_base
                self._live_estimate = stale[0] + (self._live_estimate - live0)
                self._tombs_bound = (stale[1] - stale[0]) + (self._tombs_bound - tombs0)
                live = self._live_estimate
            elif due(live, live + self._tombs_bound) and self._occ_pending is None:
                self._occ_launch()
        self.phase_s["spill.occupancy_logic"] += time.perf_counter() - t_occ
        if live > self.max_load * self.nslots and wm > I64_MIN:
            # LRU by last event time: keys idle for idle_spill_ms move to host DRAM (keys with no
            # live session are simply freed).
            self._evict(idle_before=wm - self.idle_spill_ms)
        # Store empty again: clear the device set (drops its tombstones) and skip set probes.
        if (self.spill_any and self.store.spill_completed() == self.store.spill_submitted()
                and self.store.num_keys() == 0):
            self.spill_set.fill_(EMPTY_KEY)
            self.set_used = 0
            self.spill_any = False

    # ---- inspection -------------------------------------------------------------------------
    def resident_keys(self) -> int:
        self._sync_pending()
        if not self.gpu:
            return 0
        k = self.keys_g
        return int(((k != EMPTY_KEY) & (k != TOMB_KEY)).sum().item())

    def snapshot(self) -> dict:
        """All live sessions (both tiers) as host columns key/start/end/acc/cnt/flags. Pipelined:
        the pending step is applied first (its fired rows come with the next call -- a caller
        that checkpoints calls flush() before and emits them)."""
        self._sync_pending()
        if self.gpu:
            self._join_spill()
        names = ("key", "start", "end", "acc", "cnt", "flags")
        if not self.gpu:
            return self.store.snapshot()
        # Live HBM sessions selected on the device (session-index-major, then slot); only their
        # rows cross to the host, straight into the tail of the store's snapshot columns.
        keys = self.keys_g
        rec = self.sess.view(self.nslots, K_SESS, 4)
        live = ((keys != EMPTY_KEY) & (keys != TOMB_KEY))[None, :] & \
            ((rec[:, :, 3] & 0xFFFFFFFF) > 0).t()
        j, s = live.nonzero(as_tuple=True)
        n_dev = int(s.numel())
        out = self.store.snapshot(n_dev)
        if n_dev:
            n0 = len(out["key"]) - n_dev
            r = rec[s, j]
            cols = (keys[s], r[:, 0], r[:, 1], r[:, 2], r[:, 3] & 0xFFFFFFFF, r[:, 3] >> 32)
            for f, t in zip(names, cols):
                torch.from_numpy(out[f][n0:]).copy_(t, non_blocking=True)
            torch.cuda.current_stream(keys.device).synchronize()
        return out

    # ---- checkpoint / restore (runtime/checkpoint.py) --------------------------------------
    def owned_key_groups(self) -> tuple[int, int]:
        from .checkpoint import owned_key_groups

        return owned_key_groups(self.rank, self.world, self.parallelism, self.max_parallelism)

    def snapshot_state(self):
        """Every live session of both tiers (HBM slots and the host store), by key group."""
        from .checkpoint import OperatorSnapshot

        snap = self.snapshot()
        keys = torch.from_numpy(np.ascontiguousarray(snap["key"], dtype=np.int64))
        kg = K.keygroups(keys, max_parallelism=self.max_parallelism).numpy()
        cols = {k: np.ascontiguousarray(snap[k], dtype=np.int64)
                for k in ("key", "start", "end", "acc", "cnt", "flags")}
        meta = {"kind": "session", "gap": self.gap, "lateness": self.lateness, "agg": self.agg,
                "wm": self.wm, "metrics": {k: v for k, v in self.metrics.__dict__.items()
                                           if isinstance(v, int)}}
        return OperatorSnapshot(kg, cols, meta)

    def restore_state(self, rows: dict, meta: dict) -> None:
        """Restored sessions go to the HBM slot table (keys with <= kSess sessions) or to the
        host store (the rest), exactly like state that overflowed during processing."""
        for k in ("gap", "agg"):
            if meta[k] != getattr(self, k):
                raise ValueError(f"checkpoint {k} does not match the operator")
        self._pend, self._carry, self._rehash_due = None, [], False
        self.wm = meta["wm"]
        for k, v in meta.get("metrics", {}).items():
            setattr(self.metrics, k, v)
        self.store = self.native.SessionStore(self.gap, self.lateness, self.agg, _STORE_SHARDS)
        if self.gpu:
            self._occ_exact = True  # slots written below: the next check scans the table
        cols = [np.ascontiguousarray(rows[k], dtype=np.int64)
                for k in ("key", "start", "end", "acc", "cnt", "flags")]
        if not self.gpu:
            if len(cols[0]):
                self.store.insert(*cols, False)
            return
        self._join_spill()
        self._alloc_state()
        self.spill_set.fill_(EMPTY_KEY)
        self.set_used, self.spill_any = 0, False
        if not len(cols[0]):
            return
        key = cols[0]
        order = np.argsort(key, kind="stable")
        cols = [c[order] for c in cols]
        key = cols[0]
        uniq, first, counts = np.unique(key, return_index=True, return_counts=True)
        pos = np.arange(len(key)) - np.repeat(first, counts)  # session index within its key
        many = np.repeat(counts > K_SESS, counts)
        if many.any():  # more sessions than an HBM slot holds: host tier
            self.store.insert(*[c[many] for c in cols], False)
        dev = self.device
        fit_keys = uniq[counts <= K_SESS]
        if len(fit_keys):
            slots_u = K.table_insert(torch.from_numpy(fit_keys).to(dev), self.keys_g,
                                     nsub_log2=self.nsub_log2, cap_log2=self.cap_log2)
            if bool((slots_u < 0).any()):
                raise RuntimeError("restore: session keys do not fit the slot table")
            sel = ~many
            slot_of = dict(zip(fit_keys.tolist(), slots_u.cpu().tolist()))
            slot = np.array([slot_of[k] for k in key[sel].tolist()], dtype=np.int64)
            rec = np.zeros((len(slot), 4), dtype=np.int64)
            rec[:, 0], rec[:, 1], rec[:, 2] = cols[1][sel], cols[2][sel], cols[3][sel]
            rec[:, 3] = (cols[4][sel] & 0xFFFFFFFF) | (cols[5][sel] << 32)
            view = self.sess.view(self.nslots * K_SESS, 4)
            dst = torch.from_numpy(slot * K_SESS + pos[sel]).to(dev)
            view[dst] = torch.from_numpy(rec).to(dev)
            # Due times: recomputed by one fire sweep at the restored watermark; mark all due now.
            self.slot_due[torch.from_numpy(np.unique(slot)).to(dev)] = I64_MIN
        if len(self.store.key_list()):
            self._rebuild_spill_set(max(16, _next_pow2(4 * self.store.num_keys()).bit_length() - 1))
