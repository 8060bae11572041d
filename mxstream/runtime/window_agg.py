"""State-update half of the keyed window operator (runtime/window_operator.py): bucket and
exchange buffers, key-group ownership tables, the G > 1 combiner (pre-aggregation of the
partitioned records before the all-to-all), the equal-split exchange, the window_agg launch into
the pane ring, and ring growth.

Reference semantics: BandwidthMonitorWithEventTime.java:45-47 (keyBy -> sliding window reduce);
Flink's key-group assignment murmur(hash) % maxParallelism * P / maxParallelism.
"""
from __future__ import annotations

import math
import os as _os

import torch

from ..ops import kernels as K
from .host_rows import _host_wait, _next_pow2

I64_MIN = K.I64_MIN
I64_MAX = K.I64_MAX



# > 1: every sub-table's records split over this many workgroups even when none is hot (dense
# ids, additive aggregates: partial sums merge with atomic adds) -- more workgroups than CUs
# (A/B, MXS_AGG_FORCE_SPLIT).
_FORCE_SPLIT = int(_os.environ.get("MXS_AGG_FORCE_SPLIT", "0"))

class _AggMixin:
    """Methods of KeyedWindowOperator (mixed in; state lives on the operator)."""

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
        per_wg = self._part_ranks * self.bucket_cap
        if _FORCE_SPLIT > 1 and self.dense_bits and self._part_ranks == 1 and self.dlist is None:
            per_wg = -(-self.bucket_cap // _FORCE_SPLIT)  # forced split: a share per workgroup
        return (self.agg in (K.AGG_SUM_I64, K.AGG_AVG_I64) and rw <= 2 and not self.combine
                and per_wg < 65536 and _os.environ.get("MXS_AGG_PACK", "1") != "0")

    def _zero_pane(self, so: int, k: int = 1) -> None:
        """Reset k consecutive pane slabs starting at slot index `so` (pane-major state)."""
        e = so + k * self.nslots
        self.acc_g[so:e].zero_()
        self.cnt_g[so:e].zero_()
        self.dirty_g[so:e].zero_()
