"""Firing half of the keyed window operator (runtime/window_operator.py KeyedWindowOperator):
due windows -> fire kernels (single, batched multi-window, fused dirty-pane re-firing) -> counted
D2H of the fired rows into pinned slabs -> FireResult rows in firing order; late re-firing and
pane purging after a watermark advance. The window arithmetic and the firing cursor are C++
(csrc/window_control.h, through self._ctl); these methods drive the kernels and the host rows.

Reference semantics: BandwidthMonitorWithEventTime.java:45-55 (event-time sliding window, the
Mbps map and filter fused into the fire kernel), chapter3/README.md:209-228 (allowed lateness:
re-firing until maxTimestamp + lateness <= watermark, then cleanup).
"""
from __future__ import annotations

import os as _os

import numpy as np
import torch

from ..ops import expr as E
from ..ops import kernels as K
from .host_rows import CountedHostRows, to_host_arrays
from .window_types import FireResult, _PendingFire

I64_MIN = K.I64_MIN
I64_MAX = K.I64_MAX


class _FireMixin:
    """Methods of KeyedWindowOperator (mixed in; state lives on the operator)."""

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
                and type(self)._fire_window is _FireMixin._fire_window)

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
