"""Host-DRAM tier half of the keyed window operator (runtime/window_operator.py): the spill
check, window_compact evictions (grouped by pane on the GPU, counted D2H on the copy stream,
absorbed into the C++ tier of runtime/window_spill.py), and tiered firings that merge the tier's
rows of a window with the device's rows on the GPU (tier_merge + fused fire epilogue).

BASELINE north star: keyed state with spill to host DRAM; SURVEY.md 5.7.
"""
from __future__ import annotations

import numpy as np
import torch

from ..ops import expr as E
from ..ops import kernels as K
from .host_rows import CountedHostRows, PinnedSlabPool, _next_pow2, to_host_arrays
from .window_types import FireResult, _PendingFire, _agg_identity

I64_MIN = K.I64_MIN
I64_MAX = K.I64_MAX

import os as _os

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


class _TierMixin:
    """Methods of KeyedWindowOperator (mixed in; state lives on the operator)."""

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
        ex = self.host_tier.export(p0, p1, dev)
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
