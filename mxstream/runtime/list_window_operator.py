"""Keyed windows that need every element (``process`` windows: ComputeCpuMiddle.java:34-48).

Flink keeps a ListState per (key, window) and hands the full Iterable to the ProcessWindowFunction.
Here the elements live in a **device pane arena** (csrc/mxs_listwin.h): pane = gcd(size, slide),
a power-of-two ring of pane slots, each an append buffer of (key, f64 bits) on the device.

* ``process``: one readback of the batch's timestamp/key range (ring sizing), one of its
  per-pane counts (``lw_pane_count``: buffer growth), then ``lw_pane_scatter`` appends every
  element to its pane with one global cursor atomic per touched pane per workgroup. Elements
  older than the allowed lateness are dropped (counted).
* the append also records each element's rank among its key's elements of the pane (per-pane
  per-key counts, dense key ranges up to 16 Mi ids), so a firing needs no atomics: per-key
  totals and per-pane prefixes from the panes' counts (``lw_rank_prefix``), the order-preserving
  scan of the totals (``lw_scan``: offsets + the non-empty keys in key order), every element
  placed at segment start + prefix + rank (``lw_rank_scatter``, as order bits), and each
  segment's median selected in LDS (``segment_median_select``). Panes without ranks (wide key
  ranges, restored panes) fire through a counting sort with atomics (``lw_key_count`` /
  ``lw_key_scatter``); key ranges over 16 Mi ids are mapped to dense ids first. No comparison
  sort of the window, no per-pane host loop.
* late-but-allowed data re-fires the already fired windows of its panes for the keys it touched
  (EventTimeTrigger.onElement per key).
* ``snapshot_state`` / ``restore_state``: the live panes' elements as rows (pane, key, value).

CPU (device="cpu") runs the same arena through the C++ twins (csrc/listwin_cpu.cpp).
"""
from __future__ import annotations

import math

import numpy as np
import torch

from ..ops import kernels as K
from ..ops.native import load
from .window_operator import OperatorMetrics

I64_MIN, I64_MAX = K.I64_MIN, K.I64_MAX
_MAX_DENSE = 1 << 24  # key range of the direct counting sort


def _next_pow2(x: int) -> int:
    return 1 << max(0, int(x - 1).bit_length())


class KeyedListWindowOperator:
    def __init__(self, *, size: int, slide: int | None = None, offset: int = 0,
                 lateness: int = 0, device="cpu", time_mode: str = "event", func: str = "median"):
        slide = size if slide is None else slide
        if func != "median":
            raise ValueError("supported list-window functions: median")
        self.size, self.slide, self.offset, self.lateness = int(size), int(slide), int(offset), int(lateness)
        self.pane = math.gcd(self.size, self.slide)
        self.ppw = self.size // self.pane
        self.device = K.resolve_device(device)
        self.cuda = self.device.type == "cuda"
        self.time_mode = time_mode
        self.wm = I64_MIN
        self.next_fire_start: int | None = None
        self.metrics = OperatorMetrics()
        self.late_side: list = []
        self._m = load()
        self._ctl = self._m.WindowControl(self.size, self.slide, self.offset, self.lateness)
        # Pane arena: ring slot -> absolute pane id (or None), buffers, fill, key range.
        self.ring = _next_pow2(self.ppw + -(-self.lateness // self.pane) + 2)
        self._alloc_ring(self.ring)

    # ---- arena -----------------------------------------------------------------------------
    def _alloc_ring(self, ring: int) -> None:
        self.ring = ring
        self.slot_pane: list[int | None] = [None] * ring
        self.kbuf: list[torch.Tensor | None] = [None] * ring
        self.vbuf: list[torch.Tensor | None] = [None] * ring
        self.fill = [0] * ring
        self.krange: list[tuple[int, int] | None] = [None] * ring
        # Ranked slots: per-element rank among the key's elements of the pane (rbuf) and the
        # per-key counts over [kbase, kbase + numel) (kcnt): the firing places elements without
        # atomics. A slot whose key range grows past _MAX_DENSE (or was restored) is unranked.
        self.rbuf: list[torch.Tensor | None] = [None] * ring
        self.kcnt: list[torch.Tensor | None] = [None] * ring
        self.kbase = [0] * ring
        self.ranked = [True] * ring
        self._tab = torch.zeros(5 * ring, dtype=torch.int64, device=self.device)
        self._tab_dirty = True

    @property
    def panes(self) -> dict:
        """Live pane ids -> element count (inspection / tests)."""
        return {p: self.fill[r] for r, p in enumerate(self.slot_pane) if p is not None}

    def _slot_of(self, p: int) -> int:
        return p & (self.ring - 1)

    def _live_range(self):
        live = [p for p in self.slot_pane if p is not None]
        return (min(live), max(live)) if live else None

    _SLOT_FIELDS = ("slot_pane", "kbuf", "vbuf", "fill", "krange", "rbuf", "kcnt", "kbase",
                    "ranked")

    def _regrow_ring(self, need_lo: int, need_hi: int) -> None:
        """Re-lay the ring so panes need_lo..need_hi fit without aliasing (keeps buffers)."""
        old = [[getattr(self, f)[r] for f in self._SLOT_FIELDS]
               for r, p in enumerate(self.slot_pane) if p is not None]
        self._alloc_ring(_next_pow2(need_hi - need_lo + 1))
        for vals in old:
            r = self._slot_of(vals[0])
            for f, v in zip(self._SLOT_FIELDS, vals):
                getattr(self, f)[r] = v

    def _ensure_key_range(self, r: int, kmin: int, kmax: int) -> None:
        """The slot's per-key counts cover [kmin, kmax] (grown by copy), or the slot stops
        recording ranks when its key range would exceed _MAX_DENSE ids."""
        if not self.ranked[r]:
            return
        kc = self.kcnt[r]
        lo, hi = (kmin, kmax) if kc is None else (min(kmin, self.kbase[r]),
                                                 max(kmax, self.kbase[r] + kc.numel() - 1))
        if hi - lo + 1 > _MAX_DENSE:
            self.ranked[r] = False
            self.kcnt[r] = None
            self._tab_dirty = True
            return
        if kc is not None and lo == self.kbase[r] and hi - lo + 1 <= kc.numel():
            return
        size = _next_pow2(hi - lo + 1) if kc is None else max(_next_pow2(hi - lo + 1), kc.numel())
        size = min(size, _MAX_DENSE) if hi - lo + 1 <= _MAX_DENSE else hi - lo + 1
        nc = torch.zeros(size, dtype=torch.int32, device=self.device)
        if kc is not None:
            o = self.kbase[r] - lo
            nc[o:o + kc.numel()].copy_(kc)
        self.kcnt[r], self.kbase[r] = nc, lo
        self._tab_dirty = True

    def _ensure_capacity(self, r: int, extra: int) -> None:
        need = self.fill[r] + extra
        kb = self.kbuf[r]
        if kb is not None and kb.numel() >= need:
            return
        cap = _next_pow2(max(need, 1 << 12))
        nk = torch.empty(cap, dtype=torch.int64, device=self.device)
        nv = torch.empty(cap, dtype=torch.int64, device=self.device)
        nr = torch.empty(cap, dtype=torch.int32, device=self.device)
        f = self.fill[r]
        if kb is not None and f:
            nk[:f].copy_(kb[:f])
            nv[:f].copy_(self.vbuf[r][:f])
            nr[:f].copy_(self.rbuf[r][:f])
        self.kbuf[r], self.vbuf[r], self.rbuf[r] = nk, nv, nr
        self._tab_dirty = True

    def _sync_tab(self) -> None:
        if not self._tab_dirty:
            return
        R = self.ring
        addr = [0] * (5 * R)
        for r in range(R):
            if self.kbuf[r] is not None:
                addr[r] = self.kbuf[r].data_ptr()
                addr[R + r] = self.vbuf[r].data_ptr()
                addr[2 * R + r] = self.rbuf[r].data_ptr()
            if self.ranked[r] and self.kcnt[r] is not None:
                addr[3 * R + r] = self.kcnt[r].data_ptr()
                addr[4 * R + r] = self.kbase[r]
        self._tab.copy_(torch.tensor(addr, dtype=torch.int64))
        self._tab_dirty = False

    def _stream(self) -> int:
        return torch.cuda.current_stream(self.device).cuda_stream if self.cuda else 0

    # ---- window arithmetic ----------------------------------------------------------------
    # Flink window arithmetic: the shared C++ implementation (csrc/window_control.h).
    def _pane_of(self, t):
        return self._ctl.pane_of(t)

    def _late_ts(self) -> int:
        return self._ctl.late_ts(self.wm, self.time_mode == "event")

    def _align_up(self, t: int) -> int:
        return self._ctl.align_up(t)

    def _first_start_containing(self, t: int) -> int:
        return self._ctl.first_start_containing(t)

    # ---- ingest ---------------------------------------------------------------------------
    def process(self, keys: torch.Tensor, ts: torch.Tensor, vals_f64: torch.Tensor) -> list:
        """keys int64 (or int32 dictionary ids), ts int64, vals: f64 bit patterns (int64).
        Returns fired rows (window_start, window_end, keys, medians) of late re-firings."""
        n = keys.numel()
        if n == 0:
            return []
        keys = keys.to(torch.int64).contiguous()
        ts = ts.contiguous()
        vals_f64 = vals_f64.contiguous()
        late_ts = self._late_ts()
        # Readback 1: timestamp and key range of the batch (ring sizing, dense key range).
        tmin, tmax, kmin, kmax = torch.stack([ts.min(), ts.max(), keys.min(), keys.max()]).tolist()
        lo_t = max(tmin, late_ts) if late_ts > I64_MIN else tmin
        if lo_t > tmax:  # everything late
            self.metrics.num_late_records_dropped += n
            return []
        plo, phi = self._pane_of(lo_t), self._pane_of(tmax)
        live = self._live_range()
        need_lo, need_hi = (plo, phi) if live is None else (min(plo, live[0]), max(phi, live[1]))
        if need_hi - need_lo + 1 > self.ring:
            self._regrow_ring(need_lo, need_hi)
        R, st = self.ring, self._stream()
        counts = torch.zeros(R + 1, dtype=torch.int64, device=self.device)
        self._m.lw_pane_count(self.cuda, ts.data_ptr(), n, self.offset, self.pane, R, late_ts,
                              counts.data_ptr(), st)
        # Readback 2: elements per ring slot (buffer growth) + late count.
        hc = counts.tolist()
        self.metrics.num_late_records_dropped += hc[R]
        self.metrics.num_records_in += n - hc[R]
        touched_panes = []
        for r in range(R):
            if not hc[r]:
                continue
            p = plo + ((r - plo) & (R - 1))  # the batch's pane in ring slot r
            if self.slot_pane[r] is not None and self.slot_pane[r] != p:
                raise RuntimeError("list window: pane ring aliasing")  # sizing above prevents it
            self.slot_pane[r] = p
            self._ensure_capacity(r, hc[r])
            kr = self.krange[r]
            self.krange[r] = (kmin, kmax) if kr is None else (min(kr[0], kmin), max(kr[1], kmax))
            self._ensure_key_range(r, kmin, kmax)
            touched_panes.append(p)
        self._sync_tab()
        cursor = torch.tensor(self.fill, dtype=torch.int64).to(self.device, non_blocking=True)
        self._m.lw_pane_scatter(self.cuda, keys.data_ptr(), ts.data_ptr(), vals_f64.data_ptr(), n,
                                self.offset, self.pane, R, late_ts, self._tab.data_ptr(),
                                cursor.data_ptr(), st)
        for r in range(R):
            self.fill[r] += hc[r]
        if not touched_panes:
            return []
        first = self._first_start_containing(self.offset + min(touched_panes) * self.pane)
        if self.wm > I64_MIN:
            first = max(first, self._align_up(self.wm - self.size + 2))
        self.next_fire_start = first if self.next_fire_start is None else min(self.next_fire_start, first)
        out = []
        # Late-but-allowed data: re-fire, for the keys that received it, the windows that
        # already fired and contain those panes (EventTimeTrigger.onElement per key).
        if self.wm > I64_MIN:
            fired_panes = [p for p in touched_panes
                           if self._first_start_containing(self.offset + p * self.pane)
                           + self.size - 1 <= self.wm]
            if fired_panes:
                pcol = torch.div(ts - self.offset, self.pane, rounding_mode="floor")
                for p in sorted(fired_panes):
                    touched = torch.unique(keys[pcol == p])
                    s = self._first_start_containing(self.offset + p * self.pane)
                    while s <= self.offset + p * self.pane:
                        if s + self.size - 1 <= self.wm < s + self.size - 1 + self.lateness:
                            out += self._fire_window(s, only_keys=touched)
                        s += self.slide
        return out

    # ---- firing -----------------------------------------------------------------------------
    def advance_watermark(self, wm: int) -> list:
        if wm <= self.wm:
            return []
        self.wm = wm
        out = []
        if self.next_fire_start is not None:
            s = self.next_fire_start
            live = self._live_range()
            last_pane = live[1] if live else None
            # Windows after the last pane hold no data: never iterate past it (wm may be MAX).
            while s + self.size - 1 <= wm and last_pane is not None \
                    and self._pane_of(s) <= last_pane:
                out += self._fire_window(s)
                s += self.slide
            if s + self.size - 1 <= wm:  # caught up: resume at the first window not yet due
                s = self._align_up(wm - self.size + 2) if wm < I64_MAX - self.size else s
            self.next_fire_start = s
        self._purge()
        return out

    def _purge(self) -> None:
        if self.wm == I64_MAX:
            keep_from = None
        else:
            keep_from = self._pane_of(self._align_up(self.wm - self.size - self.lateness + 2))
        for r, p in enumerate(self.slot_pane):
            if p is not None and (keep_from is None or p < keep_from):
                self.slot_pane[r] = None
                self.fill[r] = 0
                self.krange[r] = None
                self.kcnt[r] = None  # a new pane in this slot starts its counts afresh
                self.ranked[r] = True
                self._tab_dirty = True

    def _window_panes(self, s: int) -> list[int]:
        p0 = self._pane_of(s)
        out = []
        for p in range(p0, p0 + self.ppw):
            r = self._slot_of(p)
            if self.slot_pane[r] == p and self.fill[r]:
                out.append(r)
        return out

    def _fire_window(self, s: int, only_keys: torch.Tensor | None = None) -> list:
        slots = self._window_panes(s)
        if not slots:
            return []
        self.metrics.num_fires += 1
        total = sum(self.fill[r] for r in slots)
        kmin = min(self.krange[r][0] for r in slots)
        kmax = max(self.krange[r][1] for r in slots)
        ranked = len(slots) <= 32 and all(self.ranked[r] and self.kcnt[r] is not None
                                          for r in slots)
        if ranked:
            rlo = min(self.kbase[r] for r in slots)
            rhi = max(self.kbase[r] + self.kcnt[r].numel() for r in slots)
            ranked = rhi - rlo <= _MAX_DENSE
        if ranked:
            keys_out, med = self._median_ranked(slots, rlo, rhi - rlo, total)
        elif kmin >= 0 and kmax - kmin < _MAX_DENSE and len(slots) <= 64:
            keys_out, med = self._median_dense(slots, kmin, kmax - kmin + 1, total)
        else:
            keys_out, med = self._median_mapped(slots)
        if only_keys is not None:
            sel = torch.isin(keys_out, only_keys.to(keys_out.device))
            keys_out, med = keys_out[sel], med[sel]
        if not keys_out.numel():
            return []
        self.metrics.num_records_out += int(keys_out.numel())
        return [(s, s + self.size, keys_out.cpu().numpy(), med.cpu().numpy())]

    def _median_ranked(self, slots, kmin: int, nk: int, total: int):
        """Ranked firing: per-key totals and per-pane prefixes from the panes' counts, the
        order-preserving scan, then every element placed at segment start + prefix + rank (no
        atomics), then the per-segment median."""
        m, st, dev = self._m, self._stream(), self.device
        panes = [(self.kbuf[r].data_ptr(), self.vbuf[r].data_ptr(), self.rbuf[r].data_ptr(),
                  self.kcnt[r].data_ptr(), self.kbase[r], self.kcnt[r].numel(), self.fill[r])
                 for r in slots]
        tot = torch.empty(nk, dtype=torch.int32, device=dev)
        pre = torch.empty(len(slots) * nk, dtype=torch.int32, device=dev)
        m.lw_rank_prefix(self.cuda, panes, kmin, nk, tot.data_ptr(), pre.data_ptr(), st)
        offs = torch.empty(nk + 1, dtype=torch.int64, device=dev)
        heads = torch.empty(nk, dtype=torch.int64, device=dev)
        hkeys = torch.empty(nk, dtype=torch.int64, device=dev)
        nh = torch.zeros(1, dtype=torch.int64, device=dev)
        scratch = torch.empty(max(16, m.lw_scan_scratch_bytes(nk)), dtype=torch.uint8, device=dev)
        m.lw_scan(self.cuda, tot.data_ptr(), nk, kmin, scratch.data_ptr(), offs.data_ptr(),
                  heads.data_ptr(), hkeys.data_ptr(), nh.data_ptr(), st)
        ordv = torch.empty(max(total, 1), dtype=torch.int64, device=dev)
        m.lw_rank_scatter(self.cuda, panes, kmin, nk, offs.data_ptr(), pre.data_ptr(),
                          ordv.data_ptr(), st)
        k = int(nh.item())
        med = torch.empty(k, dtype=torch.float64, device=dev)
        if k:
            args = (heads.data_ptr(), k, total, ordv.data_ptr(), med.data_ptr())
            if self.cuda:
                m.gpu_segment_median_select(*args, st)
            else:
                m.cpu_segment_median_select(*args)
        return hkeys[:k], med

    def _median_dense(self, slots, kmin: int, nk: int, total: int):
        m, st, dev = self._m, self._stream(), self.device
        panes = [(self.kbuf[r].data_ptr(), self.vbuf[r].data_ptr(), self.fill[r]) for r in slots]
        counts = torch.zeros(nk, dtype=torch.int32, device=dev)
        m.lw_key_count(self.cuda, panes, kmin, nk, counts.data_ptr(), st)
        offs = torch.empty(nk + 1, dtype=torch.int64, device=dev)
        heads = torch.empty(nk, dtype=torch.int64, device=dev)
        hkeys = torch.empty(nk, dtype=torch.int64, device=dev)
        nh = torch.zeros(1, dtype=torch.int64, device=dev)
        scratch = torch.empty(max(16, m.lw_scan_scratch_bytes(nk)), dtype=torch.uint8, device=dev)
        m.lw_scan(self.cuda, counts.data_ptr(), nk, kmin, scratch.data_ptr(), offs.data_ptr(),
                  heads.data_ptr(), hkeys.data_ptr(), nh.data_ptr(), st)
        cursor = offs[:nk].clone()
        ordv = torch.empty(max(total, 1), dtype=torch.int64, device=dev)
        m.lw_key_scatter(self.cuda, panes, kmin, cursor.data_ptr(), ordv.data_ptr(), st)
        k = int(nh.item())
        med = torch.empty(k, dtype=torch.float64, device=dev)
        if k:
            args = (heads.data_ptr(), k, total, ordv.data_ptr(), med.data_ptr())
            if self.cuda:
                m.gpu_segment_median_select(*args, st)
            else:
                m.cpu_segment_median_select(*args)
        return hkeys[:k], med

    def _median_mapped(self, slots):
        """Keys outside a dense id range: dense ids by torch.unique, then the same firing."""
        keys = torch.cat([self.kbuf[r][:self.fill[r]] for r in slots])
        vals = torch.cat([self.vbuf[r][:self.fill[r]] for r in slots])
        uniq, ids = torch.unique(keys, return_inverse=True)
        ids = ids.to(torch.int64).contiguous()
        vals = vals.contiguous()
        m, st, dev = self._m, self._stream(), self.device
        n, nk = ids.numel(), uniq.numel()
        panes = [(ids.data_ptr(), vals.data_ptr(), n)]
        counts = torch.zeros(nk, dtype=torch.int32, device=dev)
        m.lw_key_count(self.cuda, panes, 0, nk, counts.data_ptr(), st)
        offs = torch.empty(nk + 1, dtype=torch.int64, device=dev)
        heads = torch.empty(nk, dtype=torch.int64, device=dev)
        hkeys = torch.empty(nk, dtype=torch.int64, device=dev)
        nh = torch.zeros(1, dtype=torch.int64, device=dev)
        scratch = torch.empty(max(16, m.lw_scan_scratch_bytes(nk)), dtype=torch.uint8, device=dev)
        m.lw_scan(self.cuda, counts.data_ptr(), nk, 0, scratch.data_ptr(), offs.data_ptr(),
                  heads.data_ptr(), hkeys.data_ptr(), nh.data_ptr(), st)
        cursor = offs[:nk].clone()
        ordv = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
        m.lw_key_scatter(self.cuda, panes, 0, cursor.data_ptr(), ordv.data_ptr(), st)
        med = torch.empty(nk, dtype=torch.float64, device=dev)
        args = (heads.data_ptr(), nk, n, ordv.data_ptr(), med.data_ptr())
        if self.cuda:
            m.gpu_segment_median_select(*args, st)
        else:
            m.cpu_segment_median_select(*args)
        return uniq, med

    # ---- checkpoints ------------------------------------------------------------------------
    def snapshot_state(self):
        """Live panes' elements as rows (pane, key, f64 bits) + the firing bookkeeping."""
        from .checkpoint import OperatorSnapshot

        pk, kk, vv = [], [], []
        for r, p in enumerate(self.slot_pane):
            if p is None or not self.fill[r]:
                continue
            f = self.fill[r]
            kk.append(self.kbuf[r][:f].cpu().numpy())
            vv.append(self.vbuf[r][:f].cpu().numpy())
            pk.append(np.full(f, p, dtype=np.int64))
        cat = lambda xs: np.concatenate(xs) if xs else np.zeros(0, np.int64)  # noqa: E731
        keys = cat(kk)
        kg = (K.keygroups(torch.from_numpy(keys), max_parallelism=128).numpy()
              if keys.size else np.zeros(0, np.int32))
        cols = {"key": keys, "pane": cat(pk), "val": cat(vv)}
        meta = {"kind": "list_window", "size": self.size, "slide": self.slide,
                "offset": self.offset, "lateness": self.lateness, "wm": self.wm,
                "next_fire_start": self.next_fire_start,
                "metrics": {"num_records_in": self.metrics.num_records_in,
                            "num_late_records_dropped": self.metrics.num_late_records_dropped,
                            "num_records_out": self.metrics.num_records_out,
                            "num_fires": self.metrics.num_fires}}
        return OperatorSnapshot(kg, cols, meta)

    def restore_state(self, rows: dict, meta: dict) -> None:
        if meta.get("kind") != "list_window" or (meta["size"], meta["slide"], meta["offset"]) != \
                (self.size, self.slide, self.offset):
            raise ValueError("checkpoint of a different list window")
        self._alloc_ring(self.ring)
        self.wm = meta["wm"]
        self.next_fire_start = meta["next_fire_start"]
        for k, v in meta.get("metrics", {}).items():
            setattr(self.metrics, k, v)
        panes = np.asarray(rows.get("pane", np.zeros(0, np.int64)), dtype=np.int64)
        if not panes.size:
            return
        keys = np.asarray(rows["key"], dtype=np.int64)
        vals = np.asarray(rows["val"], dtype=np.int64)
        up = np.unique(panes)
        if up.max() - up.min() + 1 > self.ring:
            self._alloc_ring(_next_pow2(int(up.max() - up.min() + 1)))
        for p in up.tolist():
            sel = panes == p
            r = self._slot_of(p)
            f = int(sel.sum())
            self.slot_pane[r] = p
            self._ensure_capacity(r, f)
            self.kbuf[r][:f].copy_(torch.from_numpy(keys[sel]))
            self.vbuf[r][:f].copy_(torch.from_numpy(vals[sel]))
            self.fill[r] = f
            self.krange[r] = (int(keys[sel].min()), int(keys[sel].max()))
            self.ranked[r] = False  # no element ranks in the checkpoint: counting-sort firing
        self._tab_dirty = True
