"""Host-DRAM tier of the keyed window state (BASELINE: keyed state with spill to host DRAM).

The device tables of a hashed-key ``KeyedWindowOperator`` hold every key that ever sent data;
with an unbounded key space they fill up. When a sub-table passes the operator's load budget,
``window_compact`` (csrc/kernels_hip.hip, one workgroup per sub-table) drops keys that have no
data in the live panes, evicts *cold* keys -- whose newest data pane is older than the cutoff --
into this tier, and rehashes the kept keys. New data for an evicted key simply re-inserts it on
the device; nothing is diverted. When a window fires and this tier holds data for its panes, the
device fires without its epilogue, this tier's part of the same window is combined key by key
(every aggregate is associative), and the map/filter epilogue is evaluated on the host with the
fire kernel's expression-VM semantics (``expr.eval_numpy``).

The tier itself is C++ (csrc/window_tier.h): evicted rows (key, pane, acc, cnt, dirty) are
appended as chunks (no re-concatenation per eviction), a purge drops whole chunks below the live
range; rows are merged per (key, pane) only for a snapshot. A firing exports the live rows of its
panes (threaded, uncombined) into a pinned slab; on a GPU they are combined with the device's rows
ON THE DEVICE (KeyedWindowOperator._fire_window_tiered: tier_merge + the fused fire epilogue), the
host-side merge_fire below is the CPU-free fallback and the test oracle.
"""
from __future__ import annotations

import numpy as np

from ..ops import expr as E
from ..ops import kernels as K

_F64 = (K.AGG_SUM_F64, K.AGG_AVG_F64, K.AGG_MIN_F64, K.AGG_MAX_F64)
_MIN = (K.AGG_MIN_I64, K.AGG_MIN_F64)
_MAX = (K.AGG_MAX_I64, K.AGG_MAX_F64)


def _reduce(agg: int, acc: np.ndarray, starts: np.ndarray) -> np.ndarray:
    """Combine runs of raw accumulators (int64 bit patterns) starting at `starts`."""
    x = acc.view(np.float64) if agg in _F64 else acc
    if agg in _MIN:
        r = np.minimum.reduceat(x, starts)
    elif agg in _MAX:
        r = np.maximum.reduceat(x, starts)
    else:
        r = np.add.reduceat(x, starts)
    return r.view(np.int64) if agg in _F64 else r.astype(np.int64)


def combine_rows(agg: int, keys: np.ndarray, acc: np.ndarray, cnt: np.ndarray):
    """Group rows by key and combine: -> (unique keys, acc, cnt)."""
    if not keys.size:
        return keys, acc, cnt
    order = np.argsort(keys, kind="stable")
    k, a, c = keys[order], acc[order], cnt[order]
    starts = np.flatnonzero(np.r_[True, k[1:] != k[:-1]])
    return k[starts], _reduce(agg, a, starts), np.add.reduceat(c.astype(np.int64), starts)


def result_values(agg: int, raw: np.ndarray, cnt: np.ndarray) -> np.ndarray:
    """agg_result_f64 (csrc/mxs_common.h): the window result as double."""
    if agg in (K.AGG_SUM_F64, K.AGG_MIN_F64, K.AGG_MAX_F64):
        return raw.view(np.float64).copy()
    if agg == K.AGG_AVG_F64:
        return raw.view(np.float64) / np.maximum(cnt, 1)
    if agg == K.AGG_AVG_I64:
        return raw.astype(np.float64) / np.maximum(cnt, 1)
    if agg == K.AGG_COUNT:
        return cnt.astype(np.float64)
    return raw.astype(np.float64)


class HostWindowTier:
    """Thin wrapper of the C++ tier (csrc/window_tier.h): append-only chunks of evicted rows,
    hash-combined per key for a firing, whole chunks dropped by a purge."""

    def __init__(self, agg: int, _core=None):
        from ..ops.native import load

        self.agg = agg
        self._t = _core if _core is not None else load().WindowTier(agg)
        # columns of the next eviction's chunk mapped on a background thread after every absorb
        # (csrc/window_tier.h prefault_async); "0": A/B
        self._t.prefault = __import__("os").environ.get("MXS_TIER_PREFAULT", "1") != "0"
        # An eviction absorbed on a background thread (absorb_presorted(background=True)): every
        # reader joins it first; a purge meanwhile is deferred to the join (purges only free
        # memory -- a firing's export never reads panes below the purge cutoff).
        self._bg = None
        self._bg_err = None
        self._purge_pending = None

    def _join(self) -> None:
        t, self._bg = self._bg, None
        if t is not None:
            t.join()
            if self._bg_err is not None:
                e, self._bg_err = self._bg_err, None
                raise e
        if self._purge_pending is not None:
            k, self._purge_pending = self._purge_pending, None
            self._t.purge(int(k))

    @property
    def nrows(self) -> int:
        self._join()
        return int(self._t.nrows)

    @property
    def nbytes(self) -> int:
        self._join()
        return int(self._t.nbytes)

    @property
    def rows_in(self) -> int:
        self._join()
        return int(self._t.rows_in)

    def absorb(self, key, pane, acc, cnt, dirty) -> None:
        self._join()
        self._t.absorb(np.ascontiguousarray(key).view(np.uint64) if key.dtype == np.int64
                       else np.ascontiguousarray(key, dtype=np.uint64),
                       np.ascontiguousarray(pane, dtype=np.int64),
                       np.ascontiguousarray(acc, dtype=np.int64),
                       np.ascontiguousarray(cnt, dtype=np.int64),
                       np.ascontiguousarray(dirty, dtype=np.uint8))

    def absorb_presorted(self, key, acc, cnt, dirty, p0: int, counts,
                         background: bool = False) -> None:
        """Rows grouped by pane on the device (window_rows_pane_sort): pane p0 + j holds the
        next counts[j] rows. background=True: the copy into the tier (threaded C++, GIL
        released) runs on a thread while the caller goes on; the arrays must stay valid until
        the next reader joins it (the pinned slab they view is held by these references)."""
        self._join()
        args = (np.ascontiguousarray(key).view(np.uint64), np.ascontiguousarray(acc).view(np.uint64),
                np.ascontiguousarray(cnt).view(np.uint32),
                np.ascontiguousarray(dirty, dtype=np.uint8), int(p0),
                np.ascontiguousarray(counts).view(np.uint32))
        if not background:
            self._t.absorb_presorted(*args)
            return
        import threading

        def work():
            try:
                self._t.absorb_presorted(*args)
            except BaseException as e:  # re-raised by _join
                self._bg_err = e

        self._bg = threading.Thread(target=work, name="mxs-tier-absorb", daemon=True)
        self._bg.start()

    def pane_range(self) -> tuple[int, int] | None:
        self._join()
        return self._t.pane_range()

    def overlaps(self, p0: int, p1: int) -> bool:
        r = self.pane_range()
        return r is not None and r[0] <= p1 and r[1] >= p0

    def export(self, p0: int, p1: int, device, pool=None):
        """Live rows of panes [p0, p1], uncombined, as (keys int64, acc int64, cnt int32, n,
        None) on `device` (the device-merged tiered firing). GPU: piece by piece through the
        ring of page-locked slabs (_export_ring), the copies asynchronous on the current stream.
        None: no rows. (`pool`: unused, kept for callers.)"""
        import torch

        self._join()
        bound = self.nrows
        if bound == 0:
            return None
        if torch.device(device).type == "cuda":
            return self._export_ring(p0, p1, device)
        k = np.empty(bound, np.int64)
        a = np.empty(bound, np.int64)
        c = np.empty(bound, np.int32)
        n = int(self._t.export_rows(int(p0), int(p1), k.ctypes.data, a.ctypes.data, c.ctypes.data,
                                    bound))
        if n > bound:
            raise RuntimeError(f"tier export: {n} live rows exceed the {bound}-row bound")
        if n == 0:
            return None
        return (torch.from_numpy(k[:n]), torch.from_numpy(a[:n]), torch.from_numpy(c[:n]), n,
                None)

    # Ring of fixed page-locked slabs for the device export: a large export goes piece by piece
    # (C++ export_window writes rows [r, r + piece) of the export's row order), each piece's H2D
    # on the current stream, a slab reused once its earlier copy has completed. The pinned
    # memory never grows with the tier (a growing single slab was re-page-locked inside the
    # stream: 44-88 ms per growth on the box).
    _RING_SLABS = 4
    _RING_ROWS = 1 << 22  # rows per piece: 80 MB per slab (8 + 8 + 4 bytes a row)

    def _export_ring(self, p0: int, p1: int, device):
        import torch

        if getattr(self, "_ring", None) is None:
            pr = self._RING_ROWS
            self._ring = [[torch.empty(pr * 20, dtype=torch.uint8, pin_memory=True), None]
                          for _ in range(self._RING_SLABS)]
        pr = self._RING_ROWS
        total = None
        dk = da = dc = None
        r, i = 0, 0
        while total is None or r < total:
            slot = self._ring[i % len(self._ring)]
            if slot[1] is not None:
                slot[1].synchronize()  # this slab's previous piece has reached the device
                slot[1] = None
            t = slot[0]
            base = t.data_ptr()
            n = int(self._t.export_window(int(p0), int(p1), base, base + 8 * pr, base + 16 * pr,
                                          r, pr))
            if total is None:
                if n == 0:
                    return None
                total = n
                dk = torch.empty(total, dtype=torch.int64, device=device)
                da = torch.empty(total, dtype=torch.int64, device=device)
                dc = torch.empty(total, dtype=torch.int32, device=device)
            elif n != total:
                raise RuntimeError("tier export: the tier changed between pieces (internal error)")
            m = min(pr, total - r)
            dk[r:r + m].copy_(t[:8 * m].view(torch.int64), non_blocking=True)
            da[r:r + m].copy_(t[8 * pr:8 * pr + 8 * m].view(torch.int64), non_blocking=True)
            dc[r:r + m].copy_(t[16 * pr:16 * pr + 4 * m].view(torch.int32), non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(device))
            slot[1] = ev
            r += m
            i += 1
        return dk, da, dc, total, None

    def part(self, p0: int, p1: int):
        """This tier's share of the window over panes [p0, p1]: (keys, acc, cnt) per key."""
        self._join()
        return self._t.part(int(p0), int(p1))

    def purge(self, keep_from: int) -> None:
        if self._bg is not None:
            self._purge_pending = (keep_from if self._purge_pending is None
                                   else max(keep_from, self._purge_pending))
            return
        self._join()
        self._t.purge(int(keep_from))

    def rows(self) -> dict:
        self._join()
        return self._t.rows()

    def clear(self) -> None:
        self._join()
        self._t.clear()

    def copy(self) -> "HostWindowTier":
        """An independent copy (the frozen tier of an asynchronous snapshot)."""
        self._join()
        return HostWindowTier(self.agg, _core=self._t.copy())


def merge_fire(agg: int, dev_keys, dev_raw, dev_cnt, host, only_dirty: bool,
               map_prog: E.Program, filter_prog: E.Program, wstart: int, wend: int,
               panes: tuple[int, int] | None = None):
    """Device rows (no epilogue) + the host tier's part of the same window -> the epilogue's
    (keys, values, raw, counts). A re-firing covers only the device's dirty keys.
    host: a HostWindowTier (combined in C++ with the device rows over `panes`) or an already
    combined (keys, acc, cnt) part."""
    if isinstance(host, HostWindowTier):
        # Merge + result + map + filter in C++ (threaded), the numpy epilogue below stays the
        # path for an already combined part.
        mc, mk = map_prog.as_args()
        fc, fk = filter_prog.as_args()
        host._join()
        keys, mapped, raw, cnt = host._t.merge_fire_epilogue(
            int(panes[0]), int(panes[1]), np.ascontiguousarray(dev_keys, dtype=np.uint64),
            np.ascontiguousarray(dev_raw, dtype=np.int64),
            np.ascontiguousarray(dev_cnt, dtype=np.int64), bool(only_dirty), mc, mk, fc, fk,
            int(wstart), int(wend))
        return keys, mapped, raw, cnt
    hk, hacc, hcnt = host
    if only_dirty and hk.size:
        sel = np.isin(hk, dev_keys)
        hk, hacc, hcnt = hk[sel], hacc[sel], hcnt[sel]
    keys, raw, cnt = combine_rows(agg, np.concatenate([dev_keys.astype(np.uint64), hk]),
                                  np.concatenate([dev_raw.astype(np.int64), hacc]),
                                  np.concatenate([dev_cnt.astype(np.int64), hcnt]))
    res = result_values(agg, raw, cnt)
    vars_ = [res, cnt.astype(np.float64), float(wstart), float(wend), keys.astype(np.float64),
             raw.astype(np.float64), res, 0.0]
    mapped = np.asarray(E.eval_numpy(map_prog, vars_), dtype=np.float64) if map_prog.code else res
    mapped = np.broadcast_to(mapped, res.shape).astype(np.float64)
    if filter_prog.code:
        vars_[E.VAR_MAPPED] = mapped
        keep = np.broadcast_to(np.asarray(E.eval_numpy(filter_prog, vars_)) != 0.0, res.shape)
        keys, mapped, raw, cnt = keys[keep], mapped[keep], raw[keep], cnt[keep]
    return keys, mapped, raw, cnt.astype(np.int32)
