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

The tier is columnar rows (key, pane, acc, cnt, dirty) in numpy arrays, merged per (key, pane)
lazily; it is purged with the device's panes.
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
    def __init__(self, agg: int):
        self.agg = agg
        self._cols = self._empty()
        self._merged = 0          # rows [0, _merged) are unique per (key, pane)
        self.rows_in = 0

    @staticmethod
    def _empty():
        return {"key": np.zeros(0, np.uint64), "pane": np.zeros(0, np.int64),
                "acc": np.zeros(0, np.int64), "cnt": np.zeros(0, np.int64),
                "dirty": np.zeros(0, np.uint8)}

    @property
    def nrows(self) -> int:
        return int(self._cols["key"].size)

    @property
    def nbytes(self) -> int:
        return sum(v.nbytes for v in self._cols.values())

    def absorb(self, key, pane, acc, cnt, dirty) -> None:
        c = self._cols
        self._cols = {"key": np.concatenate([c["key"], key.astype(np.uint64)]),
                      "pane": np.concatenate([c["pane"], pane.astype(np.int64)]),
                      "acc": np.concatenate([c["acc"], acc.astype(np.int64)]),
                      "cnt": np.concatenate([c["cnt"], cnt.astype(np.int64)]),
                      "dirty": np.concatenate([c["dirty"], dirty.astype(np.uint8)])}
        self.rows_in += int(key.size)
        if self.nrows > 2 * max(self._merged, 1 << 16):
            self._merge()

    def _merge(self) -> None:
        """Fold rows of the same (key, pane) (a key evicted, re-inserted and evicted again)."""
        c = self._cols
        if not c["key"].size:
            self._merged = 0
            return
        order = np.lexsort((c["key"], c["pane"]))
        k, p = c["key"][order], c["pane"][order]
        starts = np.flatnonzero(np.r_[True, (k[1:] != k[:-1]) | (p[1:] != p[:-1])])
        self._cols = {"key": k[starts], "pane": p[starts],
                      "acc": _reduce(self.agg, c["acc"][order], starts),
                      "cnt": np.add.reduceat(c["cnt"][order], starts),
                      "dirty": np.maximum.reduceat(c["dirty"][order], starts)}
        self._merged = self.nrows

    def pane_range(self) -> tuple[int, int] | None:
        p = self._cols["pane"]
        return (int(p.min()), int(p.max())) if p.size else None

    def overlaps(self, p0: int, p1: int) -> bool:
        r = self.pane_range()
        return r is not None and r[0] <= p1 and r[1] >= p0

    def part(self, p0: int, p1: int):
        """This tier's share of the window over panes [p0, p1]: (keys, acc, cnt) per key."""
        c = self._cols
        sel = (c["pane"] >= p0) & (c["pane"] <= p1)
        return combine_rows(self.agg, c["key"][sel], c["acc"][sel], c["cnt"][sel])

    def purge(self, keep_from: int) -> None:
        c = self._cols
        if c["pane"].size and int(c["pane"].min()) < keep_from:
            sel = c["pane"] >= keep_from
            self._cols = {k: v[sel] for k, v in c.items()}
            self._merged = min(self._merged, self.nrows)

    def rows(self) -> dict:
        self._merge()
        return {k: v.copy() for k, v in self._cols.items()}

    def clear(self) -> None:
        self._cols = self._empty()
        self._merged = 0

    def copy(self) -> "HostWindowTier":
        """An independent copy (the frozen tier of an asynchronous snapshot)."""
        t = HostWindowTier(self.agg)
        t._cols = {k: v.copy() for k, v in self._cols.items()}
        t._merged, t.rows_in = self._merged, self.rows_in
        return t


def merge_fire(agg: int, dev_keys, dev_raw, dev_cnt, host_part, only_dirty: bool,
               map_prog: E.Program, filter_prog: E.Program, wstart: int, wend: int):
    """Device rows (no epilogue) + the host tier's part of the same window -> the epilogue's
    (keys, values, raw, counts). A re-firing covers only the device's dirty keys."""
    hk, hacc, hcnt = host_part
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
