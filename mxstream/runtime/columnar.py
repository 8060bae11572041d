"""Columnar micro-batches for the DataStream executor (text ingest without per-record Python).

A text source whose consumer chain the planner could trace (api/textplan.py) emits ``TextBatch``
items -- the raw bytes of a micro-batch of lines -- instead of one ``Rec`` per line. The fused
``TextParseOp`` (timestamp extractor + map + filter of the job, ``Main.java:17-33``,
``BandwidthMonitorWithEventTime.java:28-55``) turns each into a ``ColumnBatch``:

  * C++ ``parse_lines`` over the whole batch (multi-threaded, Java parse semantics, string
    fields interned into one StringDict -> dense dictionary ids);
  * event timestamps from the traced extractor column; the periodic bounded-out-of-orderness
    watermark after the batch (``TimestampsAndWatermarksOp`` semantics);
  * the round-robin subtask of every row (RebalancePartitioner from the parallelism-1 source);
  * the traced filter evaluated over the columns (expression VM semantics, numpy).

Native keyed operators (runtime/native_ops.py) consume ``ColumnBatch`` directly: the key column
already holds dense dictionary ids, the value and timestamp columns go to the device as they
are. Host operators receive ordinary ``Rec``s (``ColumnBatch.to_recs``), so the semantics of a
plan that mixes both are unchanged.
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field

import numpy as np

from ..api.tuples import Tuple
from ..ops import expr as E
from ..ops.text import FK_DOUBLE, FK_STR
from .operators import LONG_MAX, LONG_MIN, Operator, Rec, WM


@dataclass
class TextBatch:
    """A micro-batch of raw lines ('\\n'-separated, trailing '\\r' allowed)."""
    data: bytes
    n: int
    sub0: int = 0        # subtask of the first line (round-robin from the source edge)
    parallelism: int = 1


@dataclass
class ColumnBatch:
    """n rows of TupleN values as columns; string fields hold ids of `strings`."""
    n: int
    cols: list
    kinds: tuple
    strings: object                      # StringDict of FK_STR columns
    ts: np.ndarray | None = None         # event timestamps (None: no timestamp)
    sub: np.ndarray | None = None        # subtask per row
    _cache: dict = field(default_factory=dict)

    def field_value(self, j: int, i: int):
        v = self.cols[j][i]
        k = self.kinds[j]
        if k == FK_STR:
            return self.strings.get(int(v))
        if k == FK_DOUBLE:
            return float(v)
        return int(v)

    def value(self, i: int) -> Tuple:
        return Tuple([self.field_value(j, i) for j in range(len(self.cols))])

    def to_recs(self) -> list[Rec]:
        """Materialise the rows (host operators downstream of the columnar section)."""
        cols = []
        for j, k in enumerate(self.kinds):
            c = self.cols[j]
            if k == FK_STR:
                names = self.strings.strings()
                cols.append([names[x] for x in c.tolist()])
            elif k == FK_DOUBLE:
                cols.append(c.tolist())
            else:
                cols.append(c.tolist())
        ts = self.ts.tolist() if self.ts is not None else [LONG_MIN] * self.n
        sub = self.sub.tolist() if self.sub is not None else [0] * self.n
        return [Rec(Tuple(row), t, s) for row, t, s in zip(zip(*cols), ts, sub)]

    def take(self, mask: np.ndarray) -> "ColumnBatch":
        idx = np.nonzero(mask)[0]
        return ColumnBatch(int(idx.size), [c[idx] for c in self.cols], self.kinds, self.strings,
                           None if self.ts is None else self.ts[idx],
                           None if self.sub is None else self.sub[idx])


def expand_columns(items: list) -> list:
    """ColumnBatch items -> Recs, for operators without columnar input."""
    if not any(isinstance(it, ColumnBatch) for it in items):
        return items
    out = []
    for it in items:
        out.extend(it.to_recs() if isinstance(it, ColumnBatch) else [it])
    return out


def rows_in(items: list) -> int:
    return sum(it.n if isinstance(it, ColumnBatch) else 1 for it in items
               if isinstance(it, (Rec, ColumnBatch)))


class PassThroughOp(Operator):
    """A node whose work was fused into an upstream TextParseOp (e.g. the filter)."""

    accepts_columns = True
    name = "Fused"

    def process(self, items):
        return items


class TextParseOp(Operator):
    """timestamps/watermarks + map + filter of a text job, over whole text batches."""

    accepts_columns = True
    name = "Map"

    def __init__(self, spec, *, ts_spec=None, bound: int = 0, filter_prog=None,
                 threads: int | None = None):
        self.spec = spec
        self.ts_spec = ts_spec
        self.bound = int(bound)
        self.filter_prog = filter_prog
        self.threads = threads or min(16, os.cpu_count() or 1)
        self.cur_max = LONG_MIN + self.bound  # BoundedOutOfOrdernessTimestampExtractor state
        self.cur_wm = LONG_MIN

    def open(self, ctx):
        super().open(ctx)
        from ..ops.native import load

        self.m = load()
        self.strings = self.m.StringDict()
        fields = list(self.spec.fields)
        if self.ts_spec is not None:
            if self.ts_spec.sep != self.spec.sep:
                raise ValueError("extractor and map split the line differently")
            fields.append((self.ts_spec.idx, self.ts_spec.kind))
        self.pspec = fields
        self.offset_s = self.spec.offset_s if self.ts_spec is None else (
            self.ts_spec.offset_s or self.spec.offset_s)

    def _parse(self, tb: TextBatch) -> ColumnBatch | None:
        cols, done, err_idx, err = self.m.parse_lines(tb.data, self.pspec, self.spec.sep,
                                                      self.strings, self.offset_s, self.threads)
        if err_idx >= 0:
            from ..api import java as J

            kind = err.split(":", 1)[0]
            msg = err.split(": ", 1)[1] if ": " in err else err
            exc = {"NumberFormatException": J.NumberFormatException,
                   "ArrayIndexOutOfBoundsException": J.ArrayIndexOutOfBoundsException}.get(kind, ValueError)
            raise exc(msg)
        n = int(done)
        nf = len(self.spec.fields)
        ts = cols[nf] if self.ts_spec is not None else None
        sub = ((tb.sub0 + np.arange(n, dtype=np.int64)) % max(1, self.ctx.parallelism)).astype(np.int32)
        return ColumnBatch(n, list(cols[:nf]), tuple(k for _, k in self.spec.fields), self.strings,
                           ts, sub)

    def _watermark(self, cb: ColumnBatch) -> list:
        if self.ts_spec is None or cb.n == 0:
            return []
        m = int(cb.ts.max())
        if m > self.cur_max:
            self.cur_max = m
        wm = self.cur_max - self.bound
        if wm > self.cur_wm:
            self.cur_wm = wm
            return [WM(wm)]
        return []

    def process(self, items):
        out = []
        for it in items:
            if isinstance(it, WM):
                # Upstream watermarks are swallowed except the end-of-input MAX (Flink 1.8), as in
                # TimestampsAndWatermarksOp; without an extractor they pass through.
                if self.ts_spec is None or it.ts == LONG_MAX:
                    out.append(it)
                continue
            if not isinstance(it, TextBatch):
                raise TypeError(f"TextParseOp got {type(it).__name__}")
            cb = self._parse(it)
            wm = self._watermark(cb)
            if self.filter_prog is not None and cb.n:
                keep = E.eval_numpy(self.filter_prog, [c.astype(np.float64) if self.spec.fields[j][1] != FK_STR
                                                       else np.zeros(cb.n) for j, c in enumerate(cb.cols)])
                cb = cb.take(np.asarray(keep) != 0.0)
            if cb.n:
                out.append(cb)
            out.extend(wm)
        return out

    def snapshot(self) -> dict:
        return {"cur_max": self.cur_max, "cur_wm": self.cur_wm, "strings": list(self.strings.strings())}

    def restore(self, snap: dict) -> None:
        self.cur_max, self.cur_wm = snap["cur_max"], snap["cur_wm"]
        for s in snap.get("strings", []):
            self.strings.intern(s)
