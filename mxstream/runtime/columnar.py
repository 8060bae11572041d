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
    """A micro-batch of raw lines ('\\n'-separated, trailing '\\r' allowed). `data` is bytes,
    or a 1-D uint8 tensor in a pinned slot of the source's ring (`token` returns the slot once
    the consumer's H2D copy has completed)."""
    data: object
    n: int
    sub0: int = 0        # subtask of the first line (round-robin from the source edge)
    parallelism: int = 1
    token: object = None
    ready: object = None  # device data: event after which the H2D copy is complete

    def host_bytes(self) -> bytes:
        if isinstance(self.data, (bytes, bytearray)):
            return bytes(self.data)
        if self.ready is not None:
            self.ready.synchronize()
        b = self.data.cpu().numpy().tobytes()
        if self.token is not None:
            self.token.consumed()
        return b


@dataclass
class ColumnBatch:
    """n rows of TupleN values as columns; string fields hold ids of `strings`."""
    n: int
    cols: list
    kinds: tuple
    strings: object                      # StringDict of FK_STR columns
    ts: np.ndarray | None = None         # event timestamps (None: no timestamp)
    sub: np.ndarray | None = None        # subtask per row
    scalar: bool = False                 # one column of bare values (not Tuple1 rows)
    _cache: dict = field(default_factory=dict)

    def field_value(self, j: int, i: int):
        v = self.cols[j][i]
        k = self.kinds[j]
        if k == FK_STR:
            return self.strings.get(int(v))
        if k == FK_DOUBLE:
            return float(v)
        return int(v)

    def value(self, i: int):
        if self.scalar:
            return self.field_value(0, i)
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
        if self.scalar:
            return [Rec(v, t, s) for v, t, s in zip(cols[0], ts, sub)]
        return [Rec(Tuple(row), t, s) for row, t, s in zip(zip(*cols), ts, sub)]

    def take(self, mask: np.ndarray) -> "ColumnBatch":
        idx = np.nonzero(mask)[0]
        return ColumnBatch(int(idx.size), [c[idx] for c in self.cols], self.kinds, self.strings,
                           None if self.ts is None else self.ts[idx],
                           None if self.sub is None else self.sub[idx], self.scalar)


class DeviceColumnBatch(ColumnBatch):
    """A ColumnBatch whose columns live on the device (the device text ingest,
    ops/ingest.py): string columns hold int32 ids of a DeviceDict, ``ts`` is a device int64
    column. Native operators read the columns in place; anything that needs host values
    (host operators, print sinks, late side outputs) materialises ``host()`` once."""

    def __init__(self, n: int, cols: list, kinds: tuple, strings, ts, *, sub0: int = 0,
                 parallelism: int = 1, line_idx=None, max_ts: int | None = None,
                 sub_dev=None, scalar: bool = False):
        """sub_dev: the subtask of every row as a device int32 column (a keyed operator's
        output: the key's subtask); otherwise rows are round-robin from sub0 (source edge)."""
        self.n, self.cols, self.kinds, self.strings, self.ts = n, cols, kinds, strings, ts
        self.sub0, self.parallelism, self.line_idx, self.max_ts = sub0, parallelism, line_idx, max_ts
        self.sub_dev, self.scalar = sub_dev, scalar
        self._cache = {}
        self._host = None

    @property
    def sub(self):
        return self.host().sub

    def host(self) -> ColumnBatch:
        parts = getattr(self, "_parts", None)
        if self._host is None and parts:
            self._host = _concat_host([b.host() for b in parts])
        if self._host is None:
            import torch

            # one D2H for all columns (a keyed operator's emit: several narrow columns)
            dev = [c[:self.n] for c in self.cols]
            if self.sub_dev is not None:
                dev.append(self.sub_dev[:self.n].to(torch.int64))
            elif self.line_idx is not None:
                dev.append(self.line_idx[:self.n].to(torch.int64))
            if self.ts is not None:
                dev.append(self.ts[:self.n])
            host = _to_host(dev)
            cols = []
            for a, k in zip(host, self.kinds):
                cols.append(a.astype(np.int64) if k == FK_STR else a)
            rest = host[len(self.cols):]
            if self.sub_dev is not None:
                sub = rest.pop(0).astype(np.int32)
            else:
                line = rest.pop(0) if self.line_idx is not None else np.arange(self.n, dtype=np.int64)
                sub = ((self.sub0 + line) % max(1, self.parallelism)).astype(np.int32)
            ts = rest.pop(0) if self.ts is not None else None
            self._host = ColumnBatch(self.n, cols, self.kinds, self.strings, ts, sub, self.scalar)
        return self._host

    def field_value(self, j: int, i: int):
        return self.host().field_value(j, i)

    def value(self, i: int) -> Tuple:
        return self.host().value(i)

    def to_recs(self) -> list[Rec]:
        return self.host().to_recs()

    def take(self, mask: np.ndarray) -> ColumnBatch:
        return self.host().take(mask)


def _to_host(cols: list) -> list:
    """Device columns -> numpy arrays with one D2H copy: the columns are packed as bytes into
    one device buffer (a cat of byte views), copied once, and cut back into typed arrays."""
    import torch

    if not cols:
        return []
    if cols[0].device.type != "cuda" or len(cols) == 1:
        return [c.cpu().numpy() for c in cols]
    parts, meta = [], []
    for c in cols:
        c = c.contiguous()
        b = c.view(torch.uint8) if c.numel() else torch.empty(0, dtype=torch.uint8, device=c.device)
        pad = (-b.numel()) % 8
        parts.append(b)
        if pad:
            parts.append(torch.zeros(pad, dtype=torch.uint8, device=c.device))
        meta.append((c.dtype, c.numel(), b.numel() + pad))
    buf = torch.cat(parts).cpu().numpy()
    out, off = [], 0
    for dt, n, nb in meta:
        npdt = torch.empty(0, dtype=dt).numpy().dtype
        out.append(buf[off:off + n * npdt.itemsize].view(npdt).copy() if n else np.zeros(0, npdt))
        off += nb
    return out


def concat_device(batches: list) -> DeviceColumnBatch:
    """Concatenate device batches of one layout and one dictionary."""
    if len(batches) == 1:
        return batches[0]
    import torch

    b0 = batches[0]
    if any(b.kinds != b0.kinds or b.strings is not b0.strings for b in batches):
        raise TypeError("incompatible column batches")
    cols = [torch.cat([b.cols[j][:b.n] for b in batches]) for j in range(len(b0.cols))]
    ts = None if b0.ts is None else torch.cat([b.ts[:b.n] for b in batches])
    out = DeviceColumnBatch(sum(b.n for b in batches), cols, b0.kinds, b0.strings, ts)
    out._parts = list(batches)  # host() concatenates the parts' host views (sub / late rows)
    return out


def _concat_host(batches: list) -> ColumnBatch:
    b0 = batches[0]
    cat = lambda xs: None if xs[0] is None else np.concatenate(xs)  # noqa: E731
    return ColumnBatch(sum(b.n for b in batches),
                       [np.concatenate([b.cols[j] for b in batches]) for j in range(len(b0.cols))],
                       b0.kinds, b0.strings, cat([b.ts for b in batches]),
                       cat([b.sub for b in batches]), b0.scalar)


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
                 threads: int | None = None, device: str | None = None, shared=None,
                 defer: bool = False):
        self.spec = spec
        self.ts_spec = ts_spec
        self.bound = int(bound)
        self.filter_prog = filter_prog
        self.threads = threads or min(16, os.cpu_count() or 1)
        # device: parse on this device (ops/ingest.py: device parse kernels + device string
        # dictionary, C++ twins on "cpu"); None: the host C++ parser (parse_lines).
        self.device = device
        self.shared = shared if shared is not None else {}
        self.agree = None
        # defer (device ingest, one rank): batch i's parse is enqueued and its result is read
        # one pass later, after batch i + 1's parse was enqueued -- the host's work downstream of
        # batch i overlaps the GPU's parse of batch i + 1. The planner enables it only where a
        # pass's delay changes nothing (no processing-time windows, no checkpoints).
        self.defer = bool(defer)
        self._pending = None
        self.cur_max = LONG_MIN + self.bound  # BoundedOutOfOrdernessTimestampExtractor state
        self.cur_wm = LONG_MIN

    def open(self, ctx):
        super().open(ctx)
        from ..ops.native import load

        self.m = load()
        fields = list(self.spec.fields)
        if self.ts_spec is not None:
            if self.ts_spec.sep != self.spec.sep:
                raise ValueError("extractor and map split the line differently")
            fields.append((self.ts_spec.idx, self.ts_spec.kind))
        self.pspec = fields
        self.offset_s = self.spec.offset_s if self.ts_spec is None else (
            self.ts_spec.offset_s or self.spec.offset_s)
        self.ingest = None
        if self.device is not None:
            from ..ops.ingest import DeviceDict, TextIngest

            self.strings = DeviceDict(self.device)
            self.shared["dict"] = self.strings
            self.ingest = TextIngest(fields, sep=self.spec.sep, offset_s=self.offset_s,
                                     ts_field=len(self.spec.fields) if self.ts_spec is not None else -1,
                                     device=self.device, dictionary=self.strings,
                                     filter_prog=self.filter_prog)
            ctrl = getattr(ctx, "ctrl", None)
            if ctrl is not None and ctrl.world > 1:
                # Several ranks: one id space for every rank (keyBy across GPUs). Each pass parses
                # this rank's batch and agrees on the new strings with every rank (collective).
                self.collective = True

                def agree(local, ctrl=ctrl):
                    # Steady state (no rank met a new string): one packed int64 all-reduce and
                    # no pickling; the strings themselves move only on passes that have some.
                    from ..parallel.comm import control_reduce

                    _, (nmax,) = control_reduce(ctrl, maxs=[len(local)])
                    if nmax == 0:
                        return []
                    seen, out = set(), []
                    for lst in ctrl.all_gather_object(local):
                        for b in lst:
                            if b not in seen:
                                seen.add(b)
                                out.append(b)
                    return out

                self.agree = agree
        else:
            self.strings = self.m.StringDict()

    def _parse_device(self, tb: TextBatch, res=None) -> DeviceColumnBatch:
        if res is None:
            res = self.ingest.parse(tb.data, tb.n, on_upload=None if (tb.token is None or tb.ready)
                                    else tb.token.uploaded, agree=self.agree, ready=tb.ready)
        nf = len(self.spec.fields)
        return DeviceColumnBatch(res.n, res.cols[:nf], tuple(k for _, k in self.spec.fields),
                                 self.strings, res.ts, sub0=tb.sub0,
                                 parallelism=max(1, self.ctx.parallelism), line_idx=res.line_idx,
                                 max_ts=res.max_ts)

    def _advance(self, max_ts) -> list:
        if self.ts_spec is None or max_ts is None:
            return []
        if max_ts > self.cur_max:
            self.cur_max = max_ts
        wm = self.cur_max - self.bound
        if wm > self.cur_wm:
            self.cur_wm = wm
            return [WM(wm)]
        return []

    def _parse(self, tb: TextBatch) -> ColumnBatch | None:
        cols, done, err_idx, err = self.m.parse_lines(tb.host_bytes(), self.pspec, self.spec.sep,
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

    @staticmethod
    def _one_batch(batches: list) -> TextBatch:
        """A pass's text batches as one (one dictionary agreement per pass on every rank)."""
        if len(batches) == 1:
            return batches[0]
        parts = []
        for b in batches:
            d = b.host_bytes()
            parts.append(d if not d or d.endswith(b"\n") else d + b"\n")
        return TextBatch(b"".join(parts), sum(b.n for b in batches), batches[0].sub0,
                         batches[0].parallelism)

    def _complete(self) -> list:
        """The deferred batch's columns and watermark (TextIngest.finish)."""
        p, self._pending = self._pending, None
        if p is None:
            return []
        pend, tb = p
        res = pend if not hasattr(pend, "hb") else self.ingest.finish(pend)
        dcb = self._parse_device(tb, res)
        wm = self._advance(dcb.max_ts)
        return ([dcb] if dcb.n else []) + wm

    def finish(self):
        return self._complete()

    def process(self, items):
        if self.defer and self.ingest is not None and self.agree is None:
            out = []
            for it in items:
                if isinstance(it, WM):
                    if it.ts == LONG_MAX:
                        out.extend(self._complete())  # every batch before end of input
                    if self.ts_spec is None or it.ts == LONG_MAX:
                        out.append(it)
                    continue
                if not isinstance(it, TextBatch):
                    raise TypeError(f"TextParseOp got {type(it).__name__}")
                pend = self.ingest.begin(it.data, it.n,
                                         on_upload=None if (it.token is None or it.ready)
                                         else it.token.uploaded, ready=it.ready)
                out.extend(self._complete())
                self._pending = (pend, it)
            return out
        if self.agree is not None:
            # Multi-rank device ingest: exactly one parse (and dictionary agreement) per pass.
            tbs = [it for it in items if isinstance(it, TextBatch)]
            tb = self._one_batch(tbs) if tbs else TextBatch(b"", 0)
            rest = [it for it in items if not isinstance(it, TextBatch)]
            items = rest[:0] + [tb] + rest
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
            if self.ingest is not None:
                # Device ingest: the traced filter already ran on the device; the watermark
                # comes from the batch maximum over every parsed line (before the filter).
                dcb = self._parse_device(it)
                wm = self._advance(dcb.max_ts)
                if dcb.n:
                    out.append(dcb)
                out.extend(wm)
                continue
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
        if self._pending is not None:
            raise RuntimeError("snapshot with a deferred ingest batch in flight")
        return {"cur_max": self.cur_max, "cur_wm": self.cur_wm, "strings": list(self.strings.strings())}

    def restore(self, snap: dict) -> None:
        self.cur_max, self.cur_wm = snap["cur_max"], snap["cur_wm"]
        strings = snap.get("strings", [])
        if self.ingest is not None:
            self.strings.intern_many(list(strings))
            return
        for s in strings:
            self.strings.intern(s)
