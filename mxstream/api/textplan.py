"""Tracing of text-parsing user functions into a columnar parse plan (DataStream planner, N4).

Every reference job starts from ``socketTextStream`` and a ``MapFunction`` that splits the line
and parses fields (``Main.java:18-26``, ``ComputeCpuAvg.java:19-26``, ``BandwidthMonitor.java:
25-31``, ``BandwidthMonitorWithEventTime.java:30-45``). Written with the Java-semantics helpers
of ``mxstream.api.java`` (``split``, ``get``, ``parse_double``, ``parse_long``,
``iso_epoch_seconds``), such a function can be *traced*: it is called once with a ``LineProxy``
and the helpers return proxies that record which field is read and how it is parsed. The
result -- separator, (field index, kind) per output tuple position -- is what the C++ parser
(``csrc/runtime.cpp parse_lines``) executes over a whole text batch, so the job never runs the
Python function per line. Anything the proxies cannot express raises ``TraceError`` and the
planner keeps the per-record host operators.
"""
from __future__ import annotations

from dataclasses import dataclass

from ..ops import expr as E
from ..ops.text import FK_DOUBLE, FK_INT, FK_LONG, FK_STR, FK_TS_INTSEC
from .tuples import Tuple

FK_ISO_SEC = 7  # (int) LocalDateTime.parse(x).toEpochSecond(offset): int32 seconds (csrc/runtime.cpp)

TraceError = E.TraceError


class _Proxy:
    def __bool__(self):
        raise TraceError("data-dependent control flow on a traced line")

    def __hash__(self):
        return id(self)


class LineProxy(_Proxy):
    """The input line."""

    def split(self, sep: str = " ") -> "FieldsProxy":
        if not isinstance(sep, str) or len(sep) != 1:
            raise TraceError("split separator must be one character")
        return FieldsProxy(sep)


class FieldsProxy(_Proxy):
    """``line.split(sep)``: indexing selects a field."""

    def __init__(self, sep: str):
        self.sep = sep

    def __getitem__(self, i):
        if not isinstance(i, int) or i < 0:
            raise TraceError("field index must be a non-negative int")
        return FieldProxy(self.sep, i)

    def __len__(self):
        raise TraceError("len() of split fields is data dependent")


class FieldProxy(_Proxy):
    """One unparsed field (a String: becomes a dictionary id column)."""

    def __init__(self, sep: str, idx: int):
        self.sep, self.idx = sep, idx


class ParsedProxy(_Proxy):
    """A parsed numeric field (optionally scaled by an integer, e.g. seconds * 1000)."""

    def __init__(self, sep: str, idx: int, kind: int, offset_s: int = 0, scale: int = 1):
        self.sep, self.idx, self.kind, self.offset_s, self.scale = sep, idx, kind, offset_s, scale

    def __mul__(self, k):
        if not isinstance(k, int) or isinstance(k, bool):
            raise TraceError("only integer scaling of a parsed field is traced")
        return ParsedProxy(self.sep, self.idx, self.kind, self.offset_s, self.scale * k)

    __rmul__ = __mul__


def is_proxy(x) -> bool:
    return isinstance(x, _Proxy)


@dataclass(frozen=True)
class TextSpec:
    """Columnar parse plan of a traced map: output tuple position j reads field fields[j][0]
    with kind fields[j][1] (FK_*)."""
    sep: str
    fields: tuple[tuple[int, int], ...]
    offset_s: int = 0  # zone offset of ISO date-time fields

    @property
    def arity(self) -> int:
        return len(self.fields)


@dataclass(frozen=True)
class TsSpec:
    """Traced timestamp extractor: field, kind (FK_TS_INTSEC: int seconds * 1000)."""
    sep: str
    idx: int
    kind: int
    offset_s: int


def _one_sep(seps: set[str]) -> str:
    if len(seps) != 1:
        raise TraceError("fields split with different separators")
    return seps.pop()


def trace_text_map(fn) -> TextSpec:
    """Trace a MapFunction (or callable) over a text line into a TextSpec."""
    from .functions import MapFunction

    call = fn.map if isinstance(fn, MapFunction) else fn
    try:
        out = call(LineProxy())
    except TraceError:
        raise
    except Exception as e:
        raise TraceError(f"map not traceable: {type(e).__name__}: {e}") from e
    if not isinstance(out, Tuple) or not 1 <= len(out) <= 8:
        raise TraceError("map must return a Tuple of 1..8 traced fields")
    fields, seps, offs = [], set(), set()
    for f in out:
        if isinstance(f, FieldProxy):
            fields.append((f.idx, FK_STR))
            seps.add(f.sep)
        elif isinstance(f, ParsedProxy):
            if f.scale != 1:
                raise TraceError("scaled fields are only traced in timestamp extractors")
            fields.append((f.idx, f.kind))
            seps.add(f.sep)
            if f.kind == FK_ISO_SEC:
                offs.add(f.offset_s)
        else:
            raise TraceError(f"output field of type {type(f).__name__} is not a traced field")
    if len(offs) > 1:
        raise TraceError("date-time fields with different zone offsets")
    return TextSpec(_one_sep(seps), tuple(fields), offs.pop() if offs else 0)


def trace_extractor(assigner) -> TsSpec:
    """Trace a BoundedOutOfOrdernessTimestampExtractor's user timestamp function."""
    from .watermarks import BoundedOutOfOrdernessTimestampExtractor

    if type(assigner).extract_timestamp is not BoundedOutOfOrdernessTimestampExtractor.extract_timestamp:
        raise TraceError("only the bounded out-of-orderness extractor is traced")
    fn = assigner._extractor if assigner._extractor is not None else assigner.extractTimestamp
    try:
        ts = fn(LineProxy())
    except TraceError:
        raise
    except Exception as e:
        raise TraceError(f"extractor not traceable: {type(e).__name__}: {e}") from e
    if not isinstance(ts, ParsedProxy):
        raise TraceError("timestamp is not a parsed field")
    if ts.kind == FK_ISO_SEC and ts.scale == 1000:
        return TsSpec(ts.sep, ts.idx, FK_TS_INTSEC, ts.offset_s)
    if ts.kind == FK_LONG and ts.scale == 1:
        return TsSpec(ts.sep, ts.idx, FK_LONG, 0)
    raise TraceError("timestamp must be iso_epoch_seconds(...) * 1000 or an epoch-ms long field")


def trace_tuple_filter(fn, kinds: tuple[int, ...]) -> E.Program:
    """Trace a FilterFunction over the map's output tuple (numeric fields only) to the
    expression VM."""
    from .functions import FilterFunction

    call = fn.filter if isinstance(fn, FilterFunction) else fn
    row = [E.FieldRef(f"f{i}") if k == FK_STR else E.var(i) for i, k in enumerate(kinds)]
    res = E.trace_row_fn(call, row)
    if not isinstance(res, E.Expr):
        raise TraceError("filter result is not a traced expression")
    return E.compile_expr(res)


_ = (FK_DOUBLE, FK_INT)
