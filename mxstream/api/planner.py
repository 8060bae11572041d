"""Planner: rewrites recognised keyed-window shapes onto native operators.

A window transformation runs natively (runtime/native_ops.py -> C++ twin or gfx950 kernels)
when all of the following are provable at plan time; otherwise the exact host WindowOperator
runs:
  * assigner: tumbling/sliding, event or processing time, default trigger, no evictor;
  * key: keyBy(<int field>);
  * function: ``sum/min/max(pos)``, a builtin aggregate (api/aggregations.py), or a reduce
    lambda whose trace is "field pos = a.pos + b.pos, every other field = a's" (Flink's
    ``reduce((a, b) -> new TupleN(a.f0, .., a.fk + b.fk, ..))``, BandwidthMonitor.java:37);
  * keep-first fields other than the key are dead: the only consumer is a map whose traced
    output reads just the key and the aggregate (BandwidthMonitorWithEventTime.java:48-53),
    or the tuple has no such fields.
"""
from __future__ import annotations

from ..ops import expr as E
from ..runtime.executor import Transformation
from . import windowing as W


class _Probe:
    """Records which tuple fields a traced function touches."""

    def __init__(self, arity: int):
        self.used: set[int] = set()
        self.arity = arity

    def row(self):
        probe = self

        class Row(tuple):
            def __getitem__(self, i):
                probe.used.add(int(i))
                return E.var(int(i))

            def __getattr__(self, name):
                if name.startswith("f") and name[1:].isdigit():
                    return self[int(name[1:])]
                raise AttributeError(name)

        return Row([None] * self.arity)


def trace_fieldwise_reduce(fn, arity: int) -> int | None:
    """Return the summed field index if `fn(a, b)` is a field-wise sum of one field keeping
    a's other fields, else None."""
    from .functions import ReduceFunction

    call = fn.reduce if isinstance(fn, ReduceFunction) else fn

    class Row(tuple):
        def __getattr__(self, name):
            if name.startswith("f") and name[1:].isdigit():
                return self[int(name[1:])]
            raise AttributeError(name)

    a = Row([E.var(100 + i) for i in range(arity)])
    b = Row([E.var(200 + i) for i in range(arity)])
    try:
        out = call(a, b)
    except Exception:
        return None
    if not isinstance(out, tuple) or len(out) != arity:
        return None
    summed = None
    for i, f in enumerate(out):
        if not isinstance(f, E.Expr):
            return None
        if f.op == "var" and f.value == 100 + i:
            continue
        if f.op == "+" and {a_.value for a_ in f.args if a_.op == "var"} == {100 + i, 200 + i} \
                and all(a_.op == "var" for a_ in f.args):
            if summed is not None:
                return None
            summed = i
            continue
        return None
    return summed


def _consumers(sinks):
    from ..runtime.executor import Executor

    nodes = Executor._topo(sinks)
    ch = {n.id: [] for n in nodes}
    for n in nodes:
        for p in n.parents:
            ch[p.id].append(n)
    return nodes, ch


def _dead_fields_ok(t: Transformation, children, key_pos: int, val_pos: int, arity: int) -> bool:
    keep = set(range(arity)) - {key_pos, val_pos}
    if not keep:
        return True
    kids = children.get(t.id, [])
    if len(kids) != 1:
        return False
    c = kids[0]
    meta = getattr(c, "meta", None) or {}
    if meta.get("kind") != "map":
        return False
    probe = _Probe(arity)
    try:
        from .functions import MapFunction

        fn = meta["fn"]
        (fn.map if isinstance(fn, MapFunction) else fn)(probe.row())
    except Exception:
        return False
    return not (probe.used & keep)


def plan(env, sinks):
    if env.config.native == "off":
        return sinks
    nodes, children = _consumers(sinks)
    for t in nodes:
        meta = getattr(t, "meta", None) or {}
        if meta.get("kind") == "rolling" and meta["agg"] in ("sum", "min", "max") \
                and meta["key_pos"] is not None:
            _install_native_rolling(env, t, meta)
            continue
        if meta.get("kind") != "window":
            continue
        ws = meta["stream"]
        spec = meta["spec"]
        a = ws.assigner
        session = type(a) is W.EventTimeSessionWindows
        if session and ws._late_tag is not None:
            continue  # late side output of merging windows: host operator
        if not session and not isinstance(a, (W.TumblingEventTimeWindows,
                                              W.SlidingEventTimeWindows)):
            continue
        if ws._trigger is not None or ws._evictor is not None or ws.keyed is None:
            continue
        key_pos = ws.keyed.key_pos
        if key_pos is None:
            continue
        kind = val_pos = None
        ok_arities: set[int] = set()
        if meta.get("native_hint") and meta["native_hint"][0] in ("sum", "min", "max"):
            kind, val_pos = meta["native_hint"]
            result = "tuple"
            ok_arities = {ar for ar in range(2, 9) if ar > max(key_pos, val_pos)
                          and _dead_fields_ok(t, children, key_pos, val_pos, ar)}
        elif spec.kind == "aggregate" and spec.window_fn is None and hasattr(spec.fn, "native"):
            kind, val_pos = spec.fn.native
            result = "value"
            ok_arities = set(range(max(key_pos, val_pos) + 1, 64))
        elif spec.kind == "process" and getattr(spec.fn, "native", (None,))[0] == "median" \
                and not session:
            kind, val_pos = "median", spec.fn.native[1]
            result = "value"
            ok_arities = set(range(max(key_pos, val_pos) + 1, 64))
        elif spec.kind == "reduce" and spec.window_fn is None:
            result = "tuple"
            for ar in range(2, 9):
                p = trace_fieldwise_reduce(spec.fn, ar)
                if p is None or p == key_pos or ar <= key_pos:
                    continue
                if val_pos is not None and p != val_pos:
                    continue
                if _dead_fields_ok(t, children, key_pos, p, ar):
                    kind, val_pos = "sum", p
                    ok_arities.add(ar)
        if kind is None or not ok_arities:
            continue
        _install_native(env, t, ws, spec, key_pos, val_pos, kind, result, ok_arities,
                        session=session)
    return sinks


def _install_native(env, t, ws, spec, key_pos, val_pos, kind, result, ok_arities,
                    session: bool = False):
    from ..runtime import operators as O
    from ..runtime.native_ops import NativeSessionOp, NativeWindowOp
    from .tuples import Tuple

    fallback = t.factory
    assigner, late, tag = ws.assigner, ws._lateness, ws._late_tag
    key_fn = ws.keyed.key_fn

    if result == "value":
        def builder(template, res, key):
            return res
    else:
        def builder(template, res, key, vp=val_pos):
            row = list(template)
            row[vp] = res
            return Tuple(row)

    device = env.config.device

    from ..runtime.native_ops import NativeMedianOp

    from ..runtime.native_ops import NativeVectorWindowOp

    if session and kind in ("vsum", "vavg"):
        return  # merging windows over vectors: exact host operator
    cls = NativeSessionOp if session else (
        NativeMedianOp if kind == "median" else
        NativeVectorWindowOp if kind in ("vsum", "vavg") else NativeWindowOp)

    def factory():
        return cls(key_fn=key_fn, key_pos=key_pos, val_pos=val_pos, kind=kind,
                   assigner=assigner, lateness=late, late_tag=tag, device=device,
                   fallback_factory=fallback, result_builder=builder, ok_arities=ok_arities)

    t.factory = factory
    t.meta = dict(t.meta, native=True)
    _ = O


def _install_native_rolling(env, t, meta):
    """keyBy(<int field>).sum/min/max(p) -> NativeRollingOp (ComputeCpuMax.java:26)."""
    from ..runtime.native_ops import NativeRollingOp

    fallback = t.factory
    device = env.config.device
    key_fn, key_pos, pos, kind = meta["key_fn"], meta["key_pos"], meta["pos"], meta["agg"]

    def factory():
        return NativeRollingOp(key_fn=key_fn, key_pos=key_pos, val_pos=pos, kind=kind,
                               device=device, fallback_factory=fallback)

    t.factory = factory
    t.meta = dict(t.meta, native=True)
