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


def trace_avg_aggregate(fn, arity: int) -> int | None:
    """Recognise a user AggregateFunction computing the average of one numeric field with a
    (count, sum) accumulator (ComputeCpuAvg.java:31-58): `add` traced symbolically must be
    "count + 1, sum + value.f<p>" (in either accumulator order), and `get_result` / `merge`
    checked on concrete accumulators (get_result branches on count == 0, which no trace
    expresses). Returns p, or None."""
    from .functions import AggregateFunction

    if not isinstance(fn, AggregateFunction):
        return None
    try:
        acc0 = fn.create_accumulator()
        if not isinstance(acc0, tuple) or len(acc0) != 2 or any(x != 0 for x in acc0):
            return None

        class Row(tuple):
            def __getattr__(self, name):
                if name.startswith("f") and name[1:].isdigit():
                    return self[int(name[1:])]
                raise AttributeError(name)

        out = fn.add(Row([E.var(i) for i in range(arity)]), Row([E.var(100), E.var(101)]))
        if not isinstance(out, tuple) or len(out) != 2:
            return None
        cnt_i = sum_i = field = None
        for i, f in enumerate(out):
            if not isinstance(f, E.Expr) or f.op != "+" or len(f.args) != 2:
                return None
            a, b = f.args
            names = {x.value for x in (a, b) if x.op == "var"}
            consts = [x.value for x in (a, b) if x.op == "const"]
            if names == {100 + i} and consts == [1.0]:
                cnt_i = i
            elif len(names) == 2 and 100 + i in names and all(x.op == "var" for x in (a, b)):
                sum_i, field = i, (names - {100 + i}).pop()
            else:
                return None
        if cnt_i is None or sum_i is None or not 0 <= field < arity:
            return None
        T = type(acc0)

        def mk(c, sm):
            v = [0, 0]
            v[cnt_i], v[sum_i] = c, sm
            return T(v)
        for c, sm in ((0, 0.0), (3, 6.0), (7, 10.5), (2, -3.0), (5, 1e300)):
            want = 0.0 if c == 0 else sm / c
            if fn.get_result(mk(c, sm)) != want:
                return None
        m = fn.merge(mk(2, 1.5), mk(3, 4.0))
        if tuple(m) != tuple(mk(5, 5.5)):
            return None
        return field
    except Exception:
        return None


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


def _defer_safe(env, nodes) -> bool:
    """A pass's delay of the device ingest's output changes nothing the job can observe: no
    checkpoints (a deferred batch would sit between two passes), and every operator is a
    map / filter / timestamp assigner / rolling aggregate / event-time window / sink -- none
    reads the processing-time clock."""
    if env.checkpoint_config.is_checkpointing_enabled():
        return False
    for n in nodes:
        if n.kind in ("source", "sink", "union", "side"):
            continue
        meta = getattr(n, "meta", None) or {}
        kind = meta.get("kind")
        if kind in ("map", "filter", "timestamps", "rolling"):
            continue
        if kind == "window" and meta["stream"].assigner.is_event_time():
            continue
        return False
    return True


def _lower_text(env, sinks) -> None:
    """Columnar text ingest: source(text) -> [timestamps] -> map(parse) -> [filter] becomes one
    TextParseOp fed by raw line batches, when the map (and extractor / filter) trace
    (api/textplan.py). The filter node stays in the graph as a pass-through."""
    from ..runtime.columnar import PassThroughOp, TextParseOp
    from . import textplan as T

    nodes, children = _consumers(sinks)
    defer = _defer_safe(env, nodes) and getattr(env.config, "ingest_defer", True)
    for t in nodes:
        meta = getattr(t, "meta", None) or {}
        if meta.get("kind") != "map" or meta.get("columnar") or len(t.parents) != 1:
            continue
        parent, ts_node = t.parents[0], None
        pmeta = getattr(parent, "meta", None) or {}
        if pmeta.get("kind") == "timestamps" and len(parent.parents) == 1:
            ts_node, parent = parent, parent.parents[0]
            pmeta = getattr(parent, "meta", None) or {}
        if parent.kind != "source" or not pmeta.get("text"):
            continue
        if len(children[parent.id]) != 1 or (ts_node is not None and len(children[ts_node.id]) != 1):
            continue
        try:
            spec = T.trace_text_map(meta["fn"])
            ts_spec, bound = None, 0
            if ts_node is not None:
                a = ts_node.meta["assigner"]
                ts_spec = T.trace_extractor(a)
                bound = a.get_max_out_of_orderness_in_millis()
        except T.TraceError:
            continue
        filt, fnode = None, None
        kids = children[t.id]
        if len(kids) == 1 and (getattr(kids[0], "meta", None) or {}).get("kind") == "filter" \
                and (kids[0].parallelism or env.parallelism) == (t.parallelism or env.parallelism):
            try:
                filt = T.trace_tuple_filter(kids[0].meta["fn"], tuple(k for _, k in spec.fields))
                fnode = kids[0]
            except T.TraceError:
                filt = None
        mode = getattr(env.config, "text_ingest", "auto")
        dev = str(env.config.device)
        ingest_dev = dev if (mode == "device" or (mode == "auto" and dev.startswith("cuda"))) \
            else None
        # The device ingest's dictionary is shared with the keyed native operators downstream
        # (names of fired keys, Java hashes of key groups at G > 1).
        shared: dict = {}
        t.factory = (lambda spec=spec, ts_spec=ts_spec, bound=bound, filt=filt, d=ingest_dev,
                     sh=shared, df=defer: TextParseOp(spec, ts_spec=ts_spec, bound=bound,
                                                      filter_prog=filt, device=d, shared=sh,
                                                      defer=df))
        t.parents = [parent]
        if fnode is not None:
            fnode.factory = PassThroughOp
            fnode.meta = dict(fnode.meta, fused=True)
        src_factory = parent.factory

        def columnar_source(f=src_factory, ring=ingest_dev is not None, dev=ingest_dev):
            s = f()
            s.columnar = True
            if ring and hasattr(type(s), "ring"):
                s.ring = True  # file -> pinned ring slots (C++ reader) -> device ingest
                s.ring_device = dev
            return s

        parent.factory = columnar_source
        t.meta = dict(meta, columnar=True, text_spec=spec,
                      device_ingest=shared if ingest_dev is not None else None,
                      event_ts=ts_spec is not None)


def plan(env, sinks):
    if env.config.native == "off":
        return sinks
    _lower_text(env, sinks)
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
        if type(a) is W.GlobalWindows:
            _lower_count_window(env, t, ws, spec, meta, children)
            continue
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
        elif spec.kind == "aggregate" and spec.window_fn is None and not session:
            # A user AggregateFunction: the (count, sum) average of one field?
            for ar in range(2, 9):
                if ar <= key_pos:
                    continue
                p = trace_avg_aggregate(spec.fn, ar)
                if p is not None and p != key_pos:
                    kind, val_pos, result = "avg", p, "value"
                    ok_arities.add(ar)
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
        if not session and kind in ("sum", "min", "max") and result == "tuple":
            _fuse_window_epilogue(env, t, children, key_pos, val_pos, ok_arities)
    return sinks


def _count_window_size(ws) -> int | None:
    """n of a tumbling count window: GlobalWindows + PurgingTrigger(CountTrigger(n)), no evictor
    (KeyedStream.countWindow(n)); None for anything else (sliding count windows use an evictor)."""
    tr = ws._trigger
    if ws._evictor is not None or not isinstance(tr, W.PurgingTrigger):
        return None
    inner = tr.nested
    if type(inner) is not W.CountTrigger or not isinstance(inner.count, int) or inner.count < 1:
        return None
    return inner.count


def _lower_count_window(env, t, ws, spec, meta, children) -> None:
    """keyBy(k).countWindow(n).sum/min/max(p) | reduce(field-wise sum) | aggregate(avg) ->
    NativeCountWindowOp (segmented-scan count windows on the GPU / C++ twin)."""
    n = _count_window_size(ws)
    if n is None or ws.keyed is None or ws.keyed.key_pos is None or ws._late_tag is not None:
        return
    key_pos = ws.keyed.key_pos
    kind = val_pos = None
    ok: set[int] = set()
    result = "tuple"
    if meta.get("native_hint") and meta["native_hint"][0] in ("sum", "min", "max"):
        kind, val_pos = meta["native_hint"]
        ok = {ar for ar in range(2, 9) if ar > max(key_pos, val_pos)
              and _dead_fields_ok(t, children, key_pos, val_pos, ar)}
    elif spec.kind == "aggregate" and spec.window_fn is None and hasattr(spec.fn, "native"):
        kind, val_pos = spec.fn.native
        result = "value"
        ok = set(range(max(key_pos, val_pos) + 1, 64))
    elif spec.kind == "aggregate" and spec.window_fn is None:
        for ar in range(2, 9):
            if ar <= key_pos:
                continue
            p = trace_avg_aggregate(spec.fn, ar)
            if p is not None and p != key_pos:
                kind, val_pos, result = "avg", p, "value"
                ok.add(ar)
    elif spec.kind == "reduce" and spec.window_fn is None:
        for ar in range(2, 9):
            p = trace_fieldwise_reduce(spec.fn, ar)
            if p is None or p == key_pos or ar <= key_pos:
                continue
            if val_pos is not None and p != val_pos:
                continue
            if _dead_fields_ok(t, children, key_pos, p, ar):
                kind, val_pos = "sum", p
                ok.add(ar)
    if kind not in ("sum", "min", "max", "count", "avg") or not ok:
        return
    from ..runtime.native_ops import NativeCountWindowOp
    from .tuples import Tuple

    if result == "value":
        def builder(template, res, key):
            return res
    else:
        def builder(template, res, key, vp=val_pos):
            row = list(template)
            row[vp] = res
            return Tuple(row)

    fallback = t.factory
    device = env.config.device
    key_fn = ws.keyed.key_fn

    def factory():
        return NativeCountWindowOp(count=n, result_builder=builder, ok_arities=ok, key_fn=key_fn,
                                   key_pos=key_pos, val_pos=val_pos, kind=kind, device=device,
                                   fallback_factory=fallback)

    t.factory = factory
    t.meta = dict(t.meta, native=True)


def _expr_vars(e) -> set:
    if e.op == "var":
        return {e.value}
    return set().union(*(_expr_vars(a) for a in e.args)) if e.args else set()


def _fuse_window_epilogue(env, t, children, key_pos: int, val_pos: int, ok_arities) -> None:
    """window(reduce/sum/min/max) -> map -> [filter] (BandwidthMonitorWithEventTime.java:46-55):
    the map and filter are traced over the window's output tuple (the aggregate as
    VAR_RESULT, other fields passed through by name) and run inside the fire kernel's epilogue;
    only the rows that pass leave the device. The map / filter nodes become pass-throughs."""
    from ..runtime.columnar import PassThroughOp
    from .functions import FilterFunction, MapFunction

    par = lambda n: n.parallelism or env.parallelism  # noqa: E731
    kids = children.get(t.id, [])
    if len(kids) != 1:
        return
    m = kids[0]
    mmeta = getattr(m, "meta", None) or {}
    spec = None
    for p in t.parents:
        spec = (getattr(p, "meta", None) or {}).get("text_spec") or spec
    arity = spec.arity if spec is not None else (next(iter(ok_arities)) if len(ok_arities) == 1 else None)
    if arity is None or arity not in ok_arities or par(m) != par(t):
        return
    if mmeta.get("kind") == "filter" and not mmeta.get("fused"):
        # window -> filter (BandwidthMonitor.java:37-39): the predicate over the aggregate runs
        # in the fire kernel.
        ff = mmeta["fn"]
        try:
            row = [E.var(E.VAR_RESULT) if i == val_pos else E.FieldRef(f"f{i}") for i in range(arity)]
            r = E.trace_row_fn(ff.filter if isinstance(ff, FilterFunction) else ff, row)
        except E.TraceError:
            return
        if not isinstance(r, E.Expr) or not _expr_vars(r) <= {E.VAR_RESULT}:
            return
        inner, prog = t.factory, E.compile_expr(r)

        def ffactory(inner=inner, prog=prog):
            op = inner()
            op.filter_prog = prog
            return op

        t.factory = ffactory
        m.factory = PassThroughOp
        m.meta = dict(mmeta, fused=True)
        return
    if mmeta.get("kind") != "map" or mmeta.get("columnar"):
        return
    fn = mmeta["fn"]
    try:
        row = [E.var(E.VAR_RESULT) if i == val_pos else E.FieldRef(f"f{i}") for i in range(arity)]
        out = E.trace_row_fn(fn.map if isinstance(fn, MapFunction) else fn, row)
        from .tuples import Tuple

        comps = list(out) if isinstance(out, Tuple) else [out]
        layout, exprs = [], []
        for c in comps:
            if isinstance(c, E.FieldRef):
                layout.append(int(c.name[1:]))
            elif isinstance(c, E.Expr):
                if not _expr_vars(c) <= {E.VAR_RESULT}:
                    return
                layout.append(-1)
                exprs.append(c)
            else:
                return
        if len(exprs) > 1:
            return
        map_prog = E.compile_expr(exprs[0]) if exprs else E.EMPTY
        filt_prog, fnode = E.EMPTY, None
        mk = children.get(m.id, [])
        if len(mk) == 1 and (getattr(mk[0], "meta", None) or {}).get("kind") == "filter" \
                and par(mk[0]) == par(m):
            ff = mk[0].meta["fn"]
            row2 = [E.var(E.VAR_MAPPED) if j < 0 else E.FieldRef(f"f{j}") for j in layout]
            try:
                r2 = E.trace_row_fn(ff.filter if isinstance(ff, FilterFunction) else ff,
                                    row2 if isinstance(out, Tuple) else [E.var(E.VAR_MAPPED)])
                if not isinstance(out, Tuple):
                    r2 = ff.filter(E.var(E.VAR_MAPPED)) if isinstance(ff, FilterFunction) else ff(E.var(E.VAR_MAPPED))
                if isinstance(r2, E.Expr) and _expr_vars(r2) <= {E.VAR_MAPPED, E.VAR_RESULT}:
                    filt_prog, fnode = E.compile_expr(r2), mk[0]
            except E.TraceError:
                pass
    except E.TraceError:
        return
    inner = t.factory
    scalar = not isinstance(out, Tuple)

    def factory(inner=inner, map_prog=map_prog, filt_prog=filt_prog, layout=tuple(layout)):
        op = inner()
        op.map_prog, op.filter_prog = map_prog, filt_prog
        op.fused_layout = None if scalar else layout
        op.fused_scalar = scalar
        return op

    t.factory = factory
    m.factory = PassThroughOp
    m.meta = dict(mmeta, fused=True)
    if fnode is not None:
        fnode.factory = PassThroughOp
        fnode.meta = dict(fnode.meta, fused=True)


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
    # Input straight from the device ingest: the operator knows its column kinds up front and
    # shares the ingest's dictionary (the G > 1 device exchange needs both before any data).
    device_input = None
    for p in t.parents:
        pm = getattr(p, "meta", None) or {}
        if pm.get("device_ingest") is not None and pm.get("text_spec") is not None:
            device_input = (tuple(k for _, k in pm["text_spec"].fields), pm["device_ingest"])

    def factory():
        op = cls(key_fn=key_fn, key_pos=key_pos, val_pos=val_pos, kind=kind,
                 assigner=assigner, lateness=late, late_tag=tag, device=device,
                 fallback_factory=fallback, result_builder=builder, ok_arities=ok_arities)
        op.device_input = device_input
        op.scalar_result = result == "value"
        op.dense_budget = int(env.config.window_dense_max_keys)
        return op

    t.factory = factory
    t.meta = dict(t.meta, native=True)
    _ = O


def _install_native_rolling(env, t, meta):
    """keyBy(<int field>).sum/min/max(p) -> NativeRollingOp (ComputeCpuMax.java:26)."""
    from ..runtime.native_ops import NativeRollingOp

    fallback = t.factory
    device = env.config.device
    key_fn, key_pos, pos, kind = meta["key_fn"], meta["key_pos"], meta["pos"], meta["agg"]
    device_input, event_ts = None, True
    for p in t.parents:
        pm = getattr(p, "meta", None) or {}
        if pm.get("device_ingest") is not None and pm.get("text_spec") is not None:
            device_input = (tuple(k for _, k in pm["text_spec"].fields), pm["device_ingest"])
            event_ts = bool(pm.get("event_ts"))

    def factory():
        op = NativeRollingOp(key_fn=key_fn, key_pos=key_pos, val_pos=pos, kind=kind,
                             device=device, fallback_factory=fallback)
        op.device_input, op.event_ts = device_input, event_ts
        return op

    t.factory = factory
    t.meta = dict(t.meta, native=True)
