"""DataStream API (Flink 1.8 method names; snake_case with camelCase aliases).

Reference surface: socketTextStream, map, filter, keyBy(int), max(int),
timeWindow(Time[,Time]), reduce, aggregate, process, assignTimestampsAndWatermarks, print,
execute. Extended with the rest of the DataStream vocabulary the tutorial describes (flatMap,
union, window(...) with assigners/triggers/evictors, allowedLateness, sideOutputLateData,
countWindow, session windows, rolling sum/min/minBy/maxBy, keyed process functions).
"""
from __future__ import annotations

import itertools
from typing import Any, Callable

from ..runtime import operators as O
from ..runtime.executor import Transformation
from . import functions as F
from . import windowing as W
from .time import TimeCharacteristic, to_ms

_ids = itertools.count(1)


class OutputTag:
    _tag_ids = itertools.count(1)

    def __init__(self, tag_id: str, type_info: Any = None):
        self.tag_id = str(tag_id)
        self.type_info = type_info

    def get_id(self) -> str:
        return self.tag_id

    def __eq__(self, o):
        return isinstance(o, OutputTag) and o.tag_id == self.tag_id

    def __hash__(self):
        return hash(self.tag_id)


def _field_key(pos):
    """keyBy(int...) -> key of the tuple field(s) (Tuple1 hashes as its field)."""
    if isinstance(pos, (list, tuple)):
        if len(pos) == 1:
            pos = pos[0]
        else:
            ps = tuple(pos)
            return lambda v: tuple(v[p] for p in ps)
    if isinstance(pos, str):  # field expression "f0" / attribute
        name = pos
        if name.startswith("f") and name[1:].isdigit():
            i = int(name[1:])
            return lambda v: v[i]
        return lambda v: getattr(v, name)
    p = int(pos)
    return lambda v: v[p]


class DataStream:
    def __init__(self, env, t: Transformation):
        self.env = env
        self.t = t

    # -- helpers --
    def _one_input(self, name: str, factory, parallelism: int | None = None) -> "SingleOutputStreamOperator":
        t = Transformation(next(_ids), name, "op", [self.t], factory, parallelism)
        return SingleOutputStreamOperator(self.env, t)

    def get_id(self) -> int:
        return self.t.id

    def get_parallelism(self) -> int:
        return self.t.parallelism or self.env.parallelism

    # -- stateless --
    def map(self, fn) -> "SingleOutputStreamOperator":
        op = self._one_input("Map", lambda: O.MapOp(fn))
        op.t.meta = {"kind": "map", "fn": fn}
        return op

    def filter(self, fn) -> "SingleOutputStreamOperator":
        op = self._one_input("Filter", lambda: O.FilterOp(fn))
        op.t.meta = {"kind": "filter", "fn": fn}
        return op

    def flat_map(self, fn) -> "SingleOutputStreamOperator":
        return self._one_input("Flat Map", lambda: O.FlatMapOp(fn))

    def process(self, fn: F.ProcessFunction) -> "SingleOutputStreamOperator":
        return self._one_input("Process", lambda: O.ProcessOp(fn))

    def union(self, *others: "DataStream") -> "DataStream":
        t = Transformation(next(_ids), "Union", "union", [self.t] + [o.t for o in others])
        return DataStream(self.env, t)

    def rebalance(self) -> "DataStream":
        return self._one_input("Rebalance", lambda: O.RebalanceOp(self.env.config.rebalance_start))

    def shuffle(self) -> "DataStream":
        return self.rebalance()

    def forward(self) -> "DataStream":
        return self

    # -- time --
    def assign_timestamps_and_watermarks(self, assigner) -> "SingleOutputStreamOperator":
        op = self._one_input("Timestamps/Watermarks", lambda: O.TimestampsAndWatermarksOp(assigner))
        op.t.meta = {"kind": "timestamps", "assigner": assigner}
        return op

    # -- keyed --
    def key_by(self, *fields) -> "KeyedStream":
        if len(fields) == 1 and callable(fields[0]) and not isinstance(fields[0], (int, str)):
            return KeyedStream(self, fields[0], None)
        key_fn = _field_key(list(fields))
        pos = fields[0] if len(fields) == 1 and isinstance(fields[0], int) else None
        return KeyedStream(self, key_fn, pos)

    # -- non-keyed windows --
    def time_window_all(self, size, slide=None) -> "AllWindowedStream":
        return AllWindowedStream(self, _time_assigner(self.env, size, slide))

    def window_all(self, assigner: W.WindowAssigner) -> "AllWindowedStream":
        return AllWindowedStream(self, assigner)

    def count_window_all(self, size: int) -> "AllWindowedStream":
        return AllWindowedStream(self, W.GlobalWindows.create()).trigger(
            W.PurgingTrigger.of(W.CountTrigger.of(size)))

    # -- sinks --
    def add_sink(self, fn) -> "DataStreamSink":
        t = Transformation(next(_ids), "Sink", "sink", [self.t], lambda: O.SinkOp(fn))
        self.env._sinks.append(t)
        return DataStreamSink(self.env, t)

    def print(self, sink_identifier: str | None = None) -> "DataStreamSink":
        env = self.env
        t = Transformation(next(_ids), "Print to Std. Out", "sink", [self.t],
                           lambda: O.PrintSinkOp(env._writer, sink_identifier))
        env._sinks.append(t)
        return DataStreamSink(env, t)

    def print_to_err(self, sink_identifier: str | None = None) -> "DataStreamSink":
        import sys

        t = Transformation(next(_ids), "Print to Std. Err", "sink", [self.t],
                           lambda: O.PrintSinkOp(lambda s: print(s, file=sys.stderr),
                                                 sink_identifier, True))
        self.env._sinks.append(t)
        return DataStreamSink(self.env, t)

    def collect(self, target: list | None = None, with_subtask: bool = False) -> list:
        """Test sink: appends every record (optionally (subtask, value)) to a list."""
        target = [] if target is None else target
        t = Transformation(next(_ids), "Collect", "sink", [self.t],
                           lambda: O.CollectSinkOp(target, with_subtask))
        self.env._sinks.append(t)
        return target

    def write_as_text(self, path: str) -> "DataStreamSink":
        from ..utils.javafmt import java_str

        fh = {"f": None}

        class _W(F.RichSinkFunction):
            def open(self, p=None):
                fh["f"] = open(path, "w", encoding="utf-8")

            def invoke(self, value, ctx=None):
                if fh["f"] is None:
                    self.open()
                fh["f"].write(java_str(value) + "\n")

            def close(self):
                if fh["f"] is not None:
                    fh["f"].close()

        return self.add_sink(_W())

    # camelCase aliases
    flatMap = flat_map
    keyBy = key_by
    assignTimestampsAndWatermarks = assign_timestamps_and_watermarks
    timeWindowAll = time_window_all
    windowAll = window_all
    countWindowAll = count_window_all
    addSink = add_sink
    printToErr = print_to_err
    writeAsText = write_as_text


class SingleOutputStreamOperator(DataStream):
    def name(self, name: str) -> "SingleOutputStreamOperator":
        self.t.name = name
        return self

    def uid(self, uid: str) -> "SingleOutputStreamOperator":
        self.t.uid = uid
        return self

    def set_parallelism(self, p: int) -> "SingleOutputStreamOperator":
        if p < 1:
            raise ValueError("parallelism must be >= 1")
        self.t.parallelism = p
        return self

    def get_side_output(self, tag: OutputTag) -> DataStream:
        t = Transformation(next(_ids), f"SideOutput({tag.tag_id})", "side", [self.t], None,
                           side_tag=tag)
        return DataStream(self.env, t)

    def disable_chaining(self):
        return self

    setParallelism = set_parallelism
    getSideOutput = get_side_output
    disableChaining = disable_chaining


class DataStreamSink:
    def __init__(self, env, t):
        self.env, self.t = env, t

    def name(self, n):
        self.t.name = n
        return self

    def set_parallelism(self, p: int):
        self.t.parallelism = p
        return self

    def uid(self, u):
        self.t.uid = u
        return self

    setParallelism = set_parallelism


def _time_assigner(env, size, slide=None) -> W.WindowAssigner:
    size = to_ms(size)
    event = env.time_characteristic != TimeCharacteristic.ProcessingTime
    if slide is None:
        return W.TumblingEventTimeWindows.of(size) if event else W.TumblingProcessingTimeWindows.of(size)
    slide = to_ms(slide)
    return (W.SlidingEventTimeWindows.of(size, slide) if event
            else W.SlidingProcessingTimeWindows.of(size, slide))


class KeyedStream(DataStream):
    def __init__(self, parent: DataStream, key_fn, key_pos):
        super().__init__(parent.env, parent.t)
        self.key_fn = key_fn
        self.key_pos = key_pos

    def get_key_selector(self):
        return self.key_fn

    def _one_input(self, name: str, factory, parallelism: int | None = None):
        op = super()._one_input(name, factory, parallelism)
        op.t.key_fn_in = self.key_fn  # hash-partitioned edge (multi-rank record exchange)
        return op

    # -- rolling aggregations (StreamGroupedReduce: emit per element) --
    def reduce(self, fn) -> SingleOutputStreamOperator:
        key_fn = self.key_fn
        return self._one_input("Keyed Reduce", lambda: O.RollingReduceOp(key_fn, fn))

    def _agg(self, pos, kind: str) -> SingleOutputStreamOperator:
        from ..oracle.flink import flink_max_field, flink_min_field, flink_sum_field

        p = int(pos) if not isinstance(pos, str) else int(pos[1:])
        if kind == "sum":
            red = flink_sum_field(p)
        elif kind == "max":
            red = flink_max_field(p)
        elif kind == "min":
            red = flink_min_field(p)
        elif kind == "maxBy":
            red = lambda a, b: b if b[p] > a[p] else a
        else:
            red = lambda a, b: b if b[p] < a[p] else a
        from .tuples import Tuple

        def wrapped(a, b, red=red):
            r = red(tuple(a), tuple(b))
            return Tuple(r) if isinstance(a, tuple) else r

        key_fn = self.key_fn
        op = self._one_input("Keyed Aggregation", lambda: O.RollingReduceOp(key_fn, wrapped))
        op._rolling_spec = (kind, p, self.key_pos)
        op.t.meta = {"kind": "rolling", "agg": kind, "pos": p, "key_pos": self.key_pos,
                     "key_fn": key_fn}
        return op

    def sum(self, pos) -> SingleOutputStreamOperator:
        return self._agg(pos, "sum")

    def max(self, pos) -> SingleOutputStreamOperator:
        return self._agg(pos, "max")

    def min(self, pos) -> SingleOutputStreamOperator:
        return self._agg(pos, "min")

    def max_by(self, pos) -> SingleOutputStreamOperator:
        return self._agg(pos, "maxBy")

    def min_by(self, pos) -> SingleOutputStreamOperator:
        return self._agg(pos, "minBy")

    # -- keyed process / stateful map --
    def process(self, fn) -> SingleOutputStreamOperator:
        key_fn = self.key_fn
        return self._one_input("KeyedProcess", lambda: O.KeyedProcessOp(key_fn, fn))

    def map(self, fn) -> SingleOutputStreamOperator:
        if isinstance(fn, F.RichFunction):  # may use keyed state
            key_fn = self.key_fn
            return self._one_input("Keyed Map", lambda: O.KeyedProcessOp(key_fn, fn))
        return super().map(fn)

    def flat_map(self, fn) -> SingleOutputStreamOperator:
        if isinstance(fn, F.RichFunction):
            key_fn = self.key_fn
            return self._one_input("Keyed FlatMap", lambda: O.KeyedProcessOp(key_fn, fn))
        return super().flat_map(fn)

    def filter(self, fn) -> SingleOutputStreamOperator:
        if isinstance(fn, F.RichFunction):
            key_fn = self.key_fn
            return self._one_input("Keyed Filter", lambda: O.KeyedProcessOp(key_fn, fn))
        return super().filter(fn)

    # -- windows --
    def time_window(self, size, slide=None) -> "WindowedStream":
        return WindowedStream(self, _time_assigner(self.env, size, slide))

    def window(self, assigner: W.WindowAssigner) -> "WindowedStream":
        return WindowedStream(self, assigner)

    def count_window(self, size: int, slide: int | None = None) -> "WindowedStream":
        ws = WindowedStream(self, W.GlobalWindows.create())
        if slide is None:
            return ws.trigger(W.PurgingTrigger.of(W.CountTrigger.of(size)))
        return ws.evictor(W.CountEvictor.of(size)).trigger(W.CountTrigger.of(slide))

    maxBy = max_by
    minBy = min_by
    timeWindow = time_window
    countWindow = count_window
    flatMap = flat_map
    getKeySelector = get_key_selector


class WindowedStream:
    def __init__(self, keyed: KeyedStream | None, assigner: W.WindowAssigner, non_keyed_parent=None):
        self.keyed = keyed
        self.parent = keyed if keyed is not None else non_keyed_parent
        self.env = self.parent.env
        self.assigner = assigner
        self._trigger = None
        self._evictor = None
        self._lateness = 0
        self._late_tag = None

    def trigger(self, trigger: W.Trigger) -> "WindowedStream":
        if self.assigner.merging and not trigger.can_merge():
            raise ValueError("A merging window assigner cannot be used with a trigger that does not support merging.")
        self._trigger = trigger
        return self

    def evictor(self, evictor: W.Evictor) -> "WindowedStream":
        self._evictor = evictor
        return self

    def allowed_lateness(self, t) -> "WindowedStream":
        ms = to_ms(t)
        if ms < 0:
            raise ValueError("The allowed lateness cannot be negative.")
        self._lateness = ms
        return self

    def side_output_late_data(self, tag: OutputTag) -> "WindowedStream":
        self._late_tag = tag
        return self

    def _build(self, name: str, spec: O.WindowFunctionSpec, native_hint=None) -> SingleOutputStreamOperator:
        key_fn = self.keyed.key_fn if self.keyed is not None else None
        assigner, trig, ev, late, tag = (self.assigner, self._trigger, self._evictor,
                                         self._lateness, self._late_tag)
        non_keyed = self.keyed is None

        def factory():
            return O.WindowOp(key_fn, assigner, trig, ev, late, tag, spec, non_keyed=non_keyed)

        p = 1 if non_keyed else None
        op = self.parent._one_input(name, factory, parallelism=p)
        op.t.meta = {"kind": "window", "stream": self, "spec": spec, "native_hint": native_hint}
        return op

    def reduce(self, fn, window_fn=None) -> SingleOutputStreamOperator:
        return self._build("Window(Reduce)", O.WindowFunctionSpec("reduce", fn, window_fn))

    def aggregate(self, fn: F.AggregateFunction, window_fn=None) -> SingleOutputStreamOperator:
        return self._build("Window(Aggregate)", O.WindowFunctionSpec("aggregate", fn, window_fn))

    def process(self, fn: F.ProcessWindowFunction) -> SingleOutputStreamOperator:
        return self._build("Window(Process)", O.WindowFunctionSpec("process", fn))

    def apply(self, fn) -> SingleOutputStreamOperator:
        return self._build("Window(Apply)", O.WindowFunctionSpec("apply", fn))

    def _field_agg(self, pos, kind):
        from ..oracle.flink import flink_max_field, flink_min_field, flink_sum_field
        from .tuples import Tuple

        p = int(pos)
        red = {"sum": flink_sum_field(p), "max": flink_max_field(p), "min": flink_min_field(p),
               "maxBy": (lambda a, b: b if b[p] > a[p] else a),
               "minBy": (lambda a, b: b if b[p] < a[p] else a)}[kind]

        def wrapped(a, b, red=red):
            r = red(tuple(a), tuple(b))
            return Tuple(r) if isinstance(a, tuple) else r

        return self._build(f"Window({kind})", O.WindowFunctionSpec("reduce", wrapped),
                           native_hint=(kind, p))

    def sum(self, pos):
        return self._field_agg(pos, "sum")

    def max(self, pos):
        return self._field_agg(pos, "max")

    def min(self, pos):
        return self._field_agg(pos, "min")

    def max_by(self, pos):
        return self._field_agg(pos, "maxBy")

    def min_by(self, pos):
        return self._field_agg(pos, "minBy")

    allowedLateness = allowed_lateness
    sideOutputLateData = side_output_late_data
    maxBy = max_by
    minBy = min_by


class AllWindowedStream(WindowedStream):
    def __init__(self, parent: DataStream, assigner):
        super().__init__(None, assigner, non_keyed_parent=parent)
