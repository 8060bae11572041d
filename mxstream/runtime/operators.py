"""Generic (host, per-record) stream operators — the exact-semantics path for arbitrary Python
user functions. The executor (runtime/executor.py) swaps in native-backed operators
(runtime/native_ops.py) for the recognised hot shapes.

Stream model: an operator consumes a list of *items* — ``Rec(value, ts, subtask)`` records and
``WM(ts)`` watermarks, in stream order — and returns the items it emits. ``subtask`` is the
logical subtask index that printed ``N>`` prefixes expose (SURVEY.md F-print, A.5).

Flink 1.8 behaviour reproduced (class names are Flink's):
  StreamMap/StreamFilter/StreamFlatMap/ProcessOperator, TimestampsAndPeriodicWatermarksOperator,
  TimestampsAndPunctuatedWatermarksOperator, StreamGroupedReduce (rolling, emit per element,
  ComputeCpuMax.java:26), KeyedProcessOperator (timers), WindowOperator / EvictingWindowOperator
  (assign, trigger, fire, purge, cleanup timers, allowed lateness, late side output, merging
  session windows via MergingWindowSet).
"""
from __future__ import annotations

import copy
import heapq
import itertools
from dataclasses import dataclass
from typing import Any, Callable

import numpy as np

from ..api import functions as F
from ..api.state import (AggregatingStateDescriptor, HeapKeyedStateBackend, ListStateDescriptor,
                         ReducingStateDescriptor)
from ..api.watermarks import LONG_MAX, LONG_MIN, Watermark
from ..api.windowing import TimeWindow, TriggerResult
from ..utils.hashing import key_group


@dataclass
class Rec:
    value: Any
    ts: int = LONG_MIN
    subtask: int = 0


@dataclass
class WM:
    ts: int


class OpContext:
    """What the executor hands every operator at open()."""

    def __init__(self, name: str, parallelism: int, max_parallelism: int, clock: Callable[[], int],
                 time_characteristic: str, comm=None, ctrl=None):
        self.name = name
        self.parallelism = parallelism
        self.max_parallelism = max_parallelism
        self.clock = clock
        self.time_characteristic = time_characteristic
        # Multi-rank jobs: `comm` carries device tensors (RCCL for GPU operators, gloo/loopback
        # otherwise), `ctrl` host objects; both None on one rank.
        self.comm = comm
        self.ctrl = ctrl


class Operator:
    name = "op"

    def open(self, ctx: OpContext) -> None:
        self.ctx = ctx
        self.side: dict[str, list] = {}

    def process(self, items: list) -> list:
        out = []
        for it in items:
            if isinstance(it, WM):
                out.extend(self.on_watermark(it.ts))
                out.append(it)
            else:
                out.extend(self.on_record(it))
        return out

    def on_record(self, r: Rec) -> list:
        return [r]

    def on_watermark(self, wm: int) -> list:
        return []

    def on_processing_time(self, now: int) -> list:
        return []

    def finish(self) -> list:
        """End of input (after the final MAX watermark for event time)."""
        return []

    def close(self) -> None:
        pass

    def take_side(self, tag_id: str) -> list:
        return self.side.pop(tag_id, [])

    def snapshot(self) -> dict:
        return {}

    def restore(self, snap: dict) -> None:
        pass


def _open_fn(fn, ctx: OpContext, subtask: int = 0, state_backend=None):
    if isinstance(fn, F.RichFunction):
        fn.set_runtime_context(F.RuntimeContext(ctx.name, subtask, ctx.parallelism,
                                                ctx.max_parallelism, state_backend))
        fn.open(None)


class MapOp(Operator):
    name = "Map"

    def __init__(self, fn):
        self.fn = fn

    def open(self, ctx):
        super().open(ctx)
        _open_fn(self.fn, ctx)

    def on_record(self, r):
        return [Rec(F.call_map(self.fn, r.value), r.ts, r.subtask)]


class FilterOp(Operator):
    name = "Filter"

    def __init__(self, fn):
        self.fn = fn

    def open(self, ctx):
        super().open(ctx)
        _open_fn(self.fn, ctx)

    def on_record(self, r):
        return [r] if F.call_filter(self.fn, r.value) else []


class FlatMapOp(Operator):
    name = "Flat Map"

    def __init__(self, fn):
        self.fn = fn

    def open(self, ctx):
        super().open(ctx)
        _open_fn(self.fn, ctx)

    def on_record(self, r):
        col = F.Collector()
        if isinstance(self.fn, F.FlatMapFunction):
            self.fn.flat_map(r.value, col)
        else:
            res = self.fn(r.value, col)
            if res is not None and not col.items:
                col.items.extend(res)
        return [Rec(v, r.ts, r.subtask) for v in col.items]


class RebalanceOp(Operator):
    """Round-robin channel selection (RebalancePartitioner) from a parallelism-1 source."""

    name = "Rebalance"

    def __init__(self, start: int = 0):
        self.next = start

    def on_record(self, r):
        p = self.ctx.parallelism
        sub = self.next % p
        self.next += 1
        return [Rec(r.value, r.ts, sub)]


class ProcessOp(Operator):
    """ProcessOperator (non-keyed ProcessFunction): no timers, side outputs allowed."""

    name = "Process"

    def __init__(self, fn: F.ProcessFunction):
        self.fn = fn
        self.wm = LONG_MIN

    def open(self, ctx):
        super().open(ctx)
        _open_fn(self.fn, ctx)

    def on_watermark(self, wm):
        self.wm = wm
        return []

    def on_record(self, r):
        col = F.Collector()
        c = F.ProcessFunction.Context(None if r.ts == LONG_MIN else r.ts, _NoTimers(self), self.side)
        self.fn.process_element(r.value, c, col)
        return [Rec(v, r.ts, r.subtask) for v in col.items]


class _NoTimers:
    def __init__(self, op):
        self.op = op

    def current_processing_time(self):
        return self.op.ctx.clock()

    def current_watermark(self):
        return self.op.wm

    def register_event_time_timer(self, t):
        raise RuntimeError("Setting timers is only supported on a keyed streams.")

    register_processing_time_timer = register_event_time_timer
    currentProcessingTime = current_processing_time
    currentWatermark = current_watermark


class TimestampsAndWatermarksOp(Operator):
    """Assigns timestamps; periodic assigners emit a watermark after each micro-batch (the
    engine's auto-watermark interval), punctuated ones inline after the triggering element."""

    name = "Timestamps/Watermarks"

    def __init__(self, assigner):
        # Each (re)started task gets its own copy of the user assigner, as Flink deserializes one
        # per task: a restarted job must not inherit the failed attempt's max timestamp.
        self.assigner = copy.deepcopy(assigner)
        self.current = LONG_MIN

    def process(self, items):
        out = []
        periodic = getattr(self.assigner, "periodic", True)
        for it in items:
            if isinstance(it, WM):
                # Upstream watermarks are swallowed except the end-of-input MAX (Flink 1.8).
                if it.ts == LONG_MAX:
                    self.current = LONG_MAX
                    out.append(it)
                continue
            ts = self.assigner.extract_timestamp(it.value, it.ts)
            out.append(Rec(it.value, ts, it.subtask))
            if not periodic:
                w = self.assigner.check_and_get_next_watermark(it.value, ts)
                if w is not None and w.timestamp > self.current:
                    self.current = w.timestamp
                    out.append(WM(w.timestamp))
        if periodic:
            w = self.assigner.get_current_watermark()
            if w is not None and w.timestamp > self.current:
                self.current = w.timestamp
                out.append(WM(w.timestamp))
        return out

    def on_processing_time(self, now):
        if getattr(self.assigner, "periodic", True):
            w = self.assigner.get_current_watermark()
            if w is not None and w.timestamp > self.current:
                self.current = w.timestamp
                return [WM(w.timestamp)]
        return []


# ---- keyed operators ----------------------------------------------------------------------

class KeyedOperator(Operator):
    def __init__(self, key_fn):
        self.key_fn = key_fn

    def open(self, ctx):
        super().open(ctx)
        self.backend = HeapKeyedStateBackend(ctx.max_parallelism)

    def subtask_of(self, key) -> int:
        kg = key_group(key, self.ctx.max_parallelism)
        return kg * self.ctx.parallelism // self.ctx.max_parallelism

    def snapshot(self) -> dict:
        return {"keyed": self.backend.snapshot()}

    def restore(self, snap: dict) -> None:
        if "keyed" in snap:
            self.backend.restore(snap["keyed"])


class RollingReduceOp(KeyedOperator):
    """StreamGroupedReduce: reduce into ValueState and emit the new value for every element."""

    name = "Keyed Reduce"

    def __init__(self, key_fn, reduce_fn):
        super().__init__(key_fn)
        self.reduce_fn = reduce_fn

    def on_record(self, r):
        key = F.call_key(self.key_fn, r.value)
        st = self.backend._table("_rolling")
        if key in st:
            nv = F.call_reduce(self.reduce_fn, st[key], r.value)
        else:
            nv = r.value
        st[key] = nv
        return [Rec(nv, r.ts, self.subtask_of(key))]


class _Timers:
    """InternalTimerService: event + processing timers keyed by (ts, key, namespace)."""

    def __init__(self):
        self.event: list = []
        self.proc: list = []
        self.event_set: set = set()
        self.proc_set: set = set()
        self._seq = itertools.count()

    def reg(self, kind: str, ts: int, key, ns):
        s, h = (self.event_set, self.event) if kind == "event" else (self.proc_set, self.proc)
        k = (ts, _hk(key), _hk(ns))
        if k in s:
            return
        s.add(k)
        heapq.heappush(h, (ts, next(self._seq), key, ns))

    def delete(self, kind: str, ts: int, key, ns):
        s = self.event_set if kind == "event" else self.proc_set
        s.discard((ts, _hk(key), _hk(ns)))

    def pop_due(self, kind: str, t: int):
        s, h = (self.event_set, self.event) if kind == "event" else (self.proc_set, self.proc)
        while h and h[0][0] <= t:
            ts, _, key, ns = heapq.heappop(h)
            k = (ts, _hk(key), _hk(ns))
            if k not in s:
                continue  # deleted
            s.discard(k)
            yield ts, key, ns

    def snapshot(self):
        return {"event": sorted((ts, k, n) for ts, _, k, n in self.event
                                if (ts, _hk(k), _hk(n)) in self.event_set),
                "proc": sorted((ts, k, n) for ts, _, k, n in self.proc
                               if (ts, _hk(k), _hk(n)) in self.proc_set)}

    def restore(self, snap):
        for ts, k, n in snap.get("event", []):
            self.reg("event", ts, k, n)
        for ts, k, n in snap.get("proc", []):
            self.reg("proc", ts, k, n)


def _hk(x):
    try:
        hash(x)
        return x
    except TypeError:
        return repr(x)


class _TimerService:
    def __init__(self, op: "KeyedProcessOp", key):
        self.op, self.key = op, key

    def current_processing_time(self):
        return self.op.ctx.clock()

    def current_watermark(self):
        return self.op.wm

    def register_event_time_timer(self, t):
        self.op.timers.reg("event", int(t), self.key, None)

    def register_processing_time_timer(self, t):
        self.op.timers.reg("proc", int(t), self.key, None)

    def delete_event_time_timer(self, t):
        self.op.timers.delete("event", int(t), self.key, None)

    def delete_processing_time_timer(self, t):
        self.op.timers.delete("proc", int(t), self.key, None)

    currentProcessingTime = current_processing_time
    currentWatermark = current_watermark
    registerEventTimeTimer = register_event_time_timer
    registerProcessingTimeTimer = register_processing_time_timer
    deleteEventTimeTimer = delete_event_time_timer
    deleteProcessingTimeTimer = delete_processing_time_timer


class KeyedProcessOp(KeyedOperator):
    """KeyedProcessOperator: per-element callback with keyed state and timers. Also backs
    keyed Rich{Map,FlatMap,Filter}Functions that use ValueState (BASELINE config 2)."""

    name = "KeyedProcess"

    def __init__(self, key_fn, fn):
        super().__init__(key_fn)
        self.fn = fn
        self.wm = LONG_MIN

    def open(self, ctx):
        super().open(ctx)
        self.timers = _Timers()
        _open_fn(self.fn, ctx, state_backend=self.backend)

    def _call(self, value, ts, key) -> list:
        col = F.Collector()
        self.backend.set_current_key(key)
        self.backend.set_current_namespace(None)
        fn = self.fn
        if isinstance(fn, F.ProcessFunction):
            c = F.ProcessFunction.Context(None if ts == LONG_MIN else ts, _TimerService(self, key),
                                          self.side, key)
            fn.process_element(value, c, col)
        elif isinstance(fn, F.FlatMapFunction):
            fn.flat_map(value, col)
        elif isinstance(fn, F.FilterFunction):
            if fn.filter(value):
                col.collect(value)
        elif isinstance(fn, F.MapFunction):
            col.collect(fn.map(value))
        else:
            col.collect(fn(value))
        sub = self.subtask_of(key)
        return [Rec(v, ts, sub) for v in col.items]

    def on_record(self, r):
        key = F.call_key(self.key_fn, r.value)
        return self._call(r.value, r.ts, key)

    def _fire(self, ts, key, domain) -> list:
        if not isinstance(self.fn, F.ProcessFunction):
            return []
        col = F.Collector()
        self.backend.set_current_key(key)
        self.backend.set_current_namespace(None)
        c = F.ProcessFunction.Context(ts, _TimerService(self, key), self.side, key)
        c.time_domain = domain
        self.fn.on_timer(ts, c, col)
        sub = self.subtask_of(key)
        return [Rec(v, ts, sub) for v in col.items]

    def on_watermark(self, wm):
        self.wm = wm
        out = []
        for ts, key, _ in self.timers.pop_due("event", wm):
            out.extend(self._fire(ts, key, "EVENT_TIME"))
        return out

    def on_processing_time(self, now):
        out = []
        for ts, key, _ in self.timers.pop_due("proc", now):
            out.extend(self._fire(ts, key, "PROCESSING_TIME"))
        return out

    def snapshot(self):
        return {"keyed": self.backend.snapshot(), "timers": self.timers.snapshot(), "wm": self.wm}

    def restore(self, snap):
        super().restore(snap)
        self.timers.restore(snap.get("timers", {}))
        self.wm = snap.get("wm", LONG_MIN)


# ---- windows ------------------------------------------------------------------------------

@dataclass
class WindowFunctionSpec:
    """How window contents are stored and emitted.

    kind: 'reduce' | 'aggregate' | 'process' | 'apply'
    fn: ReduceFunction / AggregateFunction / ProcessWindowFunction / WindowFunction
    window_fn: optional ProcessWindowFunction / WindowFunction applied on the pre-aggregate
    """

    kind: str
    fn: Any
    window_fn: Any = None


class _TriggerCtx:
    def __init__(self, op: "WindowOp"):
        self.op = op
        self.key = None
        self.window = None

    def get_current_watermark(self):
        return self.op.wm

    def get_current_processing_time(self):
        return self.op.ctx.clock()

    def register_event_time_timer(self, t):
        self.op.timers.reg("event", int(t), self.key, self.window)

    def register_processing_time_timer(self, t):
        self.op.timers.reg("proc", int(t), self.key, self.window)

    def delete_event_time_timer(self, t):
        self.op.timers.delete("event", int(t), self.key, self.window)

    def delete_processing_time_timer(self, t):
        self.op.timers.delete("proc", int(t), self.key, self.window)

    def get_partitioned_state(self, name, default=None):
        return self.op.trigger_state.get((self.key, self.window, name), default)

    def set_partitioned_state(self, name, value):
        self.op.trigger_state[(self.key, self.window, name)] = value

    def clear_partitioned(self):
        for k in [k for k in self.op.trigger_state if k[0] == self.key and k[1] == self.window]:
            del self.op.trigger_state[k]


class WindowOp(KeyedOperator):
    """WindowOperator / EvictingWindowOperator with Flink 1.8 semantics."""

    name = "Window"

    def __init__(self, key_fn, assigner, trigger=None, evictor=None, allowed_lateness: int = 0,
                 late_tag=None, wfn: WindowFunctionSpec | None = None, non_keyed: bool = False):
        super().__init__(key_fn)
        self.assigner = assigner
        self.trigger = trigger or assigner.default_trigger()
        self.evictor = evictor
        self.lateness = int(allowed_lateness)
        self.late_tag = late_tag
        self.wfn = wfn
        self.non_keyed = non_keyed
        self.wm = LONG_MIN
        self.num_late_records_dropped = 0

    def open(self, ctx):
        super().open(ctx)
        self.timers = _Timers()
        self.trigger_state: dict = {}
        self.tctx = _TriggerCtx(self)
        self.merging: dict = {}  # key -> {window: state_window}
        k = self.wfn.kind
        if self.evictor is not None or k in ("process", "apply"):
            self.desc = ListStateDescriptor("window-contents")
        elif k == "reduce":
            self.desc = ReducingStateDescriptor("window-contents", self.wfn.fn)
        elif k == "aggregate":
            self.desc = AggregatingStateDescriptor("window-contents", self.wfn.fn)
        else:
            raise ValueError(k)
        self.state = self.backend.get_state(self.desc)
        for f in (self.wfn.fn, self.wfn.window_fn):
            if f is not None:
                _open_fn(f, ctx, state_backend=None)

    # -- helpers --
    def _cleanup_time(self, w) -> int:
        if self.assigner.is_event_time():
            c = w.max_timestamp() + self.lateness
            return c if c >= w.max_timestamp() else LONG_MAX
        return w.max_timestamp()

    def _is_window_late(self, w) -> bool:
        return self.assigner.is_event_time() and self._cleanup_time(w) <= self.wm

    def _is_element_late(self, ts) -> bool:
        return self.assigner.is_event_time() and ts + self.lateness <= self.wm

    def _register_cleanup(self, key, w):
        c = self._cleanup_time(w)
        if c == LONG_MAX:
            return
        self.timers.reg("event" if self.assigner.is_event_time() else "proc", c, key, w)

    def _set(self, key, ns):
        self.backend.set_current_key(key)
        self.backend.set_current_namespace(ns)
        self.tctx.key = key
        self.tctx.window = ns

    def _contents(self):
        if self.desc.kind == "list":
            return self.state.get() or None
        return self.state.get()

    def _emit(self, key, window, contents) -> list:
        """emitWindowContents: user function output timestamped window.maxTimestamp()."""
        col = F.Collector()
        w = self.wfn
        if self.evictor is not None:
            elems = list(contents)
            n = len(elems)
            elems = self.evictor.evict_before(elems, n, window, None)
            vals = [v for v, _ts in elems]
            if w.kind == "reduce":
                acc = None
                for v in vals:
                    acc = v if acc is None else F.call_reduce(w.fn, acc, v)
                agg = [acc] if acc is not None else []
            elif w.kind == "aggregate":
                create, add, result, _ = F._acc_fns(w.fn)
                acc = create()
                for v in vals:
                    acc = add(v, acc)
                agg = [result(acc)]
            else:
                agg = vals
            if w.kind in ("reduce", "aggregate") and w.window_fn is None:
                for v in agg:
                    col.collect(v)
            else:
                self._call_window_fn(w.window_fn or w.fn, key, window, agg, col)
            rest = self.evictor.evict_after(elems, len(elems), window, None)
            self.state.update(rest)
        elif w.kind == "reduce":
            if w.window_fn is None:
                col.collect(contents)
            else:
                self._call_window_fn(w.window_fn, key, window, [contents], col)
        elif w.kind == "aggregate":
            if w.window_fn is None:
                col.collect(contents)
            else:
                self._call_window_fn(w.window_fn, key, window, [contents], col)
        else:
            self._call_window_fn(w.fn, key, window, [v for v, _ts in contents], col)
        sub = 0 if self.non_keyed else self.subtask_of(key)
        ts = window.max_timestamp()
        return [Rec(v, ts, sub) for v in col.items]

    def _call_window_fn(self, fn, key, window, elements, col):
        if isinstance(fn, F.ProcessWindowFunction):
            c = F.ProcessWindowFunction.Context(window, self.ctx.clock(), self.wm, self.side)
            fn.process(key, c, elements, col)
        elif isinstance(fn, F.WindowFunction):
            fn.apply(key, window, elements, col)
        elif self.non_keyed:
            fn(window, elements, col)
        else:
            fn(key, window, elements, col)

    def _add(self, value, ts):
        if self.desc.kind == "list":
            self.state.add((value, ts))
        else:
            self.state.add(value)

    # -- element path --
    def on_record(self, r):
        key = None if self.non_keyed else F.call_key(self.key_fn, r.value)
        now = self.ctx.clock()
        windows = self.assigner.assign_windows(r.value, r.ts, now)
        skipped = True
        out = []
        if self.assigner.merging:
            mws = self.merging.setdefault(_hk(key), {})
            for w in windows:
                actual = self._add_merging_window(key, mws, w)
                if self._is_window_late(actual):
                    mws.pop(actual, None)
                    continue
                skipped = False
                state_w = mws[actual]
                self._set(key, state_w)
                self._add(r.value, r.ts)
                self.tctx.window = actual
                res = self.trigger.on_element(r.value, r.ts, actual, self.tctx)
                if res.is_fire:
                    self._set(key, state_w)
                    c = self._contents()
                    if c is not None:
                        out.extend(self._emit(key, actual, c))
                if res.is_purge:
                    self._set(key, state_w)
                    self.state.clear()
                self._register_cleanup(key, actual)
        else:
            for w in windows:
                if self._is_window_late(w):
                    continue
                skipped = False
                self._set(key, w)
                self._add(r.value, r.ts)
                res = self.trigger.on_element(r.value, r.ts, w, self.tctx)
                if res.is_fire:
                    c = self._contents()
                    if c is not None:
                        out.extend(self._emit(key, w, c))
                if res.is_purge:
                    self.state.clear()
                self._register_cleanup(key, w)
        if skipped and self._is_element_late(r.ts):
            if self.late_tag is not None:
                self.side.setdefault(self.late_tag.tag_id, []).append(Rec(r.value, r.ts, r.subtask))
            else:
                self.num_late_records_dropped += 1
        return out

    def _add_merging_window(self, key, mapping: dict, new_w):
        """MergingWindowSet.addWindow with the WindowOperator merge callback."""
        windows = list(mapping.keys()) + [new_w]
        merges = []
        for merged, members in _merge_windows(windows):
            if len(members) > 1:
                merges.append((merged, list(members)))
        result = new_w
        merged_new = False
        for merge_result, merged_windows in merges:
            if new_w in merged_windows:
                merged_windows.remove(new_w)
                merged_new = True
                result = merge_result
            if not merged_windows:
                continue
            merged_state_window = mapping[merged_windows[0]]
            merged_state_windows = []
            for mw in merged_windows:
                res = mapping.pop(mw, None)
                if res is not None:
                    merged_state_windows.append(res)
            mapping[merge_result] = merged_state_window
            if merged_state_window in merged_state_windows:
                merged_state_windows.remove(merged_state_window)
            if not (merge_result in merged_windows and len(merged_windows) == 1):
                # WindowOperator merge callback
                if self.assigner.is_event_time() and merge_result.max_timestamp() + self.lateness <= self.wm:
                    raise RuntimeError("The end timestamp of an event-time window cannot become "
                                       "earlier than the current watermark by merging.")
                self.tctx.key = key
                self.tctx.window = merge_result
                if self.trigger.can_merge():
                    self.trigger.on_merge(merge_result, self.tctx)
                for m in merged_windows:
                    self.tctx.window = m
                    self.trigger.clear(m, self.tctx)
                    self.tctx.clear_partitioned()
                    self.timers.delete("event" if self.assigner.is_event_time() else "proc",
                                       self._cleanup_time(m), key, m)
                self.backend.set_current_key(key)
                self.backend.merge_namespaces(self.desc, mapping[merge_result], merged_state_windows)
        if not merges or (result == new_w and not merged_new):
            mapping[result] = result
        return result

    # -- timers --
    def _on_timer(self, ts, key, window, event: bool) -> list:
        out = []
        if self.assigner.merging:
            mws = self.merging.get(_hk(key), {})
            state_w = mws.get(window)
            if state_w is None:
                return out
        else:
            state_w = window
        self._set(key, state_w)
        self.tctx.window = window
        res = (self.trigger.on_event_time(ts, window, self.tctx) if event
               else self.trigger.on_processing_time(ts, window, self.tctx))
        if res.is_fire:
            self._set(key, state_w)
            c = self._contents()
            if c is not None:
                out.extend(self._emit(key, window, c))
        if res.is_purge:
            self._set(key, state_w)
            self.state.clear()
        if (event == self.assigner.is_event_time()) and ts == self._cleanup_time(window):
            self._set(key, state_w)
            self.state.clear()
            self.tctx.window = window
            self.trigger.clear(window, self.tctx)
            self.tctx.clear_partitioned()
            if self.assigner.merging:
                self.merging.get(_hk(key), {}).pop(window, None)
        return out

    def on_watermark(self, wm):
        self.wm = wm
        out = []
        for ts, key, w in self.timers.pop_due("event", wm):
            out.extend(self._on_timer(ts, key, w, True))
        return out

    def on_processing_time(self, now):
        out = []
        for ts, key, w in self.timers.pop_due("proc", now):
            out.extend(self._on_timer(ts, key, w, False))
        return out

    def snapshot(self):
        return {"keyed": self.backend.snapshot(), "timers": self.timers.snapshot(), "wm": self.wm,
                "merging": {k: dict(v) for k, v in self.merging.items()},
                "trigger_state": dict(self.trigger_state)}

    def restore(self, snap):
        super().restore(snap)
        self.timers.restore(snap.get("timers", {}))
        self.wm = snap.get("wm", LONG_MIN)
        self.merging = {k: dict(v) for k, v in snap.get("merging", {}).items()}
        self.trigger_state = dict(snap.get("trigger_state", {}))


def _merge_windows(windows):
    from ..api.windowing import merge_time_windows

    return merge_time_windows(windows)


# ---- sinks --------------------------------------------------------------------------------

class SinkOp(Operator):
    name = "Sink"

    def __init__(self, fn):
        self.fn = fn

    def open(self, ctx):
        super().open(ctx)
        _open_fn(self.fn, ctx)

    def on_record(self, r):
        if isinstance(self.fn, F.SinkFunction):
            self.fn.invoke(r.value, r)
        else:
            self.fn(r.value)
        return []

    def close(self):
        if isinstance(self.fn, F.RichFunction):
            self.fn.close()


# Device column batches are printed by the device row formatter (ops/rowfmt.py);
# MXS_DEVICE_FORMAT=0 formats them on the host (A/B).
_DEVICE_FORMAT = __import__("os").environ.get("MXS_DEVICE_FORMAT", "1") != "0"


class PrintSinkOp(Operator):
    """PrintSinkFunction: '{subtask+1}> ' + toString when parallelism > 1."""

    name = "Print to Std. Out"

    def __init__(self, writer: Callable[[str], None], sink_identifier: str | None = None,
                 to_stderr: bool = False, parallelism: int | None = None):
        self.writer = writer
        self.ident = sink_identifier
        self.to_stderr = to_stderr
        self.parallelism = parallelism

    accepts_columns = True

    def process(self, items: list) -> list:
        from .columnar import ColumnBatch

        if not any(isinstance(it, ColumnBatch) for it in items):
            return super().process(items)
        out = []
        for it in items:
            if isinstance(it, ColumnBatch):
                self._print_columns(it)
            else:
                out.extend(super().process([it]))
        return out

    def _prefixes(self, nsub: int) -> list[str]:
        p = self.parallelism or self.ctx.parallelism
        if self.ident:
            return [self.ident + (f":{k + 1}> " if p > 1 else "> ") for k in range(nsub)]
        return [f"{k + 1}> " if p > 1 else "" for k in range(nsub)]

    def _dict_names(self, d) -> list:
        """The names of dictionary `d` by id (mirror kept across batches, extended in place)."""
        cache = getattr(self, "_names_of", None)
        if cache is None or cache[0] is not d:
            cache = self._names_of = (d, [])
        names = cache[1]
        n = len(d)
        if len(names) < n:
            names.extend(d.get(i) for i in range(len(names), n))
        return names

    def _print_columns(self, cb) -> None:
        """A column batch in one native call (csrc/javafmt.h: Tuple/Double/Long toString), the
        lines handed to the writer at once when it takes many (the default stdout writer)."""
        from ..ops.native import load
        from ..ops.text import FK_DOUBLE, FK_INT, FK_LONG, FK_STR

        if hasattr(cb, "host") and cb.n and _DEVICE_FORMAT:
            # device batch: formatted where its columns live, one copy of the finished bytes
            if getattr(self, "_rowfmt", None) is None:
                from ..ops.rowfmt import RowFormatter

                self._rowfmt = RowFormatter()
            p = self.parallelism or self.ctx.parallelism
            mv = self._rowfmt.format(cb, self._prefixes(max(1, p)),
                                     not getattr(cb, "scalar", False))
            if mv is not None:
                raw = getattr(self.writer, "raw", None)
                if raw is not None:
                    raw(mv, cb.n)
                    return
                lines = bytes(mv).decode().split("\n")[:-1]
                many = getattr(self.writer, "many", None)
                if many is not None:
                    many(lines)
                else:
                    for ln in lines:
                        self.writer(ln)
                return
        cb = cb.host() if hasattr(cb, "host") else cb
        if cb.n == 0:
            return
        cols, keep, names = [], [], None
        # Dictionary ids index the dictionary's whole name list when it is not much larger than
        # the batch (a cached mirror, extended as the dictionary grows): no per-batch unique
        # (two sorts of the id columns) before formatting.
        whole = None
        if FK_STR in cb.kinds and cb.strings is not None and hasattr(cb.strings, "strings") \
                and len(cb.strings) <= 4 * cb.n + 4096:
            whole = self._dict_names(cb.strings)
        for c, k in zip(cb.cols, cb.kinds):
            c = np.asarray(c)[:cb.n]
            if k == FK_STR and whole is not None:
                names = whole
                a = np.ascontiguousarray(c, dtype=np.int64)
                cols.append((0, a.ctypes.data))
            elif k == FK_STR:
                u, inv = np.unique(c, return_inverse=True)
                if names is not None:  # several string columns: one name list for all
                    off = len(names)
                    names.extend(cb.strings.get(int(x)) for x in u.tolist())
                else:
                    off, names = 0, [cb.strings.get(int(x)) for x in u.tolist()]
                a = np.ascontiguousarray(inv.reshape(-1).astype(np.int64) + off)
                cols.append((0, a.ctypes.data))
            elif k == FK_DOUBLE:
                a = np.ascontiguousarray(c, dtype=np.float64)
                cols.append((1, a.ctypes.data))
            elif k in (FK_LONG, FK_INT):
                a = np.ascontiguousarray(c, dtype=np.int64)
                cols.append((2, a.ctypes.data))
            else:  # a kind without a bulk format: the per-record path
                for r in cb.to_recs():
                    self.on_record(r)
                return
            keep.append(a)
        sub = cb.sub
        if sub is not None:
            sub = np.ascontiguousarray(sub[:cb.n], dtype=np.int32)
            keep.append(sub)
        nsub = int(sub.max()) + 1 if sub is not None else 1
        as_tuple = not getattr(cb, "scalar", False)
        raw = getattr(self.writer, "raw", None)
        if raw is not None:
            # one bytes object formatted by native threads (no Python string per row)
            import os

            raw(load().java_format_bytes(cols, cb.n, names, 0 if sub is None else sub.ctypes.data,
                                         self._prefixes(nsub), as_tuple,
                                         min(16, os.cpu_count() or 1)), cb.n)
            return
        lines = load().java_format_rows(cols, cb.n, names, 0 if sub is None else sub.ctypes.data,
                                        self._prefixes(nsub), as_tuple)
        many = getattr(self.writer, "many", None)
        if many is not None:
            many(lines)
        else:
            for ln in lines:
                self.writer(ln)

    def on_record(self, r):
        from ..utils.javafmt import java_str

        p = self.parallelism or self.ctx.parallelism
        prefix = ""
        if self.ident:
            prefix = self.ident + (f":{r.subtask + 1}> " if p > 1 else "> ")
        elif p > 1:
            prefix = f"{r.subtask + 1}> "
        self.writer(prefix + java_str(r.value))
        return []


class CollectSinkOp(Operator):
    name = "Collect"

    def __init__(self, target: list, with_subtask: bool = False):
        self.target = target
        self.with_subtask = with_subtask

    def on_record(self, r):
        self.target.append((r.subtask, r.value) if self.with_subtask else r.value)
        return []


class UnionOp(Operator):
    """Merges inputs; the output watermark is the minimum over inputs (StatusWatermarkValve)."""

    name = "Union"

    def __init__(self, n_inputs: int):
        self.wms = [LONG_MIN] * n_inputs
        self.cur = LONG_MIN

    def process_input(self, idx: int, items: list) -> list:
        out = []
        for it in items:
            if isinstance(it, WM):
                self.wms[idx] = max(self.wms[idx], it.ts)
                m = min(self.wms)
                if m > self.cur:
                    self.cur = m
                    out.append(WM(m))
            else:
                out.append(it)
        return out


__all__ = [n for n in dir() if not n.startswith("_")]
_ = (Watermark, TimeWindow, TriggerResult)
