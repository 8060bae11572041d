"""User-function interfaces (Flink 1.8 ``org.apache.flink.api.common.functions`` and
``streaming.api.functions``). Every operator also accepts a plain Python callable.

Reference uses: MapFunction (Main.java:18), FilterFunction (Main.java:27), ReduceFunction
(BandwidthMonitor.java:37), AggregateFunction (ComputeCpuAvg.java:31-58), ProcessWindowFunction
(ComputeCpuMiddle.java:34-48).
"""
from __future__ import annotations

from typing import Any, Iterable


class Function:
    pass


class RuntimeContext:
    """What a RichFunction sees: subtask info + keyed state access (keyed operators only)."""

    def __init__(self, task_name: str, subtask: int, parallelism: int, max_parallelism: int,
                 state_backend=None, metric_group=None):
        self.task_name = task_name
        self.index_of_this_subtask = subtask
        self.number_of_parallel_subtasks = parallelism
        self.max_number_of_parallel_subtasks = max_parallelism
        self._state = state_backend
        self._metrics = metric_group

    def get_index_of_this_subtask(self) -> int:
        return self.index_of_this_subtask

    def get_number_of_parallel_subtasks(self) -> int:
        return self.number_of_parallel_subtasks

    def get_task_name(self) -> str:
        return self.task_name

    def _require_state(self):
        if self._state is None:
            raise RuntimeError("Keyed state is only available on a KeyedStream")
        return self._state

    def get_state(self, descriptor):
        return self._require_state().get_state(descriptor)

    def get_list_state(self, descriptor):
        return self._require_state().get_state(descriptor)

    def get_map_state(self, descriptor):
        return self._require_state().get_state(descriptor)

    def get_reducing_state(self, descriptor):
        return self._require_state().get_state(descriptor)

    def get_aggregating_state(self, descriptor):
        return self._require_state().get_state(descriptor)

    def get_metric_group(self):
        return self._metrics

    # camelCase aliases
    getState = get_state
    getListState = get_list_state
    getMapState = get_map_state
    getReducingState = get_reducing_state
    getAggregatingState = get_aggregating_state
    getIndexOfThisSubtask = get_index_of_this_subtask
    getNumberOfParallelSubtasks = get_number_of_parallel_subtasks


class RichFunction(Function):
    _runtime_context: RuntimeContext | None = None

    def open(self, parameters=None):
        pass

    def close(self):
        pass

    def get_runtime_context(self) -> RuntimeContext:
        if self._runtime_context is None:
            raise RuntimeError("runtime context not set (function not opened)")
        return self._runtime_context

    def set_runtime_context(self, ctx: RuntimeContext):
        self._runtime_context = ctx

    getRuntimeContext = get_runtime_context


class MapFunction(Function):
    def map(self, value):
        raise NotImplementedError


class RichMapFunction(RichFunction, MapFunction):
    pass


class FilterFunction(Function):
    def filter(self, value) -> bool:
        raise NotImplementedError


class RichFilterFunction(RichFunction, FilterFunction):
    pass


class FlatMapFunction(Function):
    def flat_map(self, value, out: "Collector"):
        raise NotImplementedError

    def flatMap(self, value, out):  # camelCase
        return self.flat_map(value, out)


class RichFlatMapFunction(RichFunction, FlatMapFunction):
    pass


class KeySelector(Function):
    def get_key(self, value):
        raise NotImplementedError

    def getKey(self, value):
        return self.get_key(value)


class ReduceFunction(Function):
    def reduce(self, a, b):
        raise NotImplementedError


class AggregateFunction(Function):
    """createAccumulator / add / getResult / merge (ComputeCpuAvg.java:33-58)."""

    def create_accumulator(self):
        raise NotImplementedError

    def add(self, value, accumulator):
        raise NotImplementedError

    def get_result(self, accumulator):
        raise NotImplementedError

    def merge(self, a, b):
        raise NotImplementedError

    # Java names map onto the snake_case hooks
    def createAccumulator(self):
        return self.create_accumulator()

    def getResult(self, acc):
        return self.get_result(acc)


def _acc_fns(fn: AggregateFunction):
    """Resolve an AggregateFunction's hooks whether it defines Java or snake names."""

    def pick(snake, camel):
        m = getattr(type(fn), snake, None)
        base = getattr(AggregateFunction, snake)
        if m is not None and m is not base:
            return getattr(fn, snake)
        return getattr(fn, camel)

    return (pick("create_accumulator", "createAccumulator"), fn.add,
            pick("get_result", "getResult"), fn.merge)


class Collector:
    def __init__(self):
        self.items: list = []

    def collect(self, value):
        self.items.append(value)


class ProcessWindowFunction(RichFunction):
    """process(key, context, elements, out) (ComputeCpuMiddle.java:36)."""

    class Context:
        def __init__(self, window, current_processing_time: int, current_watermark: int,
                     side_outputs=None):
            self._window = window
            self._pt = current_processing_time
            self._wm = current_watermark
            self._side = side_outputs

        def window(self):
            return self._window

        def current_processing_time(self) -> int:
            return self._pt

        def current_watermark(self) -> int:
            return self._wm

        def output(self, tag, value):
            self._side.setdefault(tag.tag_id, []).append(value)

        currentProcessingTime = current_processing_time
        currentWatermark = current_watermark

    def process(self, key, context, elements: Iterable, out: Collector):
        raise NotImplementedError


class WindowFunction(Function):
    """apply(key, window, input, out)."""

    def apply(self, key, window, inputs: Iterable, out: Collector):
        raise NotImplementedError


class ProcessFunction(RichFunction):
    class Context:
        def __init__(self, ts, timer_service, side_outputs, key=None):
            self._ts = ts
            self._timers = timer_service
            self._side = side_outputs
            self._key = key

        def timestamp(self):
            return self._ts

        def timer_service(self):
            return self._timers

        def output(self, tag, value):
            self._side.setdefault(tag.tag_id, []).append(value)

        def get_current_key(self):
            return self._key

        timerService = timer_service
        getCurrentKey = get_current_key

    def process_element(self, value, ctx, out: Collector):
        raise NotImplementedError

    def on_timer(self, timestamp: int, ctx, out: Collector):
        pass


class KeyedProcessFunction(ProcessFunction):
    pass


class SinkFunction(Function):
    def invoke(self, value, context=None):
        raise NotImplementedError


class RichSinkFunction(RichFunction, SinkFunction):
    pass


class SourceFunction(Function):
    """run(ctx) calls ctx.collect(...) / ctx.collect_with_timestamp(...) / ctx.emit_watermark."""

    def run(self, ctx):
        raise NotImplementedError

    def cancel(self):
        pass


def call_map(fn, v):
    if isinstance(fn, MapFunction):
        return fn.map(v)
    return fn(v)


def call_filter(fn, v) -> bool:
    if isinstance(fn, FilterFunction):
        return bool(fn.filter(v))
    return bool(fn(v))


def call_reduce(fn, a, b):
    if isinstance(fn, ReduceFunction):
        return fn.reduce(a, b)
    return fn(a, b)


def call_key(fn, v):
    if isinstance(fn, KeySelector):
        return fn.get_key(v)
    return fn(v)


Any_ = Any
