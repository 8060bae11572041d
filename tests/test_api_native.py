"""Differential tests: native keyed-window path (C++ twin) == exact host WindowOperator."""
from collections import Counter

from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from mxstream.api.environment import StreamExecutionEnvironment
from mxstream.api.time import Time, TimeCharacteristic
from mxstream.api.tuples import Tuple2, Tuple3
from mxstream.api.watermarks import BoundedOutOfOrdernessTimestampExtractor
from mxstream.runtime.executor import ManualClock


def _run(events, size, slide, bound, lateness, native, agg="reduce"):
    out = []
    env = StreamExecutionEnvironment(4, clock=ManualClock(0)).set_output(out.append)
    env.config.native = native
    env.set_stream_time_characteristic(TimeCharacteristic.EventTime)
    timed = [(i + 1, e) for i, e in enumerate(events)]
    ws = (env.from_timed_collection(timed)
          .assign_timestamps_and_watermarks(
              BoundedOutOfOrdernessTimestampExtractor(Time.milliseconds(bound), extractor=lambda e: e[2]))
          .map(lambda e: Tuple2(e[0], e[1]))
          .key_by(0)
          .time_window(Time.milliseconds(size), Time.milliseconds(slide))
          .allowed_lateness(Time.milliseconds(lateness)))
    if agg == "reduce":
        s = ws.reduce(lambda a, b: Tuple2(a.f0, a.f1 + b.f1))
    elif agg == "max":
        s = ws.max(1)
    else:
        s = ws.min(1)
    s.print()
    env.execute("diff")
    return out


def _final(out):
    """Last emission per (prefix, key, window order) is what both paths must agree on."""
    return Counter(out)


events_st = st.lists(
    st.tuples(st.sampled_from(["a", "b", "c", "d", "www.163.com"]), st.integers(0, 1000),
              st.integers(0, 20_000)),
    min_size=1, max_size=40)


@settings(max_examples=60, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(events=events_st, size_k=st.integers(1, 6), slide_div=st.sampled_from([1, 2, 3]),
       bound=st.sampled_from([0, 500, 3000]), agg=st.sampled_from(["reduce", "max", "min"]))
def test_native_equals_host_no_lateness(events, size_k, slide_div, bound, agg):
    size = size_k * 1200
    slide = size // slide_div
    a = _run(events, size, slide, bound, 0, "off", agg)
    b = _run(events, size, slide, bound, 0, "auto", agg)
    assert Counter(a) == Counter(b)


@settings(max_examples=40, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(events=events_st, bound=st.sampled_from([0, 1000]), lateness=st.sampled_from([500, 4000]))
def test_native_equals_host_with_lateness_final_values(events, bound, lateness):
    # With allowed lateness Flink fires once per late element; the micro-batch engine may fold
    # several late elements of one micro-batch into one firing. Each line is its own batch
    # here, so outputs must match exactly.
    a = _run(events, 2000, 1000, bound, lateness, "off")
    b = _run(events, 2000, 1000, bound, lateness, "auto")
    assert Counter(a) == Counter(b)


def test_native_path_is_selected():
    from mxstream.api import planner
    from mxstream.runtime.native_ops import NativeWindowOp

    env = StreamExecutionEnvironment(4)
    (env.from_collection([("a", 1)]).key_by(0).time_window(Time.seconds(1))
     .reduce(lambda a, b: Tuple2(a.f0, a.f1 + b.f1)).print())
    sinks = planner.plan(env, list(env._sinks))
    from mxstream.runtime.executor import Executor

    ops = [n.factory() for n in Executor._topo(sinks) if n.kind == "op"]
    assert any(isinstance(o, NativeWindowOp) for o in ops)


# ---- keyed rolling aggregations: NativeRollingOp vs the host RollingReduceOp ------------------
def _run_rolling(events, kind, native, pos=1):
    out = []
    env = StreamExecutionEnvironment(4).set_output(out.append)
    env.config.native = native
    ks = env.from_collection(events).map(lambda e: Tuple3(e[0], e[1], e[2])).key_by(0)
    getattr(ks, kind)(pos).print()
    env.execute("rolling")
    return out


roll_st = st.lists(st.tuples(st.sampled_from(["h1", "h2", "h3", "www.163.com"]),
                             st.integers(-50, 1000), st.sampled_from(["cpu0", "cpu1"])),
                   min_size=1, max_size=60)


@settings(max_examples=40, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(events=roll_st, kind=st.sampled_from(["max", "min", "sum"]))
def test_native_rolling_equals_host(events, kind):
    assert _run_rolling(events, kind, "auto") == _run_rolling(events, kind, "off")


def test_native_rolling_floats_and_selection():
    from mxstream.api import planner
    from mxstream.runtime.executor import Executor
    from mxstream.runtime.native_ops import NativeRollingOp

    ev = [("a", 1.5, "x"), ("b", 0.25, "y"), ("a", 3.75, "z"), ("a", -2.0, "w")]
    assert _run_rolling(ev, "max", "auto") == _run_rolling(ev, "max", "off")
    env = StreamExecutionEnvironment(4)
    env.from_collection([("a", 1, "c")]).map(lambda e: Tuple3(*e)).key_by(0).max(1).print()
    sinks = planner.plan(env, list(env._sinks))
    ops = [n.factory() for n in Executor._topo(sinks) if n.kind == "op"]
    assert any(isinstance(o, NativeRollingOp) for o in ops)


# ---- session windows: NativeSessionOp vs the host merging WindowOperator ----------------------
def _run_sessions(events, gap, bound, lateness, native):
    from mxstream.api.windowing import EventTimeSessionWindows

    out = []
    env = StreamExecutionEnvironment(4, clock=ManualClock(0)).set_output(out.append)
    env.config.native = native
    env.set_stream_time_characteristic(TimeCharacteristic.EventTime)
    timed = [(i + 1, e) for i, e in enumerate(events)]
    (env.from_timed_collection(timed)
     .assign_timestamps_and_watermarks(
         BoundedOutOfOrdernessTimestampExtractor(Time.milliseconds(bound), extractor=lambda e: e[2]))
     .map(lambda e: Tuple2(e[0], e[1]))
     .key_by(0)
     .window(EventTimeSessionWindows.with_gap(Time.milliseconds(gap)))
     .allowed_lateness(Time.milliseconds(lateness))
     .reduce(lambda a, b: Tuple2(a.f0, a.f1 + b.f1))
     .print())
    env.execute("sessions")
    return out


@settings(max_examples=50, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(events=events_st, gap=st.sampled_from([100, 1500, 6000]),
       bound=st.sampled_from([0, 500, 3000]), lateness=st.sampled_from([0, 2000]))
def test_native_sessions_equal_host(events, gap, bound, lateness):
    a = _run_sessions(events, gap, bound, lateness, "off")
    b = _run_sessions(events, gap, bound, lateness, "auto")
    assert Counter(a) == Counter(b)


# ---- process-window median: NativeMedianOp vs the host WindowOperator ------------------------
def _run_median(events, size, slide, bound, lateness, native):
    from mxstream.models.chapters import MedianUsage

    out = []
    env = StreamExecutionEnvironment(4, clock=ManualClock(0)).set_output(out.append)
    env.config.native = native
    env.set_stream_time_characteristic(TimeCharacteristic.EventTime)
    timed = [(i + 1, e) for i, e in enumerate(events)]
    (env.from_timed_collection(timed)
     .assign_timestamps_and_watermarks(
         BoundedOutOfOrdernessTimestampExtractor(Time.milliseconds(bound), extractor=lambda e: e[2]))
     .map(lambda e: Tuple2(e[0], float(e[1]) / 4))
     .key_by(0)
     .time_window(Time.milliseconds(size), Time.milliseconds(slide))
     .allowed_lateness(Time.milliseconds(lateness))
     .process(MedianUsage())
     .print())
    env.execute("median")
    return out


@settings(max_examples=40, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(events=events_st, size_k=st.integers(1, 4), slide_div=st.sampled_from([1, 2]),
       bound=st.sampled_from([0, 1000]), lateness=st.sampled_from([0, 3000]))
def test_native_median_equals_host(events, size_k, slide_div, bound, lateness):
    size = size_k * 2000
    a = _run_median(events, size, size // slide_div, bound, lateness, "off")
    b = _run_median(events, size, size // slide_div, bound, lateness, "auto")
    assert Counter(a) == Counter(b)


def _run_count(events, n, native, agg):
    from mxstream.api.functions import AggregateFunction

    class Avg(AggregateFunction):
        def create_accumulator(self):
            return Tuple2(0, 0)

        def add(self, v, acc):
            return Tuple2(acc.f0 + 1, acc.f1 + v.f1)

        def get_result(self, acc):
            return acc.f1 / acc.f0

        def merge(self, a, b):
            return Tuple2(a.f0 + b.f0, a.f1 + b.f1)

    out = []
    env = StreamExecutionEnvironment(4, clock=ManualClock(0)).set_output(out.append)
    env.config.native = native
    ws = (env.from_collection(events).map(lambda e: Tuple2(e[0], e[1])).key_by(0)
          .count_window(n))
    if agg == "reduce":
        s = ws.reduce(lambda a, b: Tuple2(a.f0, a.f1 + b.f1))
    elif agg == "avg":
        s = ws.aggregate(Avg())
    else:
        s = getattr(ws, agg)(1)
    s.print()
    env.execute("count")
    return out


@settings(max_examples=50, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(events=st.lists(st.tuples(st.sampled_from(["a", "b", "c", "10.8.22.1"]),
                                 st.integers(0, 1000)), min_size=1, max_size=60),
       n=st.integers(1, 6), agg=st.sampled_from(["reduce", "max", "min", "sum", "avg"]))
def test_native_count_window_equals_host(events, n, agg):
    """keyBy(0).countWindow(n) (GlobalWindows + PurgingTrigger(CountTrigger(n))): the native
    segmented-scan path emits exactly the host WindowOperator's lines."""
    a = _run_count(events, n, "off", agg)
    b = _run_count(events, n, "auto", agg)
    assert Counter(a) == Counter(b)


def test_native_count_window_is_selected():
    from mxstream.api import planner
    from mxstream.runtime.native_ops import NativeCountWindowOp

    env = StreamExecutionEnvironment(4)
    (env.from_collection([("a", 1)]).key_by(0).count_window(3)
     .reduce(lambda a, b: Tuple2(a.f0, a.f1 + b.f1)).print())
    sinks = planner.plan(env, list(env._sinks))
    from mxstream.runtime.executor import Executor

    ops = [n.factory() for n in Executor._topo(sinks) if n.kind == "op"]
    assert any(isinstance(o, NativeCountWindowOp) for o in ops)
