"""DataStream API over metric vectors: aggregate(VectorAvgAggregate / VectorSumAggregate) runs on
the native vector-window operator (C++ twin here, MFMA kernel on a GPU) and must agree with the
exact host WindowOperator (f32 vs f64 arithmetic: compared with a tolerance)."""
import ast
from collections import defaultdict

import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from mxstream.api.aggregations import VectorAvgAggregate, VectorSumAggregate
from mxstream.api.environment import StreamExecutionEnvironment
from mxstream.api.time import Time, TimeCharacteristic
from mxstream.api.tuples import Tuple2
from mxstream.api.watermarks import BoundedOutOfOrdernessTimestampExtractor
from mxstream.runtime.executor import ManualClock


def _run(events, size, slide, bound, native, agg_cls, device="cpu"):
    out = []
    env = StreamExecutionEnvironment(4, clock=ManualClock(0)).set_output(out.append)
    env.config.native = native
    env.config.device = device
    env.set_stream_time_characteristic(TimeCharacteristic.EventTime)
    timed = [(i + 1, e) for i, e in enumerate(events)]
    (env.from_timed_collection(timed)
        .assign_timestamps_and_watermarks(
            BoundedOutOfOrdernessTimestampExtractor(Time.milliseconds(bound), extractor=lambda e: e[2]))
        .map(lambda e: Tuple2(e[0], list(e[1])))
        .key_by(0)
        .time_window(Time.milliseconds(size), Time.milliseconds(slide))
        .aggregate(agg_cls(1))
        .print())
    env.execute("vector-diff")
    return out


def _parse(lines):
    got = defaultdict(list)
    for ln in lines:
        prefix, body = ln.split("> ", 1)
        got[prefix].append(ast.literal_eval(body))
    return {k: sorted(v) for k, v in got.items()}


def _same(a, b):
    pa, pb = _parse(a), _parse(b)
    assert pa.keys() == pb.keys()
    for k in pa:
        assert len(pa[k]) == len(pb[k])
        for x, y in zip(pa[k], pb[k]):
            assert x == pytest.approx(y, rel=1e-6, abs=1e-4)


vec = st.lists(st.integers(0, 100), min_size=3, max_size=3)
events_st = st.lists(st.tuples(st.sampled_from(["10.8.22.1", "10.8.22.2", "h3"]), vec,
                               st.integers(0, 20_000)), min_size=1, max_size=30)


@settings(max_examples=40, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(events=events_st, size_k=st.integers(1, 5), slide_div=st.sampled_from([1, 2]),
       bound=st.sampled_from([0, 2000]), avg=st.booleans())
def test_vector_native_equals_host(events, size_k, slide_div, bound, avg):
    size = size_k * 1500
    cls = VectorAvgAggregate if avg else VectorSumAggregate
    a = _run(events, size, size // slide_div, bound, "off", cls)
    b = _run(events, size, size // slide_div, bound, "auto", cls)
    _same(a, b)


def test_vector_native_path_is_selected():
    from mxstream.api import planner
    from mxstream.runtime.executor import Executor
    from mxstream.runtime.native_ops import NativeVectorWindowOp

    env = StreamExecutionEnvironment(4)
    (env.from_collection([("a", [1.0, 2.0])]).key_by(0).time_window(Time.seconds(1))
     .aggregate(VectorAvgAggregate(1)).print())
    sinks = planner.plan(env, list(env._sinks))
    ops = [n.factory() for n in Executor._topo(sinks) if n.kind == "op"]
    assert any(isinstance(o, NativeVectorWindowOp) for o in ops)


@pytest.mark.gpu
def test_vector_api_gpu_equals_host(gpu_device):
    events = [("h%d" % (i % 7), [i % 13, (i * 7) % 100, 3], 100 * i) for i in range(400)]
    a = _run(events, 3000, 1000, 500, "off", VectorAvgAggregate)
    b = _run(events, 3000, 1000, 500, "auto", VectorAvgAggregate, device="cuda")
    _same(a, b)


def _run_ranks(events, world, device="cpu"):
    """The vector job on `world` loopback ranks: keyed records and their vectors move inside
    the operator's all-to-all; the executor's pickled exchange carries no record."""
    from mxstream.parallel.comm import run_loopback
    from mxstream.runtime import executor as X

    seen = {"recs": 0, "device": []}
    orig = X.Executor._exchange

    def spy(self, n, items):
        out = orig(self, n, items)
        if n.key_fn_in is not None:
            dx = getattr(self.ops.get(n.id), "device_exchange", False)
            # records that stay on their rank for the operator's own exchange are not pickled
            if not dx:
                seen["recs"] += sum(1 for it in out if isinstance(it, X.Rec))
            seen["device"].append(dx)
        return out

    def body(comm):
        out = []
        env = StreamExecutionEnvironment(4, clock=ManualClock(0)).set_output(out.append)
        env.config.native = "auto"
        env.config.device = device
        env._comm = comm
        env.set_stream_time_characteristic(TimeCharacteristic.EventTime)
        (env.from_collection(events, batch_size=16)
            .assign_timestamps_and_watermarks(
                BoundedOutOfOrdernessTimestampExtractor(Time.milliseconds(500),
                                                        extractor=lambda e: e[2]))
            .map(lambda e: Tuple2(e[0], list(e[1])))
            .key_by(0)
            .time_window(Time.milliseconds(3000), Time.milliseconds(1000))
            .aggregate(VectorAvgAggregate(1))
            .print())
        env.execute("vector-ranks")
        return out

    X.Executor._exchange = spy
    try:
        kw = {"device": __import__("torch").device("cuda", 0)} if device == "cuda" else {}
        res = run_loopback(world, body, **kw)
    finally:
        X.Executor._exchange = orig
    return [l for out in res for l in out], seen


def _vec_events(n=320):
    return [("h%d" % (i % 7), [i % 13, (i * 7) % 100, 3], 100 * i) for i in range(n)]


@pytest.mark.parametrize("world", [2, 4])
def test_vector_window_device_exchange_ranks(world):
    events = _vec_events()
    ref = _run(events, 3000, 1000, 500, "auto", VectorAvgAggregate)
    got, seen = _run_ranks(events, world)
    assert seen["recs"] == 0 and seen["device"] and all(seen["device"])
    _same(ref, got)


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 4])
def test_gpu_vector_window_device_exchange_ranks(world, gpu_device):
    events = _vec_events()
    ref = _run(events, 3000, 1000, 500, "off", VectorAvgAggregate)
    got, seen = _run_ranks(events, world, device="cuda")
    assert seen["recs"] == 0 and all(seen["device"])
    _same(ref, got)
