"""All six reference jobs (models/chapters.py) at G > 1 on the device exchange.

Every rank parses its source partition with the device ingest (C++ twins on the CPU), the ranks
agree on one dictionary id space per pass, and every natively lowered keyed edge exchanges its
keys itself -- rolling max (ComputeCpuMax.java:26), processing-time tumbling aggregate / process /
reduce windows (ComputeCpuAvg.java:27-31, ComputeCpuMiddle.java:34-48,
BandwidthMonitor.java:32-37), the event-time sliding reduce (BandwidthMonitorWithEventTime.java:45-47)
and event-time session windows (chapter3/README.md:412-428). The executor's pickled record
exchange carries no record on any keyed edge (``seen["recs"] == 0``) and the union of the ranks'
printed lines equals the single-process run.

Processing time: the ranks stamp and fire on the step's agreed clock (the executor's MAX over
the ranks' clocks). Inputs are built so the comparison is exact at every G: rolling keys keep
all their lines on one source partition (a key's per-record maxima depend on its arrival order),
and averaged values are exactly representable (the order of the partial merges is free).
"""
from collections import Counter

import pytest
import torch

from mxstream.api.environment import StreamExecutionEnvironment
from mxstream.api.time import Time
from mxstream.api.tuples import Tuple2, Tuple3
from mxstream.api import windowing as W
from mxstream.models import chapters as C
from mxstream.runtime.executor import ManualClock


def _cpu_lines(n=480):
    """chapter1/2 input "ts host cpuN usage": host = f(i % 8) so a host's lines stay on one source
    partition at G = 2, 4 and 8 (CollectionSource deals lines rank::world)."""
    out = []
    for i in range(n):
        h = (i % 8) * 5 + (i // 8) % 5          # 40 hosts
        usage = ((i * 37) % 400) / 4.0          # exact doubles, some > 90
        out.append(f"{1563452000 + i} 10.8.{h}.{h % 3} cpu{i % 4} {usage}")
    return out


def _bw_lines(n=480, channels=11):
    out = []
    for i in range(n):
        c = (i * 7) % channels
        v = 40 + i % 13 if c % 5 == 0 else 9_000_000 + (i * 7919) % 1_000_000
        out.append(f"2019-08-28T10:{(i // 60) % 60:02d}:{i % 60:02d} www.ch{c}.com {v}")
    return out


def _session_job(env, text):
    from mxstream.api.time import TimeCharacteristic

    env.set_stream_time_characteristic(TimeCharacteristic.EventTime)
    s = (text.assign_timestamps_and_watermarks(C.EventTimeExtractor())
         .map(C.ParseTimedFlow())
         .key_by(1)
         .window(W.EventTimeSessionWindows.with_gap(Time.seconds(20)))
         .reduce(lambda a, b: Tuple3(a.f0, a.f1, a.f2 + b.f2))
         .map(lambda t: Tuple2(t.f1, t.f2)))
    s.print()
    return s


def _session_lines(n=400, channels=9):
    """Channels with bursts and 30 s pauses (several sessions per channel)."""
    out = []
    t = 0
    for i in range(n):
        t += 1 if i % 25 else 31
        c = (i * 5) % channels
        out.append(f"2019-08-28T10:{(t // 60) % 60:02d}:{t % 60:02d} www.s{c}.com {100 + i}")
    return out


# name -> (build, input lines, timed (processing-time) source?)
JOBS = {
    "Main": (C.build_cpu_alert, _cpu_lines, False),
    "ComputeCpuMax": (C.build_compute_cpu_max, _cpu_lines, False),
    "ComputeCpuAvg": (C.build_compute_cpu_avg, _cpu_lines, True),
    "ComputeCpuMiddle": (C.build_compute_cpu_middle, _cpu_lines, True),
    "BandwidthMonitor": (C.build_bandwidth_monitor, _bw_lines, True),
    "BandwidthMonitorWithEventTime": (C.build_bandwidth_event_time, _bw_lines, False),
    "Sessions": (_session_job, _session_lines, False),
}
KEYED = {"ComputeCpuMax", "ComputeCpuAvg", "ComputeCpuMiddle", "BandwidthMonitor",
         "BandwidthMonitorWithEventTime", "Sessions"}


def _run(name, comm=None, device="cpu", native="auto"):
    build, gen, timed = JOBS[name]
    lines = gen()
    out = []
    env = StreamExecutionEnvironment(4, clock=ManualClock(0)).set_output(out.append)
    env.config.native = native
    env.config.device = device
    env.config.text_ingest = "device"
    env._comm = comm
    if timed:
        # one line per 100 ms of processing time, the source open until 70 s: every line is in
        # the first 1-min window, which fires at 59 999 ms
        src = env.from_timed_collection([(100 * (i + 1), l) for i, l in enumerate(lines[:500])],
                                        end_time=70_000)
    else:
        src = env.from_collection(lines, batch_size=40)
    build(env, src)
    res = env.execute(name)
    return out, res, None


def _strip(lines):
    """chapter1 prints with round-robin prefixes (the rebalance start differs per rank)."""
    return [l.split("> ", 1)[1] if "> " in l else l for l in lines]


def _spy(monkeypatch):
    from mxstream.runtime import executor as X

    seen = {"recs": 0, "device": []}
    orig = X.Executor._exchange

    def spy(self, n, items):
        out = orig(self, n, items)
        if n.key_fn_in is not None:
            seen["recs"] += sum(1 for it in out if isinstance(it, X.Rec))
            seen["device"].append(getattr(self.ops.get(n.id), "device_exchange", False))
        return out

    monkeypatch.setattr(X.Executor, "_exchange", spy)
    return seen


def _check(name, ref, got, seen):
    if name == "Main":
        assert Counter(_strip(got)) == Counter(_strip(ref))
    else:
        assert Counter(got) == Counter(ref)
    if name in KEYED:
        assert seen["recs"] == 0, "a keyed edge pickled records"
        assert seen["device"] and all(seen["device"])


@pytest.mark.parametrize("name", list(JOBS))
@pytest.mark.parametrize("world", [2, 4])
def test_reference_job_loopback_ranks(name, world, monkeypatch):
    from mxstream.parallel.comm import run_loopback

    ref, _, _ = _run(name)
    assert len(ref) > 3, ref
    seen = _spy(monkeypatch)
    res = run_loopback(world, lambda comm: _run(name, comm))
    got = [l for out, _, _ in res for l in out]
    _check(name, ref, got, seen)


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(JOBS))
@pytest.mark.parametrize("world", [2, 4, 8])
def test_gpu_reference_job_loopback_ranks(name, world, gpu_device, monkeypatch):
    from mxstream.parallel.comm import run_loopback

    ref, _, _ = _run(name, device="cuda")
    assert len(ref) > 3
    seen = _spy(monkeypatch)
    res = run_loopback(world, lambda comm: _run(name, comm, device="cuda"),
                       device=torch.device("cuda", 0))
    got = [l for out, _, _ in res for l in out]
    _check(name, ref, got, seen)


def _object_spy(comm_cls, executor_cls):
    """Counts pickled (object) collectives per executor pass: returns the per-pass list of one
    rank (a pass = one Executor._push)."""
    import threading

    passes = {}
    orig_push = executor_cls._push

    def push(self, inbox, now):
        passes.setdefault(threading.get_ident(), []).append(0)
        return orig_push(self, inbox, now)

    def wrap(name):
        orig = getattr(comm_cls, name)

        def f(self, *a, **k):
            lst = passes.get(threading.get_ident())
            if lst:
                lst[-1] += 1
            return orig(self, *a, **k)

        return orig, f

    saved = {}
    for nm in ("all_gather_object", "broadcast_object"):
        saved[nm], f = wrap(nm)
        setattr(comm_cls, nm, f)
    executor_cls._push = push

    def undo():
        executor_cls._push = orig_push
        for nm, o in saved.items():
            setattr(comm_cls, nm, o)

    return passes, undo


def _steady_state_quiet(per_pass):
    """Object collectives only while the ranks still meet new dictionary strings (the first
    passes): the second half of the job's passes has none."""
    assert len(per_pass) >= 2, per_pass
    tail = per_pass[len(per_pass) // 2:]
    assert sum(tail) == 0, per_pass


@pytest.mark.parametrize("name", list(JOBS))
@pytest.mark.parametrize("world", [2, 4, 8])
def test_control_plane_has_no_object_collectives(name, world):
    """The executor's control plane at G > 1 (done flag, clock, checkpoint request, failure flag,
    watermark valve of device-exchange edges) is a packed int64 all-reduce: after the dictionary
    has settled, a pass makes no pickled all_gather_object / broadcast_object."""
    from mxstream.parallel.comm import LoopbackComm, run_loopback
    from mxstream.runtime import executor as X

    passes, undo = _object_spy(LoopbackComm, X.Executor)
    try:
        res = run_loopback(world, lambda comm: _run(name, comm))
    finally:
        undo()
    ref, _, _ = _run(name)
    got = [l for out, _, _ in res for l in out]
    _check(name, ref, got, {"recs": 0, "device": [True]})
    assert len(passes) == world
    for per_pass in passes.values():
        _steady_state_quiet(per_pass)


def _gloo_worker(rank, world, port, name, q, native="auto"):
    import os

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    try:
        from mxstream.runtime import executor as X

        seen = {"recs": 0, "device": []}
        orig = X.Executor._exchange

        def spy(self, n, items):
            out = orig(self, n, items)
            if n.key_fn_in is not None:
                seen["recs"] += sum(1 for it in out if isinstance(it, X.Rec))
                seen["device"].append(getattr(self.ops.get(n.id), "device_exchange", False))
            return out

        X.Executor._exchange = spy
        from mxstream.parallel.comm import TorchComm

        passes, _ = _object_spy(TorchComm, X.Executor)
        out, _, _ = _run(name, native=native)
        seen["passes"] = next(iter(passes.values()), [])
        q.put((rank, out, seen, None))
    except Exception:  # noqa: BLE001
        import traceback

        q.put((rank, [], None, traceback.format_exc()))
    import torch.distributed as dist

    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()


@pytest.mark.parametrize("name", ["ComputeCpuMax", "ComputeCpuAvg", "ComputeCpuMiddle", "Sessions"])
def test_reference_job_gloo_processes(name):
    """Two processes over gloo (TorchComm): the same device exchange as the loopback ranks."""
    import os
    import socket

    import torch.multiprocessing as mp

    for k in ("RANK", "WORLD_SIZE"):
        os.environ.pop(k, None)
    ref, _, _ = _run(name)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_gloo_worker, args=(r, 2, port, name, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
    errs = [e for *_, e in res if e]
    assert not errs, errs
    got = [l for _, lines, _, _ in res for l in lines]
    assert Counter(got) == Counter(ref)
    for _, _, seen, _ in res:
        assert seen["recs"] == 0 and seen["device"] and all(seen["device"])
        _steady_state_quiet(seen["passes"])


def _drift_lines(n=60000, channels=30000):
    """Timed flow lines over a channel dictionary far larger than the dense budget below; each
    channel is active for half a second, then idles (its windows stay live for the allowed
    lateness, so idle keys are moved to the host tier, not dropped)."""
    out = []
    for i in range(n):
        c = (i // 2) % channels
        t = i // 4
        out.append(f"2019-08-28T{10 + t // 3600:02d}:{(t // 60) % 60:02d}:{t % 60:02d} "
                   f"www.ch{c}.com {100 + i % 97}")
    return out


@pytest.mark.parametrize("world", [1, 2])
def test_dictionary_beyond_dense_budget_moves_to_hashed_tier(world, monkeypatch):
    """A channel dictionary that outgrows the dense id budget switches the window state to hashed
    keys with the host-DRAM tier: idle keys leave HBM, the output equals the all-dense run, at
    G = 1 and G = 2."""
    from mxstream.api.time import TimeCharacteristic
    from mxstream.parallel.comm import run_loopback
    from mxstream.runtime import native_ops as N

    lines = _drift_lines()

    def run(budget, comm=None):
        out = []
        env = StreamExecutionEnvironment(4, clock=ManualClock(0)).set_output(out.append)
        env.config.native = "auto"
        env.config.text_ingest = "device"
        env.config.window_dense_max_keys = budget
        env._comm = comm
        env.set_stream_time_characteristic(TimeCharacteristic.EventTime)
        (env.from_collection(lines, batch_size=500)
            .assign_timestamps_and_watermarks(C.EventTimeExtractor())
            .map(C.ParseTimedFlow())
            .key_by(1)
            .time_window(Time.minutes(1))
            .allowed_lateness(Time.minutes(10))
            .reduce(lambda a, b: Tuple3(a.f0, a.f1, a.f2 + b.f2))
            .map(lambda t: Tuple2(t.f1, t.f2))
            .print())
        env.execute("drift")
        return out

    ref = run(1 << 27)
    assert len(ref) > 1000
    switched = []
    orig = N.NativeWindowOp._ensure_capacity

    def spy(self):
        orig(self)
        if self._spill_state:
            switched.append(self)

    monkeypatch.setattr(N.NativeWindowOp, "_ensure_capacity", spy)
    if world == 1:
        got = run(4096)
    else:
        got = [l for out in run_loopback(world, lambda comm: run(4096, comm)) for l in out]
    ops = set(switched)
    assert ops and all(o.op.host_tier is not None and not o.op.dense_bits for o in ops)
    assert sum(o.op.metrics.extra.get("spilled_keys", 0) for o in ops) > 0  # keys left HBM
    assert Counter(got) == Counter(ref)


HOST_KEYED = ["ComputeCpuMiddle", "BandwidthMonitorWithEventTime"]


@pytest.mark.parametrize("name", HOST_KEYED)
@pytest.mark.parametrize("world", [2, 4, 8])
def test_host_keyed_edge_has_no_object_collectives(name, world):
    """Host (Python) operators on a keyed edge -- the planner does not lower them (native off):
    the executor's keyBy moves the records as typed, code-free words through the hand-written
    row exchange (parallel/exchange.exchange_records), each rank receiving only its own records;
    no pickled all_gather_object per pass once the job runs, and the output equals one process."""
    from mxstream.parallel.comm import LoopbackComm, run_loopback
    from mxstream.runtime import executor as X

    passes, undo = _object_spy(LoopbackComm, X.Executor)
    try:
        res = run_loopback(world, lambda comm: _run(name, comm, native="off"))
    finally:
        undo()
    ref, _, _ = _run(name, native="off")
    got = [l for out, _, _ in res for l in out]
    assert Counter(_strip(got)) == Counter(_strip(ref))
    assert all(r.metrics.get("objectExchangeFallbacks", 0) == 0 for _, r, _ in res)
    for per_pass in passes.values():
        assert sum(per_pass) == 0, per_pass


def test_host_keyed_edge_gloo_processes():
    """The same host keyed edge over two gloo processes (TorchComm)."""
    import os
    import socket

    import torch.multiprocessing as mp

    name = "ComputeCpuMiddle"
    for k in ("RANK", "WORLD_SIZE"):
        os.environ.pop(k, None)
    ref, _, _ = _run(name, native="off")
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_gloo_worker, args=(r, 2, port, name, q, "off")) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
    errs = [e for *_, e in res if e]
    assert not errs, errs
    got = [l for _, lines, _, _ in res for l in lines]
    assert Counter(_strip(got)) == Counter(_strip(ref))
    for _, _, seen, _ in res:
        assert sum(seen["passes"]) == 0, seen["passes"]
