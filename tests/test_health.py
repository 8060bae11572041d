"""Failure detection (runtime/health.py) and tracing (utils/trace.py, csrc/trace.cpp)."""
import json
import os
import socket
import time

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from mxstream.api.environment import RestartStrategies, StreamExecutionEnvironment
from mxstream.api.time import Time
from mxstream.api.tuples import Tuple2
from mxstream.runtime.executor import JobExecutionException
from mxstream.runtime.health import PeerHeartbeat, RankFailure, StepTimeout, Watchdog
from mxstream.utils import trace


def test_watchdog_quiet_when_beating():
    with Watchdog(200, name="t", action="none") as wd:
        for i in range(10):
            time.sleep(0.02)
            wd.beat(i)
    assert not wd.expired
    wd.check()


def test_watchdog_fires_and_check_raises():
    seen = []
    wd = Watchdog(100, name="t", action="none", on_expire=seen.append).start()
    time.sleep(0.4)
    wd.stop()
    assert wd.expired and seen == [wd]
    with pytest.raises(StepTimeout):
        wd.check()


def _slow_job(timeout_ms, sleep_s, restart=False):
    out = []
    env = StreamExecutionEnvironment(2).set_output(out.append)
    env.config.step_timeout_ms = timeout_ms
    if restart:
        env.set_restart_strategy(RestartStrategies.fixed_delay_restart(1, 0))
    (env.from_collection([1, 2, 3])
        .map(lambda x: (time.sleep(sleep_s), x)[1])
        .print())
    env.execute("slow")
    return out


def test_executor_step_timeout_fails_job():
    with pytest.raises(JobExecutionException) as ei:
        _slow_job(150, 0.5)
    assert "StepTimeout" in str(ei.value)
    assert isinstance(ei.value.__cause__, StepTimeout)


def test_executor_fast_job_unaffected():
    out = _slow_job(2000, 0.0)
    assert sorted(x.split("> ")[1] for x in out) == ["1", "2", "3"]


def test_peer_heartbeat_detects_stalled_rank(tmp_path):
    store_path = str(tmp_path / "store")
    a = PeerHeartbeat(dist.FileStore(store_path, 2), 0, 2, interval_ms=30, timeout_ms=300).start()
    b = PeerHeartbeat(dist.FileStore(store_path, 2), 1, 2, interval_ms=30, timeout_ms=300).start()
    try:
        time.sleep(0.3)
        a.check()
        b.check()
        b.pause()  # rank 1 hangs: stops publishing
        deadline = time.time() + 3.0
        while time.time() < deadline and not a.dead:
            time.sleep(0.05)
        with pytest.raises(RankFailure):
            a.check()
        assert a.dead == {1}
    finally:
        a.stop()
        b.stop()


def _hb_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mxstream.runtime.health import default_store

    hb = PeerHeartbeat(default_store(), rank, world, interval_ms=30, timeout_ms=400).start()
    time.sleep(0.3)
    ok_before = not hb.dead
    if rank == 1:
        hb.pause()
        time.sleep(1.5)
        q.put((rank, ok_before, sorted(hb.dead)))
    else:
        t0 = time.time()
        while time.time() < t0 + 3.0 and not hb.dead:
            time.sleep(0.05)
        q.put((rank, ok_before, sorted(hb.dead)))
        time.sleep(max(0.0, t0 + 1.8 - time.time()))  # keep beating while rank 1 checks
    hb.stop()
    dist.barrier()
    dist.destroy_process_group()


def test_peer_heartbeat_multiprocess_gloo():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_hb_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((r, (ok, dead)) for r, ok, dead in (q.get(timeout=60) for _ in procs))
    for p in procs:
        p.join(timeout=30)
    assert res[0] == (True, [1])      # rank 0 saw rank 1 stop
    assert res[1] == (True, [])       # rank 1 itself kept seeing rank 0


def test_trace_chrome_json_from_job(tmp_path):
    path = tmp_path / "trace.json"
    trace.clear()
    env = StreamExecutionEnvironment(2).set_output(lambda s: None)
    env.config.trace_path = str(path)
    (env.from_collection([("a", 1), ("b", 2), ("a", 3)])
        .key_by(0).time_window(Time.seconds(1))
        .reduce(lambda x, y: Tuple2(x.f0, x.f1 + y.f1)).print())
    env.execute("traced")
    trace.enable(False)
    doc = json.loads(path.read_text())
    names = {e["name"] for e in doc["traceEvents"] if e.get("ph") == "X"}
    assert any("Window" in n or "Map" in n or "Sink" in n or "Print" in n for n in names), names
    for e in doc["traceEvents"]:
        if e.get("ph") == "X":
            assert e["dur"] >= 0 and e["ts"] > 0


def test_trace_roctx_ranges_are_safe_without_profiler():
    trace.enable(False, roctx=True)
    try:
        with trace.span("partition"):
            with trace.span("inner"):
                trace.mark("m")
    finally:
        trace.enable(False, roctx=False)
