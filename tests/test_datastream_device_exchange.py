"""DataStream jobs at G > 1 on the device exchange.

The reference's BandwidthMonitorWithEventTime (BandwidthMonitorWithEventTime.java:28-55) as a
multi-rank job: every rank parses its source partition with the device ingest, the ranks agree
on one dictionary id space per pass, and the keyed window operator exchanges its keys itself
(local-global partials through the rank communicator, key groups from the dictionary's Java
hashes) -- the executor's pickled record exchange is never used for that keyed edge. The union
of the ranks' printed lines equals the single-process run.

CPU: gloo processes (C++ twins) and LoopbackComm virtual ranks; GPU (marked): virtual ranks on
one MI355X through the same operators.
"""
import os
import socket
from collections import Counter

import pytest
import torch
import torch.multiprocessing as mp


def _lines(n=2400, channels=23):
    """chapter3 input over ~40 min of event time, in order; every 7th channel is starved."""
    out = []
    for i in range(n):
        c = (i * 7) % channels
        v = 40 + (i % 11) if c % 7 == 0 else 5_000_000 + (i * 7919) % 1_000_000
        t = i  # one line per second
        out.append(f"2019-08-28T{10 + t // 3600:02d}:{(t // 60) % 60:02d}:{t % 60:02d} "
                   f"www.ch{c}.com {v}")
    return out


def _job(lines, comm=None, device="cpu"):
    from mxstream.api.environment import StreamExecutionEnvironment
    from mxstream.models import chapters as C

    out = []
    env = StreamExecutionEnvironment(4).set_output(out.append)
    env.config.native = "auto"
    env.config.device = device
    env.config.text_ingest = "device"
    env._comm = comm
    C.build_bandwidth_event_time(env, env.from_collection(lines, batch_size=300))
    res = env.execute("bw-multirank")
    return out, res


def _spy_exchange(monkeypatch):
    """Count records that crossed the executor's pickled exchange."""
    from mxstream.runtime import executor as X

    seen = {"recs": 0}
    orig = X.Executor._exchange

    def spy(self, n, items):
        out = orig(self, n, items)
        if n.key_fn_in is not None:  # a keyed edge
            seen["recs"] += sum(1 for it in out if isinstance(it, X.Rec))
        return out

    monkeypatch.setattr(X.Executor, "_exchange", spy)
    return seen


@pytest.mark.parametrize("world", [2, 4])
def test_loopback_ranks_equal_single_process(world, monkeypatch):
    from mxstream.parallel.comm import run_loopback

    lines = _lines()
    ref, _ = _job(lines)
    assert len(ref) > 20
    seen = _spy_exchange(monkeypatch)
    res = run_loopback(world, lambda comm: _job(lines, comm))
    got = [l for out, _ in res for l in out]
    assert Counter(got) == Counter(ref)
    assert seen["recs"] == 0  # the keyed edge never pickled a record


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    try:
        out, _ = _job(_lines())
        q.put((rank, out, None))
    except Exception as e:  # noqa: BLE001
        import traceback

        q.put((rank, [], traceback.format_exc()))
    import torch.distributed as dist

    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()


def test_gloo_processes_equal_single_process():
    for k in ("RANK", "WORLD_SIZE"):
        os.environ.pop(k, None)
    ref, _ = _job(_lines())
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
    errs = [e for _, _, e in res if e]
    assert not errs, errs
    got = [l for _, lines, _ in res for l in lines]
    assert Counter(got) == Counter(ref)


def test_dictionary_growth_regrows_dense_state():
    """More distinct keys than the operator's initial dense key space (2^16): the state regrows
    (snapshot -> larger table -> restore) instead of failing."""
    lines = [f"2019-08-28T10:00:{i % 60:02d} k{i} {40 if i == 69_999 else 10 ** 9}"
             for i in range(70_000)]
    out, _ = _job(lines)  # would raise "table full" without the regrow
    # only the starved key alerts, in each of the 5-min / 5 s windows holding its element
    assert len(out) == 60 and all("(k69999," in l for l in out)


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 4, 8])
def test_gpu_loopback_ranks_equal_single_process(world, gpu_device, monkeypatch):
    from mxstream.parallel.comm import run_loopback

    lines = _lines(6000, 57)
    ref, _ = _job(lines, device="cuda")
    assert len(ref) > 20
    seen = _spy_exchange(monkeypatch)
    res = run_loopback(world, lambda comm: _job(lines, comm, device="cuda"),
                       device=torch.device("cuda", 0))
    got = [l for out, _ in res for l in out]
    assert Counter(got) == Counter(ref)
    assert seen["recs"] == 0
