"""DataStream jobs on several processes (torchrun-style WORLD_SIZE/RANK, gloo): keyed edges
exchange records between ranks, watermarks merge to the minimum over ranks, and the union of
every rank's printed lines equals the single-process run (SURVEY.md F-part-key, K18)."""
import os
import socket
from collections import Counter

import pytest
import torch.multiprocessing as mp


def _events(n=600):
    hosts = ["10.8.22.1", "10.8.22.2", "www.163.com", "h4", "h5", "h6", "h7"]
    return [(hosts[(i * 7) % len(hosts)], (i * 37) % 1000, 1_000 + i * 250) for i in range(n)]


def _job(native: str):
    from mxstream.api.environment import StreamExecutionEnvironment
    from mxstream.api.time import Time, TimeCharacteristic
    from mxstream.api.tuples import Tuple2, Tuple3
    from mxstream.api.watermarks import BoundedOutOfOrdernessTimestampExtractor

    out = []
    env = StreamExecutionEnvironment(4).set_output(out.append)
    env.config.native = native
    env.set_stream_time_characteristic(TimeCharacteristic.EventTime)
    src = env.from_collection(_events())
    (src.assign_timestamps_and_watermarks(
        BoundedOutOfOrdernessTimestampExtractor(Time.milliseconds(500), extractor=lambda e: e[2]))
     .map(lambda e: Tuple2(e[0], e[1]))
     .key_by(0)
     .time_window(Time.seconds(10))
     .reduce(lambda a, b: Tuple2(a.f0, a.f1 + b.f1))
     .print())
    (src.map(lambda e: Tuple3(e[0], e[1], e[2])).key_by(0).max(1).print())
    env.execute("multirank")
    return out


def _worker(rank, world, port, native, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    try:
        q.put((rank, _job(native), None))
    except Exception as e:  # noqa: BLE001
        q.put((rank, [], repr(e)))
    import torch.distributed as dist

    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _split(lines):
    windows = [l for l in lines if l.count(",") == 1]
    rolling = [l for l in lines if l.count(",") == 2]
    return windows, rolling


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("native", ["off", "auto"])
def test_datastream_job_invariant_to_ranks(world, native):
    for k in ("RANK", "WORLD_SIZE"):
        os.environ.pop(k, None)
    ref = _job(native)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, native, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    errs = [e for _, _, e in res if e]
    assert not errs, errs
    got = [l for _, lines, _ in res for l in lines]
    rw, rr = _split(ref)
    gw, gr = _split(got)
    # Event-time windows: identical lines (prefix = the key's subtask, sums order-free).
    assert Counter(gw) == Counter(rw) and len(rw) > 10
    # Rolling max: one line per record; the per-key arrival order interleaves the ranks'
    # partitions, so compare the count per key and the final maximum per key.
    def final(lines):
        best = {}
        for l in lines:
            key = l.split("(", 1)[1].split(",", 1)[0]
            v = int(l.split(",")[1])
            best[key] = max(best.get(key, -1), v)
        return best
    assert len(gr) == len(rr) and final(gr) == final(rr)
