"""Flow control between ranks (SURVEY.md F-net): the multi-rank executor runs step-synchronously
-- every step opens with one collective over the ranks (runtime/executor.py:_step_begin) and
every keyed edge exchanges inside the step -- so a fast rank can never run more than one
micro-batch ahead of a slow one. The in-flight data between two ranks is bounded by one batch per
edge (Flink bounds it by credit-based network buffers; here the collectives are the credits).

Two gloo processes run a keyed job; rank 1's map stalls on every record of its first batches.
Each rank logs (CLOCK_MONOTONIC, step-local record count); at every moment rank 0's processed
count may exceed rank 1's by at most one batch (plus the batch in progress)."""
import os
import socket
import time

import torch.multiprocessing as mp

BATCH = 16
N = 16 * BATCH * 2  # 16 batches per rank


def _job(rank: int, log: list):
    from mxstream.api.environment import StreamExecutionEnvironment
    from mxstream.api.tuples import Tuple2

    def stamp(x):
        if rank == 1 and len(log) < 6 * BATCH:
            time.sleep(0.004)  # the slow rank: ~64 ms per batch for its first 6 batches
        log.append(time.monotonic())
        return Tuple2(x % 7, 1)

    out = []
    env = StreamExecutionEnvironment(2).set_output(out.append)
    env.config.native = "off"
    (env.from_collection(list(range(N)), batch_size=BATCH)
     .map(stamp).key_by(0).sum(1).print())
    env.execute("flow-control")
    return out


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    log: list = []
    try:
        out = _job(rank, log)
        q.put((rank, log, len(out), None))
    except Exception as e:  # noqa: BLE001
        q.put((rank, log, 0, repr(e)))
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


def test_fast_rank_stays_within_one_batch_of_slow_rank():
    for k in ("RANK", "WORLD_SIZE"):
        os.environ.pop(k, None)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=300) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
    errs = [e for *_, e in res if e]
    assert not errs, errs
    logs = {r: log for r, log, _, _ in res}
    assert sum(n for _, _, n, _ in res) == N  # one rolling-sum line per record
    fast, slow = logs[0], logs[1]
    assert len(fast) >= 8 * BATCH and len(slow) >= 8 * BATCH
    # At each of the slow rank's record times, how many records had the fast rank processed?
    lead = []
    j = 0
    for i, t in enumerate(slow):
        while j < len(fast) and fast[j] <= t:
            j += 1
        lead.append(j - (i + 1))
    # Unbounded, the fast rank would finish all of its records while the slow rank sleeps
    # through its first batches (a lead of ~10 batches).
    assert max(lead) <= 2 * BATCH, max(lead)
    # ... and it is paced by the slow rank's stalls (6 batches x 64 ms) instead of racing ahead.
    assert fast[-1] - fast[0] >= 0.5 * 6 * BATCH * 0.004
