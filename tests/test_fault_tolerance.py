"""Job-level checkpoints, restart strategies and fault injection.

A job with a replayable source, checkpointing and ``fixedDelayRestart`` is killed mid-stream by
the fault injector (``ExecutionConfig.fault_injection`` / ``MXS_FAULT``); it must restart from the
latest completed checkpoint and end with the same results as an undisturbed run (the print/collect
sink is at-least-once, as in Flink: records emitted after the checkpoint may appear twice).
"""
from collections import Counter

import pytest

from mxstream.api.environment import FsStateBackend, RestartStrategies, StreamExecutionEnvironment
from mxstream.api.time import Time, TimeCharacteristic
from mxstream.api.tuples import Tuple2
from mxstream.api.watermarks import BoundedOutOfOrdernessTimestampExtractor
from mxstream.runtime.checkpoint import read_metadata
from mxstream.runtime.executor import InjectedFault, ManualClock


def _events(n=240):
    return [(i * 50 + 10, (f"k{i % 7}", i % 11, i * 50)) for i in range(n)]


def _job(tmp_path, *, native="off", fault=None, restart=True, ckpt=True):
    out = []
    env = StreamExecutionEnvironment(4, clock=ManualClock(0))
    env.config.native = native
    env.config.fault_injection = fault
    env.set_stream_time_characteristic(TimeCharacteristic.EventTime)
    if ckpt:
        env.enable_checkpointing(500)
        env.set_state_backend(FsStateBackend(str(tmp_path)))
    if restart:
        env.set_restart_strategy(RestartStrategies.fixed_delay_restart(2, 0))
    (env.from_timed_collection(_events())
     .assign_timestamps_and_watermarks(
         BoundedOutOfOrdernessTimestampExtractor(Time.milliseconds(100), extractor=lambda e: e[2]))
     .map(lambda e: Tuple2(e[0], e[1]))
     .key_by(0)
     .time_window(Time.milliseconds(1000))
     .reduce(lambda a, b: Tuple2(a.f0, a.f1 + b.f1))
     .collect(out))
    res = env.execute("ft")
    return out, res


@pytest.mark.parametrize("native", ["off", "auto"])
def test_restart_from_checkpoint_matches_clean_run(tmp_path, native):
    clean, _ = _job(tmp_path / "clean", native=native, restart=False, ckpt=False)
    got, res = _job(tmp_path / "ft", native=native, fault="Window:150")
    assert res.metrics["numRestarts"] == 1
    assert res.metrics["restoredCheckpointId"] >= 1
    assert set(map(str, got)) == set(map(str, clean))
    # At-least-once sink: every clean result appears, replays only add duplicates.
    c_clean, c_got = Counter(map(str, clean)), Counter(map(str, got))
    assert all(c_got[k] >= v for k, v in c_clean.items())


def test_no_restart_strategy_fails_job(tmp_path):
    with pytest.raises(InjectedFault):
        _job(tmp_path, fault="Window:50", restart=False)


def test_restart_without_checkpoints_starts_over(tmp_path):
    clean, _ = _job(tmp_path / "c", restart=False, ckpt=False)
    got, res = _job(tmp_path / "r", fault="Window:100", ckpt=False)
    assert res.metrics["numRestarts"] == 1
    assert set(map(str, got)) == set(map(str, clean))


def test_checkpoint_directory_layout(tmp_path):
    _out, res = _job(tmp_path)
    assert res.metrics["numberOfCompletedCheckpoints"] >= 3
    last = res.metrics["lastCheckpointPath"]
    meta = read_metadata(last)
    job_dir = tmp_path / meta["job_id"]
    assert (job_dir / "shared").is_dir() and (job_dir / "taskowned").is_dir()
    chks = sorted(p.name for p in job_dir.iterdir() if p.name.startswith("chk-"))
    assert len(chks) == 1  # state.checkpoints.num-retained = 1


def test_execute_from_savepoint(tmp_path):
    # Checkpoint mid-stream, then start a new job from that directory: the remaining input yields
    # the remaining windows (the first run's final windows are the union's superset).
    full, res = _job(tmp_path / "a")
    path = res.metrics["lastCheckpointPath"]
    out = []
    env = StreamExecutionEnvironment(4, clock=ManualClock(0))
    env.set_stream_time_characteristic(TimeCharacteristic.EventTime)
    (env.from_timed_collection(_events())
     .assign_timestamps_and_watermarks(
         BoundedOutOfOrdernessTimestampExtractor(Time.milliseconds(100), extractor=lambda e: e[2]))
     .map(lambda e: Tuple2(e[0], e[1]))
     .key_by(0)
     .time_window(Time.milliseconds(1000))
     .reduce(lambda a, b: Tuple2(a.f0, a.f1 + b.f1))
     .collect(out))
    env.config.native = "off"
    env.execute_from_savepoint(path)
    assert out and set(map(str, out)) <= set(map(str, full))


# ---- multi-rank: one rank fails, every rank restarts from the same checkpoint ------------------
def _mr_worker(rank, world, port, root, fault_rank, q):
    import os

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    try:
        out = []
        env = StreamExecutionEnvironment(4, clock=ManualClock(0))
        env.config.native = "off"
        env.config.fault_injection = "Window:60" if rank == fault_rank else None
        env.set_stream_time_characteristic(TimeCharacteristic.EventTime)
        if root is not None:
            env.enable_checkpointing(500)
            env.set_state_backend(FsStateBackend(root))
            env.set_restart_strategy(RestartStrategies.fixed_delay_restart(2, 0))
        (env.from_timed_collection(_events())
         .assign_timestamps_and_watermarks(
             BoundedOutOfOrdernessTimestampExtractor(Time.milliseconds(100), extractor=lambda e: e[2]))
         .map(lambda e: Tuple2(e[0], e[1]))
         .key_by(0)
         .time_window(Time.milliseconds(1000))
         .reduce(lambda a, b: Tuple2(a.f0, a.f1 + b.f1))
         .collect(out))
        res = env.execute("ft-multirank")
        q.put((rank, [str(x) for x in out], dict(res.metrics), None))
    except Exception as e:  # noqa: BLE001
        q.put((rank, [], {}, repr(e)))
    import torch.distributed as dist

    if dist.is_initialized():
        dist.destroy_process_group()


def _run_ranks(world, root, fault_rank):
    import socket

    import torch.multiprocessing as mp

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_mr_worker, args=(r, world, port, root, fault_rank, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    errs = [e for *_, e in res if e]
    assert not errs, errs
    return res


def test_multirank_failure_restarts_every_rank_from_checkpoint(tmp_path):
    import os

    for k in ("RANK", "WORLD_SIZE"):
        os.environ.pop(k, None)
    clean = _run_ranks(2, None, None)
    got = _run_ranks(2, str(tmp_path), 1)  # rank 1's window operator fails mid-stream
    for _, _, m, _ in got:
        assert m["numRestarts"] == 1  # the healthy rank restarted too
        assert m["restoredCheckpointId"] >= 1
    c_clean = Counter(x for _, out, _, _ in clean for x in out)
    c_got = Counter(x for _, out, _, _ in got for x in out)
    assert len(c_clean) > 10 and set(c_got) == set(c_clean)
    assert all(c_got[k] >= v for k, v in c_clean.items())  # at-least-once sink
    meta = read_metadata(got[0][2]["lastCheckpointPath"])
    assert meta["world"] == 2 and len(meta["ranks"]) == 2


# ---- multi-rank: a failure in the end-of-input firing fails every rank -------------------------
def _eoi_worker(rank, world, port, fault, q):
    import os

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    try:
        out = []
        env = StreamExecutionEnvironment(4, clock=ManualClock(0))
        env.config.native = "off"
        env.config.fault_injection = fault if rank == 1 else None
        env.set_stream_time_characteristic(TimeCharacteristic.EventTime)
        # One window per key that only the end-of-input MAX watermark fires: the map after the
        # window first receives records in the final firing, where the fault is injected.
        (env.from_timed_collection(_events(40))
         .assign_timestamps_and_watermarks(
             BoundedOutOfOrdernessTimestampExtractor(Time.milliseconds(100), extractor=lambda e: e[2]))
         .map(lambda e: Tuple2(e[0], e[1]))
         .key_by(0)
         .time_window(Time.milliseconds(10_000_000))
         .reduce(lambda a, b: Tuple2(a.f0, a.f1 + b.f1))
         .map(lambda t: t).name("EoiMap")
         .collect(out))
        env.execute("ft-eoi")
        q.put((rank, "ok"))
    except Exception as e:  # noqa: BLE001
        q.put((rank, type(e).__name__ + ": " + str(e)))
    import torch.distributed as dist

    if dist.is_initialized():
        dist.destroy_process_group()


def test_multirank_failure_in_end_of_input_firing_fails_every_rank():
    import os
    import socket

    import torch.multiprocessing as mp

    for k in ("RANK", "WORLD_SIZE"):
        os.environ.pop(k, None)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_eoi_worker, args=(r, 2, port, "EoiMap:1", q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
    # Neither rank may report success (the failure was swallowed before) or hang.
    assert all(r != "ok" for _, r in res), res
    assert any("injected fault" in r for _, r in res), res


# ---- rescale: a checkpoint written by 2 ranks restores on 4 (key groups re-split) ----------
def _rescale_job(env, out):
    env.set_stream_time_characteristic(TimeCharacteristic.EventTime)
    (env.from_collection([(f"k{i % 13}", i % 11, i * 50) for i in range(600)], batch_size=20)
     .assign_timestamps_and_watermarks(
         BoundedOutOfOrdernessTimestampExtractor(Time.milliseconds(100), extractor=lambda e: e[2]))
     .map(lambda e: Tuple2(e[0], e[1]))
     .key_by(0)
     .time_window(Time.milliseconds(1000))
     .reduce(lambda a, b: Tuple2(a.f0, a.f1 + b.f1))
     .collect(out))


@pytest.mark.parametrize("old_world,new_world", [(2, 4), (4, 2), (2, 1)])
def test_host_checkpoint_restores_at_another_world_size(tmp_path, old_world, new_world):
    """Host (Python) operators checkpointed by `old_world` loopback ranks fail mid-stream; the
    job restarts from that checkpoint on `new_world` ranks. Keyed window state and timers are
    re-split by key group, the collection source's per-rank positions become the new ranks'
    remaining lines, and clean output is reproduced (at-least-once sink). The state files are
    typed JSON/npz: restoring reads no pickle."""
    import pickle

    from mxstream.parallel.comm import run_loopback

    def env_for(comm, out):
        # wall clock: a checkpoint after (nearly) every pass with a 1 ms interval
        env = StreamExecutionEnvironment(4)
        env.config.native = "off"
        env._comm = comm
        _rescale_job(env, out)
        return env

    def clean(comm):
        out = []
        env_for(comm, out).execute("rescale")
        return out

    ref = [str(x) for o in run_loopback(old_world, clean) for x in o]

    def first(comm):
        out = []
        env = env_for(comm, out)
        env.enable_checkpointing(1)
        env.set_state_backend(FsStateBackend(str(tmp_path)))
        env.config.fault_injection = "Window:150" if comm.rank == 0 else None
        try:
            env.execute("rescale")
        except Exception as e:  # noqa: BLE001 -- the injected fault ends the first run
            return out, repr(e)
        return out, None

    res = run_loopback(old_world, first)
    assert any(e for _, e in res)
    before = [str(x) for o, _ in res for x in o]
    ckpts = sorted(tmp_path.glob("*/chk-*"), key=lambda p: int(p.name[4:]))
    assert ckpts
    path = ckpts[-1]
    meta = read_metadata(path)
    assert meta["state_encoding"] == "mxs-typed-v1" and meta["world"] == old_world
    assert not list(path.glob("*.state")) and list(path.glob("*.state.json"))

    orig_load = pickle.load
    pickle.load = lambda *a, **k: (_ for _ in ()).throw(AssertionError("pickle.load in restore"))
    try:
        def second(comm):
            out = []
            env_for(comm, out).execute_from_savepoint(str(path), "rescale")
            return out

        after = [str(x) for o in run_loopback(new_world, second) for x in o]
    finally:
        pickle.load = orig_load
    c_ref, c_got = Counter(ref), Counter(before + after)
    # the second run resumed mid-stream (fewer results than a full run), and every window that
    # spans the checkpoint came out whole: the restored state was re-split, not lost
    assert 0 < len(after) < len(ref)
    assert len(c_ref) > 20 and set(c_got) == set(c_ref)
    assert all(c_got[k] >= v for k, v in c_ref.items())


def _drain_source(src, k):
    """Poll up to k items (k=None: all) from a source; returns the values."""
    got = []
    while k is None or len(got) < k:
        items, done = src.poll(0)
        got.extend(r.value for r in items)
        if done:
            break
    return got


@pytest.mark.parametrize("kind", ["collection", "sequence"])
def test_source_rescale_survives_later_checkpoints(kind):
    """A rescale restore's re-split is kept in later snapshots: world 2 -> 3 (rescale) ->
    checkpoint -> restore at 3 (same size) -> checkpoint -> restore at 2 (rescale again). Every
    item is emitted exactly once over the four runs (no replays folded twice into state)."""
    from mxstream.runtime.checkpoint import rescale_host_state
    from mxstream.runtime.sources import CollectionSource, SequenceSource

    n = 97

    def make():
        return (CollectionSource(list(range(n)), batch_size=3) if kind == "collection"
                else SequenceSource(0, n - 1, batch_size=3))

    def run(world, snaps, take):
        out, new = [], []
        for r in range(world):
            s = make()
            s.open(r, world, None)
            if snaps is not None:
                old_world = len(snaps)
                snap = (snaps[r] if old_world == world
                        else rescale_host_state(snaps, r, world, (0, 127), 128))
                s.restore(snap)
            out += _drain_source(s, take[r] if isinstance(take, list) else take)
            new.append(s.snapshot())
        return out, new

    emitted, snaps = run(2, None, [30, 2])  # uneven: the re-split leaves gaps to skip
    for world, take in ((3, 3), (3, 3), (2, None)):
        got, snaps = run(world, snaps, take)
        emitted += got
    assert sorted(emitted) == list(range(n)), Counter(emitted).most_common(3)


def test_rescale_uses_each_operators_own_parallelism(tmp_path):
    """A keyed operator with its own parallelism (set_parallelism(1): the executor routes every
    key to rank 0) is re-split at another world size with ITS key-group ranges, not the
    environment's: all of its state lands on rank 0, where its keys now arrive; an operator at
    the environment's parallelism is spread by the usual ranges."""
    from mxstream.runtime.checkpoint import (owned_key_groups, read_host_checkpoint,
                                             write_host_checkpoint, write_host_states)
    from mxstream.utils.hashing import key_group

    keys = [f"k{i}" for i in range(40)]
    ranks = []
    for r in range(2):  # the old job: world 2, both operators keyed
        mine = [k for k in keys if owned_key_groups(r, 2, 4, 128)[0] <= key_group(k, 128)
                <= owned_key_groups(r, 2, 4, 128)[1]]
        keyed = {}
        for k in mine:
            keyed.setdefault(key_group(k, 128), {}).setdefault("v", {})[k] = 1
        states = {"p1": {"keyed": keyed}, "p4": {"keyed": keyed}}
        files = write_host_states(tmp_path, states, r)
        ranks.append({"host_operators": files, "extra": {"clock": None}})
    write_host_checkpoint(tmp_path, job_id="j", checkpoint_id=1, states={}, extra={}, ranks=ranks)

    got = {}
    for r in range(4):
        _, st = read_host_checkpoint(tmp_path, r, 4, 4, 128, node_parallelism={"p1": 1})
        got[r] = {nid: sorted(k for t in s.get("keyed", {}).values() for k in t["v"])
                  for nid, s in st.items()}
    assert got[0]["p1"] == sorted(keys) and all(not got[r]["p1"] for r in (1, 2, 3))
    assert sorted(k for r in range(4) for k in got[r]["p4"]) == sorted(keys)
    assert sum(1 for r in range(4) if got[r]["p4"]) > 1
