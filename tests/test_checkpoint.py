"""Checkpoint / savepoint layout and restore: a run that checkpoints at step k
and a fresh operator restored from that checkpoint must produce identical results afterwards,
including at a different world size (key-group re-partitioning) and across devices."""
import os
import re
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from mxstream.ops import kernels as K
from mxstream.parallel.comm import TorchComm
from mxstream.runtime.checkpoint import (CheckpointCoordinator, CheckpointStorage, read_metadata,
                                         owned_key_groups)
from mxstream.runtime.rolling_operator import KeyedRollingOperator
from mxstream.runtime.session_operator import KeyedSessionOperator
from mxstream.runtime.window_operator import KeyedWindowOperator

STEPS, CUT, PER = 8, 4, 3000


def _batch(step, src=0, n=PER, device="cpu"):
    k = torch.empty(n, dtype=torch.int64, device=device)
    t = torch.empty_like(k)
    v = torch.empty_like(k)
    K.gen_events(k, t, v, seed=21, stream_id=src, idx0=step * n, nkeys=4000, ts_base=step * 2000,
                 ts_span=2000, disorder=600, val_lo=0, val_span=1000)
    return k, t, v


def _win(device="cpu", comm=None, **kw):
    args = dict(size=3000, slide=1000, lateness=1500, agg=K.AGG_SUM_I64, device=device,
                max_keys=8000, batch_capacity=PER * 2, ooo_bound=500, cap_log2=8)
    args.update(kw)
    return KeyedWindowOperator(comm=comm, **args)


def _fires(out):
    return sorted((r.window_start, int(k), int(a), int(c), r.refire)
                  for r in out for k, a, c in zip(r.keys, r.raw, r.counts))


@pytest.mark.parametrize("n", [1000, 2_500_000])  # 2.5M 8-byte rows: several 16 MB pieces
def test_kg_file_sorted_and_unsorted_rows_write_the_same_file(tmp_path, n):
    """The state file writer (csrc/kg_file.h) writes kg-sorted input as it is and permutes any
    other input (stable counting sort, threaded gather): both give the same file, and a key-group
    range read returns exactly that range's rows in input order."""
    from pathlib import Path

    from mxstream.runtime.checkpoint import (OperatorSnapshot, read_operator_rows,
                                             write_operator_file)

    rng = np.random.default_rng(3)
    kg = rng.integers(0, 128, n).astype(np.int32)
    cols = {"key": rng.integers(0, 1 << 40, n), "cnt": rng.integers(0, 99, n).astype(np.int32),
            "dirty": rng.integers(0, 2, n).astype(np.uint8)}
    order = np.argsort(kg, kind="stable")
    d1, d2 = Path(tmp_path / "u"), Path(tmp_path / "s")
    d1.mkdir()
    d2.mkdir()
    f1 = write_operator_file(d1, "w", 0, OperatorSnapshot(kg, cols), 128)
    f2 = write_operator_file(d2, "w", 0, OperatorSnapshot(kg[order], {c: v[order] for c, v in
                                                                        cols.items()}), 128)
    assert (d1 / f1).read_bytes() == (d2 / f2).read_bytes()
    got = read_operator_rows(d1, [f1], 40, 70)
    sel = order[(kg[order] >= 40) & (kg[order] <= 70)]
    for c, v in cols.items():
        assert np.array_equal(got[c], v[sel]), c


def test_window_checkpoint_restore_equals_uninterrupted(tmp_path):
    op = _win()
    storage = CheckpointStorage(tmp_path, job_id="a" * 32)
    coord = CheckpointCoordinator(storage, {"window": op})
    tail = []
    for s in range(STEPS):
        out = op.process(*_batch(s))
        if s == CUT:
            path = coord.trigger(s, sources={"next_step": s + 1})
        if s > CUT:
            tail += out
    tail += op.finish()
    # Flink layout
    assert path == tmp_path / ("a" * 32) / f"chk-1"
    assert (path / "_metadata").exists() and (tmp_path / ("a" * 32) / "shared").is_dir()
    assert (tmp_path / ("a" * 32) / "taskowned").is_dir()
    meta = read_metadata(path)
    assert meta["sources"][0]["next_step"] == CUT + 1 and meta["operators"]["window"]["rows"][0] > 0

    op2 = _win()
    CheckpointCoordinator(storage, {"window": op2}).restore()
    tail2 = []
    for s in range(CUT + 1, STEPS):
        tail2 += op2.process(*_batch(s))
    tail2 += op2.finish()
    assert _fires(tail) == _fires(tail2)


def _async_roundtrip(tmp_path, device):
    """Async checkpoint at CUT while the next steps run: pending until complete_pending(), then
    byte-identical rows to a synchronous checkpoint of the same step, and a restore from it
    continues exactly like the uninterrupted run."""
    op = _win(device=device)
    storage = CheckpointStorage(tmp_path / "async", job_id="c" * 32)
    coord = CheckpointCoordinator(storage, {"window": op})
    ref = _win(device=device)
    ref_coord = CheckpointCoordinator(CheckpointStorage(tmp_path / "sync", job_id="d" * 32),
                                      {"window": ref})
    tail = []
    for s in range(STEPS):
        out = op.process(*_batch(s, device=device))
        ref.process(*_batch(s, device=device))
        if s == CUT:
            coord.trigger_async(s, sources={"next_step": s + 1})
            sync_path = ref_coord.trigger(s)
        if s == CUT + 1:
            assert storage.latest() is None or coord._pending is None  # not restorable yet
        if s == CUT + 2:
            path = coord.complete_pending()
            assert storage.latest() == path
        if s > CUT:
            tail += out
    tail += op.finish()
    meta = read_metadata(path)
    assert meta["async"] and meta["step"] == CUT and meta["checkpoint_id"] == 1
    a = (path / "window-0.kg").read_bytes()
    b = (sync_path / "window-0.kg").read_bytes()
    assert a == b
    op2 = _win(device=device)
    CheckpointCoordinator(storage, {"window": op2}).restore()
    tail2 = []
    for s in range(CUT + 1, STEPS):
        tail2 += op2.process(*_batch(s, device=device))
    tail2 += op2.finish()
    assert _fires(tail) == _fires(tail2)
    st = coord.stats[-1]
    assert st["type"] == "checkpoint-async" and st["sync_ms"] <= st["ms"]


def test_async_checkpoint_matches_sync(tmp_path):
    _async_roundtrip(tmp_path, "cpu")


def test_async_checkpoint_error_surfaces(tmp_path):
    op = _win()
    coord = CheckpointCoordinator(CheckpointStorage(tmp_path), {"window": op})
    op.process(*_batch(0))

    def boom():
        raise OSError("disk full")

    op.snapshot_state_async = lambda: boom
    coord.trigger_async(0)
    with pytest.raises(RuntimeError, match="async checkpoint 1 failed"):
        coord.complete_pending()
    assert coord.storage.latest() is None


def test_retention_savepoint_and_incomplete(tmp_path):
    op = KeyedRollingOperator(agg=K.AGG_COUNT, device="cpu", max_keys=5000, batch_capacity=PER)
    storage = CheckpointStorage(tmp_path, job_id="0123456789abcdef" * 2)
    coord = CheckpointCoordinator(storage, {"count": op}, interval_steps=2, retain=2)
    for s in range(1, 8):
        k, _t, v = _batch(s)
        op.process(k, v)
        coord.maybe_trigger(s)
    done = [p.name for p in storage.completed_checkpoints()]
    assert done == ["chk-2", "chk-3"]  # steps 2,4,6 -> ids 1,2,3; retain 2
    (storage.job_dir / "chk-9").mkdir()  # no _metadata: incomplete, never restored
    assert storage.latest().name == "chk-3"
    sp = coord.savepoint(8, target=str(tmp_path / "sp"))
    assert re.fullmatch(r"savepoint-012345-[0-9a-f]{12}", sp.name)
    assert read_metadata(sp)["type"] == "savepoint"
    op2 = KeyedRollingOperator(agg=K.AGG_COUNT, device="cpu", max_keys=5000, batch_capacity=PER)
    CheckpointCoordinator(storage, {"count": op2}).restore(sp)
    for key in (1, 17, 333):
        assert op.state_of(key) == op2.state_of(key)


def test_rolling_restore_continues_counts(tmp_path):
    a = KeyedRollingOperator(agg=K.AGG_COUNT, device="cpu", max_keys=5000, batch_capacity=PER)
    storage = CheckpointStorage(tmp_path)
    coord = CheckpointCoordinator(storage, {"c": a})
    rows_a = []
    for s in range(6):
        k, _t, v = _batch(s)
        r = a.process(k, v)
        if s == 2:
            coord.trigger(s)
        if s > 2:
            rows_a.append(sorted(zip(r.keys.tolist(), r.values.tolist(), r.tags.tolist())))
    b = KeyedRollingOperator(agg=K.AGG_COUNT, device="cpu", max_keys=5000, batch_capacity=PER)
    CheckpointCoordinator(storage, {"c": b}).restore()
    rows_b = []
    for s in range(3, 6):
        k, _t, v = _batch(s)
        r = b.process(k, v)
        rows_b.append(sorted(zip(r.keys.tolist(), r.values.tolist(), r.tags.tolist())))
    assert rows_a == rows_b


def test_session_restore(tmp_path):
    mk = lambda: KeyedSessionOperator(gap=150, lateness=400, agg=K.AGG_SUM_I64, device="cpu",
                                      max_keys=8000, batch_capacity=PER, ooo_bound=500)
    a = mk()
    storage = CheckpointStorage(tmp_path)
    coord = CheckpointCoordinator(storage, {"s": a})
    got_a = []
    for s in range(STEPS):
        r = a.process(*_batch(s))
        if s == CUT:
            coord.trigger(s)
        if s > CUT:
            got_a += list(zip(r.keys.tolist(), r.start.tolist(), r.raw.tolist(), r.counts.tolist()))
    r = a.finish()
    got_a += list(zip(r.keys.tolist(), r.start.tolist(), r.raw.tolist(), r.counts.tolist()))
    b = mk()
    CheckpointCoordinator(storage, {"s": b}).restore()
    got_b = []
    for s in range(CUT + 1, STEPS):
        r = b.process(*_batch(s))
        got_b += list(zip(r.keys.tolist(), r.start.tolist(), r.raw.tolist(), r.counts.tolist()))
    r = b.finish()
    got_b += list(zip(r.keys.tolist(), r.start.tolist(), r.raw.tolist(), r.counts.tolist()))
    assert sorted(got_a) == sorted(got_b)


def test_owned_key_groups_partition_all():
    for world, par in ((1, 1), (2, 2), (2, 4), (4, 4), (3, 6)):
        seen = []
        for r in range(world):
            lo, hi = owned_key_groups(r, world, par, 128)
            seen += list(range(lo, hi + 1))
        assert seen == list(range(128))


# ---- rescale: checkpoint at world 2 (gloo), restore at world 1 and vice versa -------------------
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, port, root, mode, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    op = _win(comm=TorchComm(), batch_capacity=PER * 2)
    storage = CheckpointStorage(root, job_id="b" * 32)
    coord = CheckpointCoordinator(storage, {"window": op})
    out = []
    if mode == "write":
        for s in range(CUT + 1):
            op.process(*_batch(s, src=rank))
        coord.trigger(CUT)
    else:
        coord.restore()
        for s in range(CUT + 1, STEPS):
            out += op.process(*_batch(s, src=rank))
        out += op.finish()
    q.put((rank, _fires(out)))
    dist.barrier()
    dist.destroy_process_group()


def _spawn(world, root, mode):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_rank_main, args=(r, world, port, root, mode, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    return sorted(x for _r, f in res for x in f)


def _single_run_tail(world_sources, **kw):
    op = _win(batch_capacity=PER * world_sources, **kw)
    out = []
    for s in range(STEPS):
        parts = [_batch(s, src=r) for r in range(world_sources)]
        o = op.process(*[torch.cat([p[i] for p in parts]) for i in range(3)])
        if s > CUT:
            out += o
    out += op.finish()
    return _fires(out)


def test_rescale_2_to_1_and_1_to_2(tmp_path):
    strip = lambda f: sorted(x[:4] for x in f)
    ref = strip(_single_run_tail(2))
    # world 2 writes, world 1 restores (reads both old ranks' files)
    root = tmp_path / "a"
    _spawn(2, root, "write")
    op = _win(batch_capacity=PER * 2)
    CheckpointCoordinator(CheckpointStorage(root, job_id="b" * 32), {"window": op}).restore()
    out = []
    for s in range(CUT + 1, STEPS):
        parts = [_batch(s, src=r) for r in range(2)]
        out += op.process(*[torch.cat([p[i] for p in parts]) for i in range(3)])
    out += op.finish()
    assert strip(_fires(out)) == ref
    # world 1 writes, world 2 restores (each rank reads its key groups)
    root = tmp_path / "b"
    op = _win(batch_capacity=PER * 2)
    coord = CheckpointCoordinator(CheckpointStorage(root, job_id="b" * 32), {"window": op})
    for s in range(CUT + 1):
        parts = [_batch(s, src=r) for r in range(2)]
        op.process(*[torch.cat([p[i] for p in parts]) for i in range(3)])
    coord.trigger(CUT)
    assert strip(_spawn(2, root, "read")) == ref


# ---- GPU -------------------------------------------------------------------------------------
@pytest.mark.gpu
def test_gpu_window_checkpoint_restores_on_cpu_and_gpu(tmp_path):
    op = _win(device="cuda")
    storage = CheckpointStorage(tmp_path)
    coord = CheckpointCoordinator(storage, {"window": op})
    tail = []
    for s in range(STEPS):
        out = op.process(*_batch(s, device="cuda"))
        if s == CUT:
            coord.trigger(s)
        if s > CUT:
            tail += out
    tail += op.finish()
    for dev in ("cuda", "cpu"):
        op2 = _win(device=dev)
        CheckpointCoordinator(storage, {"window": op2}).restore()
        t2 = []
        for s in range(CUT + 1, STEPS):
            t2 += op2.process(*_batch(s, device=dev))
        t2 += op2.finish()
        assert _fires(tail) == _fires(t2), dev


@pytest.mark.gpu
def test_gpu_async_checkpoint_matches_sync(tmp_path):
    _async_roundtrip(tmp_path, "cuda")


@pytest.mark.gpu
def test_gpu_session_and_rolling_restore(tmp_path):
    s_op = KeyedSessionOperator(gap=150, lateness=400, agg=K.AGG_SUM_I64, device="cuda",
                                max_keys=8000, batch_capacity=PER, ooo_bound=500)
    r_op = KeyedRollingOperator(agg=K.AGG_COUNT, device="cuda", max_keys=5000, batch_capacity=PER)
    storage = CheckpointStorage(tmp_path)
    coord = CheckpointCoordinator(storage, {"s": s_op, "r": r_op})
    tail = []
    for s in range(STEPS):
        k, t, v = _batch(s, device="cuda")
        rs = s_op.process(k, t, v)
        r_op.process(k, v)
        if s == CUT:
            coord.trigger(s)
        if s > CUT:
            tail += list(zip(rs.keys.tolist(), rs.start.tolist(), rs.raw.tolist()))
    rs = s_op.finish()
    tail += list(zip(rs.keys.tolist(), rs.start.tolist(), rs.raw.tolist()))
    s2 = KeyedSessionOperator(gap=150, lateness=400, agg=K.AGG_SUM_I64, device="cuda",
                              max_keys=8000, batch_capacity=PER, ooo_bound=500)
    r2 = KeyedRollingOperator(agg=K.AGG_COUNT, device="cuda", max_keys=5000, batch_capacity=PER)
    CheckpointCoordinator(storage, {"s": s2, "r": r2}).restore()
    t2 = []
    for s in range(CUT + 1, STEPS):
        k, t, v = _batch(s, device="cuda")
        rs = s2.process(k, t, v)
        r2.process(k, v)
        t2 += list(zip(rs.keys.tolist(), rs.start.tolist(), rs.raw.tolist()))
    rs = s2.finish()
    t2 += list(zip(rs.keys.tolist(), rs.start.tolist(), rs.raw.tolist()))
    assert sorted(tail) == sorted(t2)
    for key in (3, 99, 2048):
        assert r_op.state_of(key) == r2.state_of(key)


# ---- local-global window state (exchange="partials") ------------------------------------------
def test_local_global_checkpoint_rescale(tmp_path):
    """Every rank of a local-global operator holds PARTIAL accumulators of every key it saw;
    its checkpoint files therefore carry several rows per (key, pane). Restoring at any world
    size folds them (restore_state combines duplicate rows with the aggregate), and the run
    continues exactly like an uninterrupted single-rank run."""
    from mxstream.parallel.comm import run_loopback

    def mk(comm=None, world=1):
        return _win(comm=comm, lateness=0, batch_capacity=PER * 2, exchange="auto")

    strip = lambda f: sorted(x[:4] for x in f)
    ref = strip(_single_run_tail(2, lateness=0))
    root = tmp_path / "lg"
    storage = CheckpointStorage(root, job_id="c" * 32)

    def write(comm):
        op = mk(comm)
        assert op.local_global
        coord = CheckpointCoordinator(storage, {"window": op})
        for s in range(CUT + 1):
            op.process(*_batch(s, src=comm.rank))
        coord.trigger(CUT)
        return True

    run_loopback(2, write)

    def read(comm):
        op = mk(comm)
        CheckpointCoordinator(storage, {"window": op}).restore()
        out = []
        for s in range(CUT + 1, STEPS):
            # Two source partitions feed the job; at world 1 one rank reads both.
            if comm.world == 1:
                parts = [_batch(s, src=r) for r in range(2)]
                out += op.process(*[torch.cat([p[i] for p in parts]) for i in range(3)])
            else:
                out += op.process(*_batch(s, src=comm.rank))
        return _fires(out + op.finish())

    for world in (1, 2):
        got = sorted(x for f in run_loopback(world, read) for x in f)
        assert strip(got) == ref, world


def test_local_global_lateness_checkpoint_restore(tmp_path):
    """Local-global aggregation with allowed lateness: a restore rebuilds the owners' merged
    values of fired-but-not-cleaned windows, so late re-firings after the restore emit the same
    totals as an uninterrupted run (at world 1 and 2)."""
    from mxstream.parallel.comm import run_loopback

    def batch(s, src):
        k, t, v = _batch(s, src=src)
        if s >= 2:
            t[::29] -= 1700  # late: behind the watermark, within the allowed lateness
        return k, t, v

    def single():
        op = _win(batch_capacity=PER * 2)
        out = []
        for s in range(STEPS):
            parts = [batch(s, r) for r in range(2)]
            o = op.process(*[torch.cat([p[i] for p in parts]) for i in range(3)])
            if s > CUT:
                out += o
        return _fires(out + op.finish())

    ref = single()
    assert any(x[4] for x in ref)  # re-firings after the cut
    storage = CheckpointStorage(tmp_path / "lgl", job_id="d" * 32)

    def write(comm):
        op = _win(comm=comm, batch_capacity=PER * 2, exchange="partials")
        assert op.local_global and op.dacc_g is not None
        coord = CheckpointCoordinator(storage, {"window": op})
        for s in range(CUT + 1):
            op.process(*batch(s, comm.rank))
        coord.trigger(CUT)
        return True

    run_loopback(2, write)

    def read(comm):
        op = _win(comm=comm, batch_capacity=PER * 2)
        CheckpointCoordinator(storage, {"window": op}).restore()
        out = []
        for s in range(CUT + 1, STEPS):
            if comm.world == 1:
                parts = [batch(s, r) for r in range(2)]
                out += op.process(*[torch.cat([p[i] for p in parts]) for i in range(3)])
            else:
                out += op.process(*batch(s, comm.rank))
        return _fires(out + op.finish())

    for world in (1, 2):
        got = sorted(x for f in run_loopback(world, read) for x in f)
        assert got == ref, world
