"""Multi-process keyBy shuffle over torch.distributed (gloo): results are invariant to G.

Each rank ingests its own source partition; the keyed window operator routes records by Flink
key group to the owning rank (equal-split all-to-all), the watermark is the MIN over ranks.
The union of what all ranks fire must equal a single-rank run over the concatenated input.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from mxstream.ops import kernels as K
from mxstream.parallel.comm import TorchComm
from mxstream.runtime.window_operator import KeyedWindowOperator

STEPS, PER = 6, 3000


def _batch(rank, step):
    keys = torch.empty(PER, dtype=torch.int64)
    ts = torch.empty_like(keys)
    vals = torch.empty_like(keys)
    K.gen_events(keys, ts, vals, seed=11, stream_id=rank, idx0=step * PER, nkeys=5000,
                 ts_base=step * 2000, ts_span=2000, disorder=700, val_lo=0, val_span=1000)
    return keys, ts, vals


def _collect(out):
    return {(r.window_start, int(k)): (int(a), int(c), r.refire)
            for r in out for k, a, c in zip(r.keys, r.raw, r.counts)}


def _worker(rank, world, port, size, slide, lateness, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    comm = TorchComm()
    op = KeyedWindowOperator(size=size, slide=slide, lateness=lateness, agg=K.AGG_SUM_I64,
                             device="cpu", comm=comm, max_keys=5000, batch_capacity=PER,
                             ooo_bound=500, cap_log2=8)
    out = []
    for step in range(STEPS):
        out += op.process(*_batch(rank, step))
    out += op.finish()
    q.put((rank, _collect(out), op.metrics.num_late_records_dropped))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("size,slide,lateness", [(3000, 3000, 0), (4000, 1000, 1500)])
def test_results_invariant_to_world_size(world, size, slide, lateness):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, size, slide, lateness, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    merged, late = {}, 0
    owners = {}
    for rank, d, nl in res:
        late += nl
        for k, v in d.items():
            assert k not in owners, "a (window, key) fired on two ranks"
            owners[k] = rank
            merged[k] = v
    # Single-rank reference: one operator sees every rank's batches, step by step.
    op = KeyedWindowOperator(size=size, slide=slide, lateness=lateness, agg=K.AGG_SUM_I64,
                             device="cpu", max_keys=5000, batch_capacity=PER * world,
                             ooo_bound=500, cap_log2=8)
    out = []
    for step in range(STEPS):
        parts = [_batch(r, step) for r in range(world)]
        out += op.process(*[torch.cat([p[i] for p in parts]) for i in range(3)])
    out += op.finish()
    ref = _collect(out)
    strip = lambda d: {k: v[:2] for k, v in d.items()}
    assert strip(merged) == strip(ref)
    assert late == op.metrics.num_late_records_dropped


# ---- session windows: same invariance ----------------------------------------------------
def _collect_sessions(rows):
    return {(int(k), int(s)): (int(e), int(a), int(c))
            for k, s, e, a, c in zip(rows.keys, rows.start, rows.end, rows.raw, rows.counts)}


def _session_worker(rank, world, port, q):
    from mxstream.runtime.session_operator import KeyedSessionOperator

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    op = KeyedSessionOperator(gap=40, lateness=300, agg=K.AGG_SUM_I64, device="cpu",
                              comm=TorchComm(), max_keys=5000, batch_capacity=PER, ooo_bound=500,
                              cap_log2=8)
    got = {}
    for step in range(STEPS):
        got.update(_collect_sessions(op.process(*_batch(rank, step))))
    got.update(_collect_sessions(op.finish()))
    q.put((rank, got, op.metrics.num_late_records_dropped))
    dist.barrier()
    dist.destroy_process_group()


def test_sessions_invariant_to_world_size():
    from mxstream.runtime.session_operator import KeyedSessionOperator

    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_session_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    merged, late = {}, 0
    for _rank, d, nl in res:
        late += nl
        assert not (set(d) & set(merged)), "a session fired on two ranks"
        merged.update(d)
    op = KeyedSessionOperator(gap=40, lateness=300, agg=K.AGG_SUM_I64, device="cpu",
                              max_keys=5000, batch_capacity=PER * world, ooo_bound=500, cap_log2=8)
    ref = {}
    for step in range(STEPS):
        parts = [_batch(r, step) for r in range(world)]
        ref.update(_collect_sessions(op.process(*[torch.cat([p[i] for p in parts])
                                                  for i in range(3)])))
    ref.update(_collect_sessions(op.finish()))
    assert merged == ref
    assert late == op.metrics.num_late_records_dropped


# ---- vector-metric windows: vectors travel with their records --------------------------------
def _vec_batch(rank, step, dim=32):
    from mxstream.ops import vector as V

    keys, ts, _ = _batch(rank, step)
    vec = torch.empty(PER, dim, dtype=torch.float32)
    V.gen_vectors(vec, seed=3, stream_id=rank, idx0=step * PER)
    return keys, ts, vec


def _collect_vec(out):
    return {(r.window_start, int(k)): (v.tolist(), int(c))
            for r in out for k, v, c in zip(r.keys, r.values, r.counts)}


def _vector_worker(rank, world, port, q):
    from mxstream.runtime.vector_window_operator import VectorWindowOperator

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    op = VectorWindowOperator(dim=32, size=3000, slide=1000, device="cpu", comm=TorchComm(),
                              max_keys=5000, batch_capacity=PER, ooo_bound=500)
    out = []
    for step in range(STEPS):
        out += op.process(*_vec_batch(rank, step))
    out += op.finish()
    q.put((rank, _collect_vec(out), op.metrics.num_late_records_dropped))
    dist.barrier()
    dist.destroy_process_group()


def test_vector_windows_invariant_to_world_size():
    import numpy as np

    from mxstream.runtime.vector_window_operator import VectorWindowOperator

    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_vector_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    merged, late = {}, 0
    for _rank, d, nl in res:
        late += nl
        assert not (set(d) & set(merged)), "a (window, key) fired on two ranks"
        merged.update(d)
    op = VectorWindowOperator(dim=32, size=3000, slide=1000, device="cpu", max_keys=5000,
                              batch_capacity=PER * world, ooo_bound=500)
    out = []
    for step in range(STEPS):
        parts = [_vec_batch(r, step) for r in range(world)]
        out += op.process(*[torch.cat([p[i] for p in parts]) for i in range(3)])
    out += op.finish()
    ref = _collect_vec(out)
    assert merged.keys() == ref.keys()
    for k, (v, c) in ref.items():
        assert merged[k][1] == c
        np.testing.assert_allclose(merged[k][0], v, rtol=1e-5, atol=1e-4)
    assert late == op.metrics.num_late_records_dropped


# ---- keyed rolling state over gloo (ComputeCpuMax.java:26 keyBy(0).max(2), config 2) ---------
def _rolling_batch(rank, step, per=2500, nkeys=400):
    keys = torch.empty(per, dtype=torch.int64)
    K.gen_events(keys, torch.empty_like(keys), torch.empty_like(keys), seed=23, stream_id=rank,
                 idx0=step * per, nkeys=nkeys, ts_base=0, ts_span=1000, disorder=0, val_lo=-50,
                 val_span=1000)
    vals = torch.empty_like(keys)
    K.gen_events(torch.empty_like(keys), torch.empty_like(keys), vals, seed=29, stream_id=rank,
                 idx0=step * per, nkeys=nkeys, ts_base=0, ts_span=1000, disorder=0, val_lo=-50,
                 val_span=1000)
    return keys, vals


def _rolling_worker(rank, world, port, agg, q):
    from mxstream.runtime.rolling_operator import KeyedRollingOperator

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    op = KeyedRollingOperator(agg=agg, device="cpu", comm=TorchComm(), max_keys=400,
                              batch_capacity=2500, cap_log2=8)
    rows = {}
    for step in range(STEPS):
        r = op.process(*_rolling_batch(rank, step))
        for key, val, tag in zip(r.keys.tolist(), r.values.tolist(), r.tags.tolist()):
            rows[(step, tag >> 32, tag & 0xFFFFFFFF)] = (key, val)
    q.put((rank, rows))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("agg", [K.AGG_MAX_I64, K.AGG_COUNT])
def test_rolling_invariant_to_world_size(world, agg):
    """Every record's post-update value over a real gloo all-to-all equals a single-rank run
    over the step-wise concatenation (per key: step, then source rank, then arrival)."""
    from mxstream.runtime.rolling_operator import KeyedRollingOperator

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rolling_worker, args=(r, world, port, agg, q))
             for r in range(world)]
    for p in procs:
        p.start()
    merged = {}
    for _ in range(world):
        _, rows = q.get(timeout=120)
        assert not (set(rows) & set(merged))
        merged.update(rows)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    per = 2500
    ref_op = KeyedRollingOperator(agg=agg, device="cpu", max_keys=400, batch_capacity=per * world,
                                  cap_log2=8)
    ref = {}
    for step in range(STEPS):
        parts = [_rolling_batch(r, step) for r in range(world)]
        r = ref_op.process(torch.cat([p[0] for p in parts]), torch.cat([p[1] for p in parts]))
        for key, val, tag in zip(r.keys.tolist(), r.values.tolist(), r.tags.tolist()):
            i = tag & 0xFFFFFFFF
            ref[(step, i // per, i % per)] = (key, val)
    assert len(ref) == per * world * STEPS
    assert merged == ref
