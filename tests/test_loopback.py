"""G virtual ranks on one device (LoopbackComm): every keyed operator's results are invariant to G.

The loopback group runs the complete G>1 path -- Flink key-group partition into G x sub-table
buckets, the sender-side combiner, the equal-split all-to-all layout, combined-record
aggregation, the MIN watermark valve, overflow regrow -- in one process, so the same test runs
on the C++ twins (CPU) and on one MI355X (``-m gpu``). The reference for every G is a single
rank that sees every rank's batch of a step concatenated in rank order; integer sums must be
bit-exact. (Flink parity: keyBy at ``ComputeCpuMax.java:26``, ``BandwidthMonitorWithEventTime
.java:45``.)
"""
import numpy as np
import pytest
import torch

from mxstream.ops import kernels as K
from mxstream.parallel.comm import LoopbackGroup, run_loopback
from mxstream.runtime.window_operator import KeyedWindowOperator

STEPS = 6


def _devices():
    return [pytest.param("cpu", id="cpu"),
            pytest.param("cuda", id="gpu", marks=pytest.mark.gpu)]


def _sizes(dev):
    # The GPU run uses batches large enough for many partition workgroups per rank.
    return (3000, 5000, 8) if dev == "cpu" else (150_000, 60_000, None)


def _batch(dev, rank, step, per, nkeys, span=2000, disorder=700, late=0):
    d = torch.device(dev)
    keys = torch.empty(per, dtype=torch.int64, device=d)
    ts = torch.empty_like(keys)
    vals = torch.empty_like(keys)
    K.gen_events(keys, ts, vals, seed=11, stream_id=rank, idx0=step * per, nkeys=nkeys,
                 ts_base=step * span, ts_span=span, disorder=disorder, val_lo=0, val_span=1000)
    if late and step >= 2:
        ts[::37] -= late  # behind the watermark: late, mostly within the allowed lateness
    # Every source partition ends its batch at the same event time, so the G-rank watermark
    # (MIN over ranks of max ts - bound) equals the single-rank reference's (max over all).
    ts[-1] = step * span + span
    return keys, ts, vals


def _concat(dev, world, step, per, nkeys, late=0):
    parts = [_batch(dev, r, step, per, nkeys, late=late) for r in range(world)]
    return [torch.cat([p[i] for p in parts]) for i in range(3)]


def _collect(out):
    return {(r.window_start, int(k)): (int(a), int(c))
            for r in out for k, a, c in zip(r.keys, r.raw, r.counts)}


def _collect_seq(out):
    seq = {}
    for r in out:
        for k, a, c in zip(r.keys, r.raw, r.counts):
            seq.setdefault((r.window_start, int(k)), []).append((bool(r.refire), int(a), int(c)))
    return seq


def _skip_no_gpu(dev):
    if dev == "cuda" and not torch.cuda.is_available():
        pytest.skip("no GPU")


@pytest.mark.parametrize("dev", _devices())
@pytest.mark.parametrize("world", [1, 2, 4, 8])
@pytest.mark.parametrize("size,slide,lateness,exchange", [
    (3000, 3000, 0, "records"), (3000, 3000, 0, "partials"), (4000, 1000, 0, "partials"),
    (4000, 1000, 1500, "records"), (4000, 1000, 1500, "partials"),
    (3000, 3000, 2500, "partials")])
@pytest.mark.parametrize("pipeline", [False, True, "stream"])
def test_window_invariant_to_world(dev, world, size, slide, lateness, exchange, pipeline):
    """pipeline=True: the partition of batch i+1 overlaps the combiner / all-to-all /
    aggregation / firing of batch i on a second stream (GPU); on the CPU twins the same
    one-step-deferred control flow runs synchronously. exchange='partials': local-global
    aggregation (no per-step exchange; partial accumulators travel when a window fires)."""
    _skip_no_gpu(dev)
    per, nkeys, cap_log2 = _sizes(dev)
    late_shift = lateness * 9 // 10 + 700 if lateness else 0

    def make(comm, batch_capacity, pipe=pipeline):
        return KeyedWindowOperator(size=size, slide=slide, lateness=lateness, agg=K.AGG_SUM_I64,
                                   device=dev, comm=comm, max_keys=nkeys,
                                   batch_capacity=batch_capacity, ooo_bound=500, cap_log2=cap_log2,
                                   pipeline=pipe, exchange=exchange)

    def rank_fn(comm):
        op = make(comm, per)
        out = []
        for step in range(STEPS):
            out += op.process(*_batch(dev, comm.rank, step, per, nkeys, late=late_shift))
        out += op.finish()
        return _collect(out), op.metrics.num_late_records_dropped, op.metrics.extra, \
            _collect_seq(out)

    res = run_loopback(world, rank_fn, device=torch.device(dev))
    merged, late, seqs = {}, 0, {}
    for d, nl, _, sq in res:
        assert not (set(d) & set(merged)), "a (window, key) fired on two ranks"
        merged.update(d)
        seqs.update(sq)
        late += nl
    ref_op = make(None, per * world, pipe=False)  # unpipelined single rank: the reference
    out = []
    for step in range(STEPS):
        out += ref_op.process(*_concat(dev, world, step, per, nkeys, late=late_shift))
    out += ref_op.finish()
    ref = _collect(out)
    assert len(ref) > 0
    assert merged == ref
    assert late == ref_op.metrics.num_late_records_dropped
    if lateness:
        # every firing and re-firing of every (window, key), in order, with its value
        ref_seq = _collect_seq(out)
        assert sum(len(v) for v in ref_seq.values()) > len(ref_seq)  # re-firings happened
        assert seqs == ref_seq


@pytest.mark.parametrize("dev", _devices())
@pytest.mark.parametrize("compact", [False, True])
def test_window_loopback_without_combiner(dev, compact):
    """The plain exchange (every record crosses the all-to-all) gives the same result, with
    24-byte and with 16-byte (compact, the GPU default for integer aggregates) records: each
    rank's chunk of the equal split is nsub * bucket_cap records of the layout in use."""
    _skip_no_gpu(dev)
    per, nkeys, cap_log2 = _sizes(dev)
    world = 4

    def rank_fn(comm):
        op = KeyedWindowOperator(size=3000, agg=K.AGG_SUM_I64, device=dev, comm=comm,
                                 max_keys=nkeys, batch_capacity=per, ooo_bound=500,
                                 cap_log2=cap_log2, combine=False, compact=compact,
                                 exchange="records")
        out = []
        for step in range(STEPS):
            out += op.process(*_batch(dev, comm.rank, step, per, nkeys))
        return _collect(out + op.finish())

    merged = {}
    for d in run_loopback(world, rank_fn, device=torch.device(dev)):
        merged.update(d)
    ref_op = KeyedWindowOperator(size=3000, agg=K.AGG_SUM_I64, device=dev, max_keys=nkeys,
                                 batch_capacity=per * world, ooo_bound=500, cap_log2=cap_log2)
    out = []
    for step in range(STEPS):
        out += ref_op.process(*_concat(dev, world, step, per, nkeys))
    assert merged == _collect(out + ref_op.finish())


@pytest.mark.parametrize("dev", _devices())
@pytest.mark.parametrize("pipeline,exchange", [(False, "records"), (True, "records"),
                                               (False, "partials")])
def test_window_loopback_bucket_regrow(dev, pipeline, exchange):
    """A skewed rank overflows its fixed-capacity buckets: every rank regrows and redoes the
    step together (the flag travels in the step's MIN all-reduce), results unchanged."""
    _skip_no_gpu(dev)
    per, nkeys, cap_log2 = _sizes(dev)
    world = 2

    def batch(rank, step):
        k, t, v = _batch(dev, rank, step, per, nkeys)
        if rank == 1:
            k = k % 7  # a handful of hot keys: a few buckets receive everything
        return k, t, v

    def rank_fn(comm):
        op = KeyedWindowOperator(size=3000, agg=K.AGG_SUM_I64, device=dev, comm=comm,
                                 max_keys=nkeys, batch_capacity=per, ooo_bound=500,
                                 cap_log2=cap_log2, bucket_slack=1.0, pipeline=pipeline,
                                 exchange=exchange)
        out = []
        for step in range(STEPS):
            out += op.process(*batch(comm.rank, step))
        return _collect(out + op.finish()), op.metrics.bucket_regrows

    res = run_loopback(world, rank_fn, device=torch.device(dev))
    assert all(r[1] >= 1 for r in res)
    merged = {}
    for d, _ in res:
        merged.update(d)
    ref_op = KeyedWindowOperator(size=3000, agg=K.AGG_SUM_I64, device=dev, max_keys=nkeys,
                                 batch_capacity=per * world, ooo_bound=500, cap_log2=cap_log2)
    out = []
    for step in range(STEPS):
        parts = [batch(r, step) for r in range(world)]
        out += ref_op.process(*[torch.cat([p[i] for p in parts]) for i in range(3)])
    assert merged == _collect(out + ref_op.finish())


# ---- keyed rolling state (ComputeCpuMax.java:26) --------------------------------------------
@pytest.mark.parametrize("dev", _devices())
@pytest.mark.parametrize("world", [2, 4, 8])
@pytest.mark.parametrize("agg", [K.AGG_SUM_I64, K.AGG_MAX_I64, K.AGG_COUNT])
def test_rolling_invariant_to_world(dev, world, agg):
    from mxstream.runtime.rolling_operator import KeyedRollingOperator

    _skip_no_gpu(dev)
    per = 2000 if dev == "cpu" else 100_000
    nkeys = 300 if dev == "cpu" else 10_000

    def rank_fn(comm):
        op = KeyedRollingOperator(agg=agg, device=dev, comm=comm, max_keys=nkeys,
                                  batch_capacity=per, cap_log2=8 if dev == "cpu" else None)
        rows = {}
        for step in range(4):
            k, _, v = _batch(dev, comm.rank, step, per, nkeys)
            r = op.process(k, v)
            for key, val, tag in zip(r.keys.tolist(), r.values.tolist(), r.tags.tolist()):
                rows[(step, tag >> 32, tag & 0xFFFFFFFF)] = (key, val)
        return rows

    merged = {}
    for d in run_loopback(world, rank_fn, device=torch.device(dev)):
        assert not (set(d) & set(merged))
        merged.update(d)
    ref_op = KeyedRollingOperator(agg=agg, device=dev, max_keys=nkeys, batch_capacity=per * world,
                                  cap_log2=8 if dev == "cpu" else None)
    ref = {}
    for step in range(4):
        k, _, v = _concat(dev, world, step, per, nkeys)
        r = ref_op.process(k, v)
        for key, val, tag in zip(r.keys.tolist(), r.values.tolist(), r.tags.tolist()):
            i = tag & 0xFFFFFFFF  # single rank: the index in the concatenated batch
            ref[(step, i // per, i % per)] = (key, val)
    assert len(ref) == per * world * 4
    assert merged == ref


# ---- session windows (chapter3/README.md:412-428, BASELINE config 5) -----------------------
def _collect_sessions(rows):
    return {(int(k), int(s)): (int(e), int(a), int(c))
            for k, s, e, a, c in zip(rows.keys, rows.start, rows.end, rows.raw, rows.counts)}


@pytest.mark.parametrize("dev", _devices())
@pytest.mark.parametrize("world", [2, 4, 8])
@pytest.mark.parametrize("pipeline", [False, True])
def test_sessions_invariant_to_world(dev, world, pipeline):
    """pipeline=True (GPU): the pipelined session step at G ranks (its fires come one call
    later; the union over ranks and calls is the same)."""
    from mxstream.runtime.session_operator import KeyedSessionOperator

    _skip_no_gpu(dev)
    per = 3000 if dev == "cpu" else 60_000
    nkeys = 5000 if dev == "cpu" else 40_000

    def make(comm, cap, pipe=pipeline):
        return KeyedSessionOperator(gap=40, lateness=300, agg=K.AGG_SUM_I64, device=dev,
                                    comm=comm, max_keys=nkeys, batch_capacity=cap, ooo_bound=500,
                                    cap_log2=8 if dev == "cpu" else None, pipeline=pipe)

    def rank_fn(comm):
        op = make(comm, per)
        got = {}
        for step in range(STEPS):
            got.update(_collect_sessions(op.process(*_batch(dev, comm.rank, step, per, nkeys))))
        got.update(_collect_sessions(op.finish()))
        return got, op.metrics.num_late_records_dropped

    merged, late = {}, 0
    for d, nl in run_loopback(world, rank_fn, device=torch.device(dev)):
        assert not (set(d) & set(merged)), "a session fired on two ranks"
        merged.update(d)
        late += nl
    op = make(None, per * world, pipe=False)
    ref = {}
    for step in range(STEPS):
        ref.update(_collect_sessions(op.process(*_concat(dev, world, step, per, nkeys))))
    ref.update(_collect_sessions(op.finish()))
    assert len(ref) > 0
    assert merged == ref
    assert late == op.metrics.num_late_records_dropped


# ---- vector-metric windows (MFMA path on the GPU) ------------------------------------------
@pytest.mark.parametrize("dev", _devices())
@pytest.mark.parametrize("world", [2, 8])
def test_vector_windows_invariant_to_world(dev, world):
    from mxstream.ops import vector as V
    from mxstream.runtime.vector_window_operator import VectorWindowOperator

    _skip_no_gpu(dev)
    per = 2000 if dev == "cpu" else 40_000
    nkeys = 3000 if dev == "cpu" else 20_000

    def vb(rank, step):
        keys, ts, _ = _batch(dev, rank, step, per, nkeys)
        vec = torch.empty(per, 32, dtype=torch.float32, device=torch.device(dev))
        V.gen_vectors(vec, seed=3, stream_id=rank, idx0=step * per)
        return keys, ts, vec

    def collect(out):
        return {(r.window_start, int(k)): (np.asarray(v), int(c))
                for r in out for k, v, c in zip(r.keys, r.values, r.counts)}

    def rank_fn(comm):
        op = VectorWindowOperator(dim=32, size=3000, slide=1000, device=dev, comm=comm,
                                  max_keys=nkeys, batch_capacity=per, ooo_bound=500)
        out = []
        for step in range(4):
            out += op.process(*vb(comm.rank, step))
        return collect(out + op.finish())

    merged = {}
    for d in run_loopback(world, rank_fn, device=torch.device(dev)):
        assert not (set(d) & set(merged))
        merged.update(d)
    op = VectorWindowOperator(dim=32, size=3000, slide=1000, device=dev, max_keys=nkeys,
                              batch_capacity=per * world, ooo_bound=500)
    out = []
    for step in range(4):
        parts = [vb(r, step) for r in range(world)]
        out += op.process(*[torch.cat([p[i] for p in parts]) for i in range(3)])
    ref = collect(out + op.finish())
    assert merged.keys() == ref.keys()
    for k, (v, c) in ref.items():
        assert merged[k][1] == c
        np.testing.assert_allclose(merged[k][0], v, rtol=1e-5, atol=1e-4)


# ---- the communicator itself ------------------------------------------------------------------
@pytest.mark.parametrize("dev", _devices())
def test_loopback_collectives_match_all_to_all_single_layout(dev):
    _skip_no_gpu(dev)
    world = 4
    d = torch.device(dev)

    def rank_fn(comm):
        inp = torch.arange(world * 3, dtype=torch.int64, device=d) + 100 * comm.rank
        out = torch.empty_like(inp)
        comm.all_to_all(out, inp)
        t = torch.tensor([comm.rank + 5, -comm.rank], dtype=torch.int64, device=d)
        comm.allreduce_min_(t)
        s = torch.tensor([comm.rank + 1], dtype=torch.int64, device=d)
        comm.allreduce_sum_(s)
        objs = comm.all_gather_object({"r": comm.rank})
        b = comm.broadcast_object("x" if comm.rank == 2 else None, src=2)
        return out.cpu().tolist(), t.cpu().tolist(), int(s.item()), objs, b

    res = run_loopback(world, rank_fn, device=d)
    for r, (out, t, s, objs, b) in enumerate(res):
        assert out == [100 * src + r * 3 + j for src in range(world) for j in range(3)]
        assert t == [5, -(world - 1)]
        assert s == sum(range(1, world + 1))
        assert objs == [{"r": i} for i in range(world)]
        assert b == "x"


def test_loopback_error_on_one_rank_propagates():
    def rank_fn(comm):
        if comm.rank == 1:
            raise ValueError("boom")
        comm.barrier()
        return comm.rank

    with pytest.raises(ValueError, match="boom"):
        run_loopback(3, rank_fn, timeout_s=30)
    assert LoopbackGroup(2).world == 2


# ---- idle source partitions (StatusWatermarkValve, SURVEY.md F-valve) --------------------------
@pytest.mark.parametrize("dev", _devices())
@pytest.mark.parametrize("exchange", ["records", "partials"])
def test_idle_partition_does_not_hold_the_watermark(dev, exchange):
    """Rank 1's source goes quiet after step 1. Without idleness its stale watermark holds the
    MIN valve back: no window fires until end of input. With idle_timeout_steps=1 the valve
    takes the MIN over active partitions and the windows fire on time, with the same results
    as one rank fed every batch."""
    _skip_no_gpu(dev)
    per, nkeys, cap_log2 = _sizes(dev)
    world, quiet_from = 2, 2

    def batch(rank, step):
        k, t, v = _batch(dev, rank, step, per, nkeys)
        if rank == 1 and step >= quiet_from:
            return k[:0], t[:0], v[:0]
        return k, t, v

    def run(idle_steps):
        def rank_fn(comm):
            op = KeyedWindowOperator(size=3000, agg=K.AGG_SUM_I64, device=dev, comm=comm,
                                     max_keys=nkeys, batch_capacity=per, ooo_bound=500,
                                     cap_log2=cap_log2, exchange=exchange,
                                     idle_timeout_steps=idle_steps)
            during = []
            for step in range(STEPS):
                during += op.process(*batch(comm.rank, step))
            return _collect(during), _collect(op.finish())
        res = run_loopback(world, rank_fn, device=torch.device(dev))
        during, total = {}, {}
        for d, f in res:
            during.update(d)
            total.update(d)
            total.update(f)
        return during, total

    ref_op = KeyedWindowOperator(size=3000, agg=K.AGG_SUM_I64, device=dev, max_keys=nkeys,
                                 batch_capacity=per * world, ooo_bound=500, cap_log2=cap_log2)
    ref_during = []
    for step in range(STEPS):
        parts = [batch(r, step) for r in range(world)]
        ref_during += ref_op.process(*[torch.cat([p[i] for p in parts]) for i in range(3)])
    ref_total = _collect(ref_during + ref_op.finish())
    ref_during = _collect(ref_during)

    held_during, held_total = run(None)
    live_during, live_total = run(1)
    assert len(ref_during) > len(_collect([])) and live_during == ref_during
    assert live_total == ref_total == held_total
    assert len(held_during) < len(ref_during)  # the quiet partition held the valve back


@pytest.mark.parametrize("dev", _devices())
@pytest.mark.parametrize("world", [1, 4])
def test_dense_keys_local_global_invariant(dev, world):
    """Dense key ids (directly addressed local tables) under local-global aggregation: the
    per-window results at G ranks equal one hashed-table rank's."""
    _skip_no_gpu(dev)
    per, nkeys, cap_log2 = _sizes(dev)

    def rank_fn(comm):
        op = KeyedWindowOperator(size=3000, slide=1000, agg=K.AGG_SUM_I64, device=dev, comm=comm,
                                 max_keys=nkeys, batch_capacity=per, ooo_bound=500,
                                 dense_keys=True, exchange="partials")
        out = []
        for step in range(STEPS):
            out += op.process(*_batch(dev, comm.rank, step, per, nkeys))
        return _collect(out + op.finish())

    merged = {}
    for d in run_loopback(world, rank_fn, device=torch.device(dev)):
        merged.update(d)
    ref_op = KeyedWindowOperator(size=3000, slide=1000, agg=K.AGG_SUM_I64, device=dev,
                                 max_keys=nkeys, batch_capacity=per * world, ooo_bound=500,
                                 cap_log2=cap_log2)
    out = []
    for step in range(STEPS):
        out += ref_op.process(*_concat(dev, world, step, per, nkeys))
    assert merged == _collect(out + ref_op.finish())


@pytest.mark.parametrize("dev", _devices())
@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("count_window", [0, 5])
def test_rolling_and_count_windows_invariant_to_world(dev, world, count_window):
    """Keyed rolling sums (ComputeCpuMax.java:26 shape) and tumbling count windows at G ranks:
    the owner sees a key's records ordered (source rank, arrival), i.e. the rank-ordered
    concatenation, so every key's emitted sequence equals the single-rank reference's."""
    _skip_no_gpu(dev)
    from mxstream.runtime.rolling_operator import KeyedRollingOperator

    per, nkeys = (4000, 700) if dev == "cpu" else (60_000, 20_000)

    def rows_by_key(rows, acc):
        order = np.argsort(rows.tags, kind="stable")  # (src << 32 | arrival): rank-major
        for i in order:
            acc.setdefault(int(rows.keys[i]), []).append(int(rows.values[i]))

    def rank_fn(comm):
        op = KeyedRollingOperator(agg=K.AGG_SUM_I64, device=dev, comm=comm, max_keys=nkeys,
                                  parallelism=comm.world, batch_capacity=per,
                                  count_window=count_window)
        got = {}
        for step in range(4):
            k, _, v = _batch(dev, comm.rank, step, per, nkeys)
            rows_by_key(op.process(k, v), got)
        return got

    ranks = run_loopback(world, rank_fn, device=torch.device(dev))
    merged = {}
    for g in ranks:
        for k, seq in g.items():
            assert k not in merged  # one owner per key
            merged[k] = seq
    ref_op = KeyedRollingOperator(agg=K.AGG_SUM_I64, device=dev, max_keys=nkeys,
                                  batch_capacity=per * world, count_window=count_window)
    ref = {}
    for step in range(4):
        k, _, v = _concat(dev, world, step, per, nkeys)
        rows_by_key(ref_op.process(k, v), ref)
    assert merged == ref and len(ref) > 0


@pytest.mark.parametrize("dev", _devices())
@pytest.mark.parametrize("world", [2, 3])
def test_deterministic_f64_sums_invariant_to_world(dev, world):
    """deterministic f64 sums at G virtual ranks (records exchange, and local-global partials)
    are bit-identical to the single-rank result on the rank-concatenated batches."""
    _skip_no_gpu(dev)
    per, nkeys = (3000, 400) if dev == "cpu" else (60_000, 20_000)
    rng = np.random.default_rng(5)
    vals = {(r, s): torch.from_numpy(rng.standard_normal(per) * 10.0 ** rng.integers(-5, 8, per))
            for r in range(world) for s in range(STEPS)}

    def batch(rank, step):
        k, t, _ = _batch("cpu", rank, step, per, nkeys)
        return k.to(dev), t.to(dev), vals[(rank, step)].view(torch.int64).to(dev)

    def collect(out, acc):
        for r in out:
            acc.update({(r.window_start, int(k)): int(a) for k, a in zip(r.keys, r.raw)})

    for exchange in ("records", "auto"):  # "auto" picks records exchange in this mode
        def rank_fn(comm):
            op = KeyedWindowOperator(size=3000, agg=K.AGG_SUM_F64, device=dev, comm=comm,
                                     max_keys=nkeys, parallelism=comm.world, batch_capacity=per,
                                     ooo_bound=700, deterministic=True, exchange=exchange)
            got = {}
            for step in range(STEPS):
                collect(op.process(*batch(comm.rank, step)), got)
            collect(op.finish(), got)
            return got

        merged = {}
        for g in run_loopback(world, rank_fn, device=torch.device(dev)):
            merged.update(g)
        ref_op = KeyedWindowOperator(size=3000, agg=K.AGG_SUM_F64, device=dev, max_keys=nkeys,
                                     batch_capacity=per * world, ooo_bound=700, deterministic=True)
        ref = {}
        for step in range(STEPS):
            parts = [batch(r, step) for r in range(world)]
            collect(ref_op.process(*[torch.cat([p[i] for p in parts]) for i in range(3)]), ref)
        collect(ref_op.finish(), ref)
        assert merged == ref and len(ref) > 100, exchange
    with pytest.raises(ValueError, match="deterministic"):
        run_loopback(2, lambda comm: KeyedWindowOperator(
            size=3000, agg=K.AGG_SUM_F64, device=dev, comm=comm, max_keys=nkeys,
            parallelism=2, deterministic=True, exchange="partials"), device=torch.device(dev))


@pytest.mark.parametrize("dev", _devices())
@pytest.mark.parametrize("pipeline", [False, "stream"])
@pytest.mark.parametrize("lateness", [0, 1500])
def test_combiner_overflow_redone_after_the_exchange(dev, pipeline, lateness):
    """The records exchange does not wait for the combiner's overflow check before the
    all-to-all: an overflowing step's aggregation skips itself on the device and the step is
    redone (larger combined buckets) when the check is read -- before any firing, re-firing or
    purge reads the state. Forced here by tiny combined buckets every step."""
    _skip_no_gpu(dev)
    per, nkeys, cap_log2 = (40_000, 20_000, 8) if dev == "cpu" else _sizes(dev)
    world = 4
    late = lateness * 9 // 10 + 700 if lateness else 0

    def make(comm, bc, pipe):
        return KeyedWindowOperator(size=4000, slide=1000, lateness=lateness, agg=K.AGG_SUM_I64,
                                   device=dev, comm=comm, max_keys=nkeys, batch_capacity=bc,
                                   ooo_bound=500, cap_log2=cap_log2, pipeline=pipe,
                                   exchange="records")

    def rank_fn(comm):
        op = make(comm, per, pipeline)
        out = []
        for step in range(STEPS):
            op.set_combine_hint(64)  # force an overflow of the combined buckets
            out += op.process(*_batch(dev, comm.rank, step, per, nkeys, late=late))
        out += op.finish()
        return _collect_seq(out), op.metrics.extra.get("combine_regrows", 0)

    res = run_loopback(world, rank_fn, device=torch.device(dev))
    assert all(r[1] >= STEPS // 2 for r in res)
    merged = {}
    for d, _ in res:
        merged.update(d)
    ref_op = make(None, per * world, False)
    out = []
    for step in range(STEPS):
        out += ref_op.process(*_concat(dev, world, step, per, nkeys, late=late))
    assert merged == _collect_seq(out + ref_op.finish())


@pytest.mark.parametrize("exchange,combine", [("records", False), ("records", None),
                                              ("partials", None)])
def test_exchange_bytes_close_to_payload_at_g8(exchange, combine):
    """The G > 1 exchanges move slices sized to the largest fill over the ranks (device repack),
    not the partition's fixed bucket capacity: at loopback G = 8 the all-to-all bytes stay
    within 1.2x of the records actually exchanged (metrics a2a_bytes / payload_bytes)."""
    W, n = 8, 1 << 18

    def rank(comm):
        op = KeyedWindowOperator(size=4000, slide=1000, agg=K.AGG_SUM_I64, device="cpu",
                                 comm=comm, max_keys=200_000, batch_capacity=n, ooo_bound=500,
                                 exchange=exchange, combine=combine, parallelism=W)
        for step in range(10):
            k = torch.empty(n, dtype=torch.int64)
            t = torch.empty_like(k)
            v = torch.empty_like(k)
            K.gen_events(k, t, v, seed=3, stream_id=comm.rank, idx0=step * n, nkeys=150_000,
                         ts_base=step * 1000, ts_span=1000, disorder=300, val_lo=0, val_span=100)
            op.process(k, t, v)
        op.finish()
        x = op.metrics.extra
        return x.get("a2a_bytes", 0), x.get("payload_bytes", 0)

    res = run_loopback(W, rank)
    a2a, payload = sum(r[0] for r in res), sum(r[1] for r in res)
    assert payload > 0 and a2a / payload <= 1.2, (a2a, payload)


@pytest.mark.parametrize("dev", _devices())
@pytest.mark.parametrize("world", [1, 2, 4])
@pytest.mark.parametrize("exchange", ["records", "partials"])
@pytest.mark.parametrize("pipeline", [False, "stream"])
def test_window_batches_outgrow_capacity_unevenly(dev, world, exchange, pipeline):
    """Ranks' batches pass the (small) batch capacity at different steps: the regrow is agreed
    through the step's reduced vector (every rank regrows to the largest batch and redoes the
    step), so the ranks keep one bucket geometry and one collective sequence; a single rank
    drains its queued state half before its buffers are reallocated. Equal to one process."""
    _skip_no_gpu(dev)
    per, nkeys, cap_log2 = _sizes(dev)
    sizes = [[per // 8 * (1 + ((s + r) % 4) * (r + 1)) for s in range(STEPS)] for r in range(world)]

    def make(comm, pipe=pipeline):
        return KeyedWindowOperator(size=3000, slide=1000, lateness=1500, agg=K.AGG_SUM_I64,
                                   device=dev, comm=comm, max_keys=nkeys, batch_capacity=per // 8,
                                   ooo_bound=500, cap_log2=cap_log2, pipeline=pipe,
                                   exchange=exchange)

    def batch(rank, step):
        k, t, v = _batch(dev, rank, step, per, nkeys, late=2000)
        n = sizes[rank][step]
        t = t[:n].contiguous()
        t[-1] = step * 2000 + 2000  # every rank's batch ends at the same event time (see _batch)
        return k[:n].contiguous(), t, v[:n].contiguous()

    def rank_fn(comm):
        op = make(comm)
        out = []
        for step in range(STEPS):
            out += op.process(*batch(comm.rank, step))
        out += op.finish()
        return _collect(out), op.metrics.num_late_records_dropped

    res = run_loopback(world, rank_fn, device=torch.device(dev))
    merged, late = {}, 0
    for d, nl in res:
        merged.update(d)
        late += nl
    ref_op = make(None, pipe=False)
    out = []
    for step in range(STEPS):
        parts = [batch(r, step) for r in range(world)]
        out += ref_op.process(*[torch.cat([p[i] for p in parts]) for i in range(3)])
    out += ref_op.finish()
    assert len(_collect(out)) > 0
    assert merged == _collect(out)
    assert late == ref_op.metrics.num_late_records_dropped


def test_loopback_collective_mismatch_is_reported():
    """A rank that enters a different collective than its peers fails every rank with a message
    naming what each rank entered (instead of pairing unrelated buffers or hanging)."""
    def fn(comm):
        t = torch.zeros(4, dtype=torch.int64)
        if comm.rank == 0:
            comm.allreduce_min_(t)
        else:
            comm.all_to_all(torch.empty_like(t), t)

    with pytest.raises(RuntimeError, match="loopback collective mismatch"):
        run_loopback(2, fn, timeout_s=30)


def test_loopback_collectives_match_in_order():
    """Equal collective sequences pass the check (including barriers and object gathers)."""
    def fn(comm):
        t = torch.full((4,), comm.rank, dtype=torch.int64)
        comm.allreduce_min_(t)
        comm.barrier()
        got = comm.all_gather_object(comm.rank)
        inp = torch.full((4,), comm.rank, dtype=torch.int64)
        out = torch.empty_like(inp)
        comm.all_to_all(out, inp)
        return int(t[0]), got, out.tolist()

    res = run_loopback(2, fn, timeout_s=30)
    assert res[0][0] == res[1][0] == 0 and res[0][1] == [0, 1]
    assert res[1][2] == [0, 0, 1, 1]
