"""KeyedWindowOperator (C++ twin path) vs the Flink-semantics oracle on random streams."""
import random

import numpy as np
import pytest
import torch

from mxstream.ops import expr as E
from mxstream.ops import kernels as K
from mxstream.oracle.flink import BoundedOutOfOrderness, WindowOracle
from mxstream.runtime.window_operator import KeyedWindowOperator


def _run_engine(batches, *, size, slide, lateness, bound, agg, max_keys=4096, cap_log2=8):
    op = KeyedWindowOperator(size=size, slide=slide, lateness=lateness, agg=agg, device="cpu",
                             max_keys=max_keys, batch_capacity=256, cap_log2=cap_log2,
                             ooo_bound=bound)
    out = []
    for keys, ts, vals in batches:
        out += op.process(torch.tensor(keys, dtype=torch.int64), torch.tensor(ts, dtype=torch.int64),
                          torch.tensor(vals, dtype=torch.int64))
    out += op.finish()
    last = {}
    for r in out:
        for k, v, raw, c in zip(r.keys.tolist(), r.values.tolist(), r.raw.tolist(), r.counts.tolist()):
            last[((r.window_start, r.window_end), k)] = (raw, c, v)
    return last, op


def _run_oracle(batches, *, size, slide, lateness, bound):
    orc = WindowOracle(size=size, slide=slide, lateness=lateness,
                       add=lambda acc, v: (v, 1) if acc is None else (acc[0] + v, acc[1] + 1))
    wm = BoundedOutOfOrderness(bound)
    last = {}

    def rec(ems):
        for e in ems:
            last[(e.window, e.key)] = e.value

    for keys, ts, vals in batches:
        for k, t, v in zip(keys, ts, vals):
            rec(orc.element(k, t, v))
            wm.observe(t)
        rec(orc.watermark(wm.current_watermark()))
    rec(orc.watermark((1 << 63) - 1))
    return last, orc


def _random_batches(seed, nbatches, per, nkeys, t0, dt, disorder, late_frac=0.0):
    rnd = random.Random(seed)
    t = t0
    out = []
    for _ in range(nbatches):
        keys, ts, vals = [], [], []
        for _ in range(per):
            t += rnd.randint(0, dt)
            tt = t - rnd.randint(0, disorder)
            if rnd.random() < late_frac:
                tt -= rnd.randint(0, 5 * disorder + 1)
            keys.append(rnd.randrange(nkeys))
            ts.append(tt)
            vals.append(rnd.randint(0, 1000))
        out.append((keys, ts, vals))
    return out


@pytest.mark.parametrize("size,slide,lateness,bound", [
    (1000, 1000, 0, 200),     # tumbling
    (1000, 250, 0, 300),      # sliding
    (3000, 1000, 500, 400),   # sliding + allowed lateness
    (600, 600, 1200, 100),    # tumbling + lateness larger than the window
])
@pytest.mark.parametrize("seed", [1, 2])
def test_window_sum_matches_oracle(size, slide, lateness, bound, seed):
    batches = _random_batches(seed, 12, 80, 37, 10_000, 40, 300, late_frac=0.1)
    got, op = _run_engine(batches, size=size, slide=slide, lateness=lateness, bound=bound,
                          agg=K.AGG_SUM_I64)
    exp, orc = _run_oracle(batches, size=size, slide=slide, lateness=lateness, bound=bound)
    assert set(got) == set(exp)
    for kw, (s, c) in exp.items():
        raw, cnt, _ = got[kw]
        assert (raw, cnt) == (s, c), kw
    assert op.metrics.num_late_records_dropped == orc.late_dropped


def test_window_count_and_avg():
    batches = _random_batches(5, 6, 50, 9, 0, 30, 100)
    got, _ = _run_engine(batches, size=500, slide=500, lateness=0, bound=100, agg=K.AGG_AVG_I64)
    exp, _ = _run_oracle(batches, size=500, slide=500, lateness=0, bound=100)
    for kw, (s, c) in exp.items():
        raw, cnt, val = got[kw]
        assert cnt == c and raw == s
        assert val == pytest.approx(s / c)


def test_epilogue_map_filter():
    from mxstream.ops import expr as E

    batches = _random_batches(7, 5, 60, 11, 0, 20, 50)
    m = E.compile_expr(E.var(E.VAR_RESULT) * 8.0 / 60 / 1024 / 1024)
    f = E.compile_expr(E.var(E.VAR_MAPPED) < 0.004)
    op = KeyedWindowOperator(size=400, agg=K.AGG_SUM_I64, device="cpu", max_keys=128,
                             batch_capacity=128, cap_log2=6, ooo_bound=50, map_prog=m,
                             filter_prog=f)
    out = []
    for keys, ts, vals in batches:
        out += op.process(torch.tensor(keys), torch.tensor(ts), torch.tensor(vals))
    out += op.finish()
    exp, _ = _run_oracle(batches, size=400, slide=400, lateness=0, bound=50)
    want = {kw: s * 8.0 / 60 / 1024 / 1024 for kw, (s, c) in exp.items()
            if s * 8.0 / 60 / 1024 / 1024 < 0.004}
    got = {}
    for r in out:
        for k, v in zip(r.keys.tolist(), r.values.tolist()):
            got[((r.window_start, r.window_end), k)] = v
    assert got == want  # bit-exact Java double semantics


def test_ring_growth_on_event_time_jump():
    batches = [([1, 2], [0, 10], [1, 1]), ([1], [10_000_000], [5]), ([2], [10_000_050], [7])]
    got, op = _run_engine(batches, size=100, slide=100, lateness=0, bound=0, agg=K.AGG_SUM_I64)
    assert got[((0, 100), 1)][:2] == (1, 1)
    assert got[((10_000_000, 10_000_100), 1)][:2] == (5, 1)
    assert got[((10_000_000, 10_000_100), 2)][:2] == (7, 1)


@pytest.mark.parametrize("agg", [K.AGG_SUM_I64, K.AGG_MAX_I64, K.AGG_COUNT, K.AGG_AVG_I64])
def test_compact_records_equal_wide(agg):
    """16-byte records (int32 values) give the same windows as 24-byte records; a value outside
    int32 switches the operator to 24-byte records and redoes the step."""
    rng = np.random.default_rng(2)
    res = {}
    for compact in (False, True):
        op = KeyedWindowOperator(size=2000, slide=1000, lateness=500, agg=agg, device="cpu",
                                 max_keys=4096, batch_capacity=4096, cap_log2=8, ooo_bound=300,
                                 compact=compact)
        out = []
        for step in range(6):
            k = torch.from_numpy(rng.integers(0, 500, 2000) if compact else
                                 np.random.default_rng(10 + step).integers(0, 500, 2000))
            t = torch.from_numpy(np.random.default_rng(20 + step).integers(step * 900,
                                                                          step * 900 + 1500, 2000))
            v = torch.from_numpy(np.random.default_rng(30 + step).integers(-5000, 5000, 2000))
            k = torch.from_numpy(np.random.default_rng(10 + step).integers(0, 500, 2000))
            out += op.process(k, t, v)
        out += op.finish()
        res[compact] = sorted((r.window_start, int(kk), int(a), int(c), r.refire)
                              for r in out for kk, a, c in zip(r.keys, r.raw, r.counts))
        assert op.compact == compact
    assert res[True] == res[False]
    op = KeyedWindowOperator(size=2000, agg=K.AGG_SUM_I64, device="cpu", max_keys=64,
                             batch_capacity=64, cap_log2=6, compact=True)
    op.process(torch.tensor([1, 2]), torch.tensor([10, 20]), torch.tensor([5, 1 << 40]))
    assert op.compact is False and op.metrics.extra["compact_fallbacks"] == 1
    fired = op.finish()
    got = {int(k): int(a) for r in fired for k, a in zip(r.keys, r.raw)}
    assert got == {1: 5, 2: 1 << 40}


def test_pinned_slab_pool_reuses_only_released_slabs():
    """The fire D2H slab pool (window_operator.PinnedSlabPool) never hands out a slab whose rows a
    caller still holds, and reuses it once they are dropped (pin=False: same logic on CPU)."""
    import numpy as np

    from mxstream.runtime.window_operator import PinnedSlabPool

    pool = PinnedSlabPool(pin=False, max_slabs=2)
    t1, a1 = pool.take(1000)
    held = a1[0:64].view(np.int64)
    del t1, a1
    t2, a2 = pool.take(1000)
    assert pool.allocs == 2  # first slab still referenced through `held`
    del t2, a2
    del held
    pool.take(1000)
    assert pool.allocs == 2  # released slab reused
    big = pool.take(1 << 20)
    assert big[0].numel() >= 1 << 20 and pool.allocs == 3 and len(pool.slabs) <= 2


@pytest.mark.parametrize("big", ["none", "value", "key", "int32"])
def test_narrow_records_match_wide(big):
    """8-byte records (32-bit key, 28-bit value, 4-bit pane) on the C++ twin give the same
    windows as 24-byte records; a key or value that does not fit widens the format (16-byte,
    or 24-byte for a value outside int32) and redoes the step."""
    import torch

    from mxstream.ops import kernels as K
    from mxstream.runtime.window_operator import KeyedWindowOperator

    def run(narrow):
        op = KeyedWindowOperator(size=2000, slide=1000, agg=K.AGG_SUM_I64, device="cpu",
                                 max_keys=4000, batch_capacity=5000, ooo_bound=300, cap_log2=8,
                                 compact=narrow, narrow=narrow)
        out = []
        for step in range(6):
            k = torch.empty(5000, dtype=torch.int64)
            t = torch.empty_like(k)
            v = torch.empty_like(k)
            K.gen_events(k, t, v, seed=9, stream_id=0, idx0=step * 5000, nkeys=3000,
                         ts_base=step * 1000, ts_span=1000, disorder=300, val_lo=-500,
                         val_span=1000)
            if step == 3 and big == "value":
                v[7] = 1 << 29
            if step == 3 and big == "key":
                k[7] = (1 << 32) + 5
            if step == 3 and big == "int32":
                v[7] = 1 << 40
            out += op.process(k, t, v)
        out += op.finish()
        return ({(r.window_start, int(a), int(b), int(c))
                 for r in out for a, b, c in zip(r.keys, r.raw, r.counts)}, op.rec_w)

    wide, rw_wide = run(False)
    nar, rw_nar = run(True)
    assert rw_wide == 3
    assert rw_nar == {"none": 1, "value": 2, "key": 2, "int32": 3}[big]
    assert nar == wide


@pytest.mark.parametrize("size,slide,lateness", [(2000, 2000, 0), (3000, 1000, 1500)])
def test_dense_keys_match_hashed(size, slide, lateness):
    """dense_keys=True (ids < max_keys directly addressed through a bijective slot map, no
    hash-table probe) fires exactly the windows of the hashed tables; an id outside the dense
    key space reports a full table."""
    import torch

    from mxstream.ops import kernels as K
    from mxstream.runtime.window_operator import KeyedWindowOperator

    def run(dense, bad=False):
        op = KeyedWindowOperator(size=size, slide=slide, lateness=lateness, agg=K.AGG_SUM_I64,
                                 device="cpu", max_keys=3000, batch_capacity=5000, ooo_bound=300,
                                 dense_keys=dense, cap_log2=8)
        out = []
        for step in range(7):
            k = torch.empty(5000, dtype=torch.int64)
            t = torch.empty_like(k)
            v = torch.empty_like(k)
            K.gen_events(k, t, v, seed=13, stream_id=0, idx0=step * 5000, nkeys=3000,
                         ts_base=step * 1000, ts_span=1000, disorder=400, val_lo=0, val_span=1000)
            if step > 3:
                t[:200] -= 1200
            if bad and step == 2:
                k[3] = 1 << 20
            out += op.process(k, t, v)
        out += op.finish()
        assert not dense or op.num_keys() >= 0
        return sorted((r.window_start, r.refire, int(a), int(b), int(c))
                      for r in out for a, b, c in zip(r.keys, r.raw, r.counts))

    assert run(True) == run(False)
    with pytest.raises(RuntimeError, match="table full"):
        run(True, bad=True)


@pytest.mark.parametrize("dense", [True, False])
def test_int32_key_ids_match_int64(dense):
    """An int32 key column (dictionary ids, as the columnar sources produce) fires exactly what
    the same ids as int64 fire; -1 stays a reserved id after the sign extension."""
    import torch

    from mxstream.ops import kernels as K
    from mxstream.runtime.window_operator import KeyedWindowOperator

    def run(dtype, bad=False):
        op = KeyedWindowOperator(size=2000, slide=1000, lateness=500, agg=K.AGG_SUM_I64,
                                 device="cpu", max_keys=3000, batch_capacity=5000, ooo_bound=300,
                                 dense_keys=dense, cap_log2=8)
        out = []
        for step in range(6):
            k = torch.empty(5000, dtype=dtype)
            t = torch.empty(5000, dtype=torch.int64)
            v = torch.empty_like(t)
            K.gen_events(k, t, v, seed=3, stream_id=0, idx0=step * 5000, nkeys=3000,
                         ts_base=step * 1000, ts_span=1000, disorder=400, val_lo=0, val_span=1000)
            if bad and step == 2:
                k[7] = -1
            out += op.process(k, t, v)
        out += op.finish()
        return sorted((r.window_start, r.refire, int(a), int(b), int(c))
                      for r in out for a, b, c in zip(r.keys, r.raw, r.counts))

    assert run(torch.int32) == run(torch.int64)
    with pytest.raises(ValueError, match="reserved"):
        run(torch.int32, bad=True)


def _f64_batches(n, steps, seed):
    import torch

    rng = np.random.default_rng(seed)
    out = []
    for step in range(steps):
        k = torch.from_numpy(rng.integers(0, 500, n).astype(np.int64))
        t = torch.from_numpy((step * 1000 + rng.integers(0, 1000, n)).astype(np.int64))
        # wide dynamic range: rounding order matters for plain f64 sums
        v = rng.standard_normal(n) * 10.0 ** rng.integers(-6, 9, n)
        out.append((k, t, torch.from_numpy(v).view(torch.int64)))
    return out


@pytest.mark.parametrize("agg_name", ["sum", "avg"])
def test_deterministic_f64_sums_order_independent(agg_name):
    """deterministic=True: permuting the records of every batch leaves every fired f64 sum
    bit-identical (128-bit fixed-point slot sums), and the sums equal math.fsum up to the final
    conversion."""
    import math

    import torch

    from mxstream.ops import kernels as K
    from mxstream.runtime.window_operator import KeyedWindowOperator

    agg = K.AGG_SUM_F64 if agg_name == "sum" else K.AGG_AVG_F64
    batches = _f64_batches(4000, 5, 3)

    def run(perm_seed):
        op = KeyedWindowOperator(size=2000, agg=agg, device="cpu", max_keys=600,
                                 batch_capacity=4000, ooo_bound=0, deterministic=True, cap_log2=8)
        rows = {}
        rng = np.random.default_rng(perm_seed)
        for k, t, v in batches:
            p = torch.from_numpy(rng.permutation(k.numel())) if perm_seed else torch.arange(k.numel())
            for r in op.process(k[p], t[p], v[p]):
                for key, raw in zip(r.keys.tolist(), r.raw.tolist()):
                    rows[(r.window_start, key)] = raw
        for r in op.finish():
            for key, raw in zip(r.keys.tolist(), r.raw.tolist()):
                rows[(r.window_start, key)] = raw
        return rows

    a, b = run(0), run(7)
    assert a == b and len(a) > 100
    # spot-check against an exact sum of one window/key
    (ws, key), raw = next(iter(sorted(a.items())))
    vals = []
    for k, t, v in batches:
        sel = (k == key) & (t >= ws) & (t < ws + 2000)
        vals += v[sel].view(torch.float64).tolist()
    got = float(np.int64(raw).view(np.float64))
    assert abs(got - math.fsum(vals)) <= 1e-9 * max(1.0, abs(math.fsum(vals)))


def _drift_batches(steps, n, seed=9):
    """Keys drift over time (1500 new ids per step) plus 50 hot ids: many more distinct keys
    than the table holds, most of them cold after a few steps."""
    import torch

    rng = np.random.default_rng(seed)
    out = []
    for step in range(steps):
        k = np.where(rng.random(n) < 0.1, rng.integers(0, 50, n),
                     1000 + step * 1500 + rng.integers(0, 2000, n)).astype(np.int64)
        t = (step * 1000 + rng.integers(0, 1000, n)).astype(np.int64)
        t[rng.random(n) < 0.03] -= 2500  # late, within the allowed lateness
        v = rng.integers(0, 1000, n).astype(np.int64)
        out.append((torch.from_numpy(k), torch.from_numpy(t), torch.from_numpy(v)))
    return out


def _run_windows(batches, **kw):
    from mxstream.ops import expr as E
    from mxstream.ops import kernels as K
    from mxstream.runtime.window_operator import KeyedWindowOperator

    op = KeyedWindowOperator(size=6000, slide=2000, lateness=3000, agg=K.AGG_SUM_I64,
                             device=kw.pop("device", "cpu"), batch_capacity=6000, ooo_bound=500,
                             map_prog=E.compile_expr(E.var(E.VAR_RESULT) * 0.5),
                             filter_prog=E.compile_expr(E.var(E.VAR_COUNT) > 1), **kw)
    rows = []
    for k, t, v in batches:
        rows += op.process(k.to(op.device), t.to(op.device), v.to(op.device))
    rows += op.finish()
    got = sorted((r.window_start, r.refire, int(a), int(b), int(c), float(x))
                 for r in rows for a, b, c, x in zip(r.keys, r.raw, r.counts, r.values))
    return got, op


def test_spill_tier_matches_unbounded_table():
    """A hashed-key table far smaller than the key space: window_compact drops keys without
    live data and moves cold keys' live panes to the host tier; every firing and late re-firing
    (device part + host part, epilogue on the host) equals a table that holds every key."""
    batches = _drift_batches(26, 6000)  # ~40K distinct keys over a 32K-slot table
    ref, _ = _run_windows(batches, max_keys=80_000)
    got, op = _run_windows(batches, max_keys=3000, spill=True, spill_check_steps=1,
                           spill_load=0.5, cap_log2=7, spill_keep_panes=1)
    ex = op.metrics.extra
    assert ex.get("spilled_keys", 0) > 0 and ex.get("spilled_rows", 0) > 0
    assert got == ref
    import pytest as _pt

    with _pt.raises(RuntimeError, match="table full"):
        _run_windows(batches, max_keys=3000, cap_log2=7)


def test_spill_tier_checkpoint_roundtrip():
    """Spilled state is part of the snapshot; a restored operator fires the same windows."""
    batches = _drift_batches(12, 6000, seed=4)
    ref, _ = _run_windows(batches, max_keys=60_000)
    from mxstream.ops import expr as E
    from mxstream.ops import kernels as K
    from mxstream.runtime.window_operator import KeyedWindowOperator

    def make():
        return KeyedWindowOperator(size=6000, slide=2000, lateness=3000, agg=K.AGG_SUM_I64,
                                   device="cpu", batch_capacity=6000, ooo_bound=500,
                                   map_prog=E.compile_expr(E.var(E.VAR_RESULT) * 0.5),
                                   filter_prog=E.compile_expr(E.var(E.VAR_COUNT) > 1),
                                   max_keys=3000, spill=True, spill_check_steps=1,
                                   spill_load=0.5, cap_log2=7, spill_keep_panes=1)

    op = make()
    rows = []
    for k, t, v in batches[:7]:
        rows += op.process(k, t, v)
    rows += op.flush()
    assert op.host_state_bytes() > 0
    snap = op.snapshot_state()
    op2 = KeyedWindowOperator(size=6000, slide=2000, lateness=3000, agg=K.AGG_SUM_I64,
                              device="cpu", batch_capacity=6000, ooo_bound=500,
                              map_prog=E.compile_expr(E.var(E.VAR_RESULT) * 0.5),
                              filter_prog=E.compile_expr(E.var(E.VAR_COUNT) > 1),
                              max_keys=60_000)
    op2.restore_state(snap.columns, snap.meta)
    for k, t, v in batches[7:]:
        rows += op2.process(k, t, v)
    rows += op2.finish()
    got = sorted((r.window_start, r.refire, int(a), int(b), int(c), float(x))
                 for r in rows for a, b, c, x in zip(r.keys, r.raw, r.counts, r.values))
    assert got == ref


def test_compact_state_drops_dead_keys():
    """compact_state() without a cutoff (no spill tier): keys with no data in the live panes are
    dropped and the kept keys rehashed; later firings are unchanged."""
    batches = _drift_batches(10, 6000, seed=2)
    ref, _ = _run_windows(batches, max_keys=60_000)
    from mxstream.ops import expr as E
    from mxstream.ops import kernels as K
    from mxstream.runtime.window_operator import KeyedWindowOperator

    op = KeyedWindowOperator(size=6000, slide=2000, lateness=3000, agg=K.AGG_SUM_I64,
                             device="cpu", batch_capacity=6000, ooo_bound=500,
                             map_prog=E.compile_expr(E.var(E.VAR_RESULT) * 0.5),
                             filter_prog=E.compile_expr(E.var(E.VAR_COUNT) > 1), max_keys=60_000)
    rows = []
    dropped = 0
    for i, (k, t, v) in enumerate(batches):
        rows += op.process(k, t, v)
        if i % 3 == 2:
            rows += op.flush()
            before = int((op.keys_g != -1).sum())
            dropped += op.compact_state()["dropped"]
            assert int((op.keys_g != -1).sum()) <= before
    rows += op.finish()
    got = sorted((r.window_start, r.refire, int(a), int(b), int(c), float(x))
                 for r in rows for a, b, c, x in zip(r.keys, r.raw, r.counts, r.values))
    assert dropped > 0 and got == ref


def _spill_op(**kw):
    from mxstream.ops import expr as E
    from mxstream.ops import kernels as K
    from mxstream.runtime.window_operator import KeyedWindowOperator

    args = dict(size=6000, slide=2000, lateness=3000, agg=K.AGG_SUM_I64, device="cpu",
                batch_capacity=6000, ooo_bound=500,
                map_prog=E.compile_expr(E.var(E.VAR_RESULT) * 0.5),
                filter_prog=E.compile_expr(E.var(E.VAR_COUNT) > 1))
    args.update(kw)
    return KeyedWindowOperator(**args)


def _rows_key(rows):
    return sorted((r.window_start, r.refire, int(a), int(b), int(c), float(x))
                  for r in rows for a, b, c, x in zip(r.keys, r.raw, r.counts, r.values))


def test_spill_checkpoint_restores_into_the_small_table():
    """A checkpoint taken with more keys than the table holds restores into an operator with the
    same small table: cold keys return to the host tier, the rest are inserted."""
    batches = _drift_batches(12, 6000, seed=4)
    ref, _ = _run_windows(batches, max_keys=60_000)
    small = dict(max_keys=3000, spill=True, spill_check_steps=1, spill_load=0.5, cap_log2=7,
                 spill_keep_panes=1)
    op = _spill_op(**small)
    rows = []
    for k, t, v in batches[:7]:
        rows += op.process(k, t, v)
    rows += op.flush()
    snap = op.snapshot_state()
    assert len(np.unique(snap.columns["key"])) > op.nslots  # more keys than slots
    op2 = _spill_op(**small)
    op2.restore_state(snap.columns, snap.meta)
    assert op2.host_state_bytes() > 0
    for k, t, v in batches[7:]:
        rows += op2.process(k, t, v)
    rows += op2.finish()
    assert _rows_key(rows) == ref


def test_async_snapshot_with_spill_is_isolated_from_later_evictions():
    """The async export reads a private copy of the spill tier: evictions between the freeze and
    the export neither lose rows nor export them twice (restore equals a synchronous snapshot)."""
    batches = _drift_batches(10, 6000, seed=5)
    small = dict(max_keys=3000, spill=True, spill_check_steps=1, spill_load=0.5, cap_log2=7,
                 spill_keep_panes=1)
    op = _spill_op(**small)
    for k, t, v in batches[:6]:
        op.process(k, t, v)
    op.flush()
    sync = op.snapshot_state()
    run = op.snapshot_state_async()
    op.compact_state(op.max_seen_pane - 1)  # evicts more keys into the live tier
    frozen = run()

    def canon(snap):
        c = snap.columns
        df = {}
        for key, pane, acc, cnt in zip(c["key"].tolist(), c["pane"].tolist(), c["acc"].tolist(),
                                       c["cnt"].tolist()):
            a0, c0 = df.get((key, pane), (0, 0))
            df[(key, pane)] = (a0 + acc, c0 + cnt)
        return df

    assert canon(frozen) == canon(sync)


@pytest.mark.parametrize("size,slide,lateness", [(2000, 2000, 0), (6000, 1000, 3000)])
def test_key_value_rows_equal_full_rows(size, slide, lateness):
    """emit="key_value" (12-byte fired rows: uint32 key id + mapped value) fires the same
    (window, key, value) rows as the full 28-byte rows, single and batched firings alike."""
    prog = E.compile_expr(E.var(E.VAR_RESULT) * 0.5)

    def run(emit):
        op = KeyedWindowOperator(size=size, slide=slide, lateness=lateness, agg=K.AGG_SUM_I64,
                                 device="cpu", max_keys=3000, batch_capacity=5000, ooo_bound=300,
                                 dense_keys=True, cap_log2=8, map_prog=prog, emit=emit)
        out = []
        for step in range(9):
            k = torch.empty(5000, dtype=torch.int64)
            t = torch.empty_like(k)
            v = torch.empty_like(k)
            K.gen_events(k, t, v, seed=17, stream_id=0, idx0=step * 5000, nkeys=3000,
                         ts_base=step * 1000 + (4000 if step == 5 else 0), ts_span=1000,
                         disorder=400, val_lo=0, val_span=1000)
            if step > 3:
                t[:200] -= 1500
            out += op.process(k, t, v)
        out += op.finish()
        if emit == "key_value":
            assert all(r.raw is None and r.counts is None and r.keys.dtype == np.uint32
                       for r in out)
        return sorted((r.window_start, r.refire, int(a), float(b))
                      for r in out for a, b in zip(r.keys, r.values))

    full = run("full")
    assert len(full) > 1000
    assert run("key_value") == full


@pytest.mark.parametrize("n", [4000, 250_000])
def test_cxx_window_tier_equals_numpy_combine(n):
    """csrc/window_tier.h: chunked absorb, per-key part() and the tiered merge_fire equal the
    numpy combine of the same rows; purge drops exactly the rows below the cutoff. n = 250K rows
    per eviction takes merge_fire's threaded radix-partitioned aggregation (256 partitions)."""
    from mxstream.runtime.window_spill import HostWindowTier, combine_rows, merge_fire

    rng = np.random.default_rng(4)
    t = HostWindowTier(K.AGG_SUM_I64)
    cols = {k: [] for k in ("key", "pane", "acc", "cnt", "dirty")}
    nkeys = n * 3 // 4
    for _ in range(5):  # evictions -> chunks (a key may be evicted twice)
        c = {"key": rng.integers(0, nkeys, n).astype(np.uint64),
             "pane": rng.integers(10, 20, n).astype(np.int64),
             "acc": rng.integers(-1000, 1000, n).astype(np.int64),
             "cnt": rng.integers(1, 5, n).astype(np.int64),
             "dirty": rng.integers(0, 2, n).astype(np.uint8)}
        t.absorb(c["key"], c["pane"], c["acc"], c["cnt"], c["dirty"])
        for k in cols:
            cols[k].append(c[k])
    cols = {k: np.concatenate(v) for k, v in cols.items()}
    assert t.nrows == cols["key"].size and t.pane_range() == (10, 19)
    sel = (cols["pane"] >= 12) & (cols["pane"] <= 15)
    k, a, c = t.part(12, 15)
    ek, ea, ec = combine_rows(K.AGG_SUM_I64, cols["key"][sel], cols["acc"][sel], cols["cnt"][sel])
    assert np.array_equal(k, ek) and np.array_equal(a, ea) and np.array_equal(c, ec)
    dk = np.arange(0, nkeys + nkeys // 6, 7, dtype=np.uint64)
    dr = rng.integers(0, 100, dk.size).astype(np.int64)
    dc = np.ones(dk.size, np.int64)
    for only in (False, True):
        got = merge_fire(K.AGG_SUM_I64, dk, dr, dc, t, only, E.EMPTY, E.EMPTY, 0, 1,
                         panes=(12, 15))
        ref = merge_fire(K.AGG_SUM_I64, dk, dr, dc, (k, a, c), only, E.EMPTY, E.EMPTY, 0, 1)
        o1, o2 = np.argsort(got[0]), np.argsort(ref[0])
        for x, y in zip(got, ref):
            assert np.array_equal(np.asarray(x)[o1], np.asarray(y)[o2])
    # purge(12): a fifth of every chunk is below -- marked dead, not copied (lazy purge); every
    # reader skips the dead rows
    before = merge_fire(K.AGG_SUM_I64, dk, dr, dc, t, False, E.EMPTY, E.EMPTY, 0, 1,
                        panes=(12, 15))
    t.purge(12)
    assert t.nrows == int((cols["pane"] >= 12).sum()) and t.pane_range() == (12, 19)
    r = t.copy().rows()  # (rows() merges the tier into one chunk: read a copy)
    assert int(r["cnt"].sum()) == int(cols["cnt"][cols["pane"] >= 12].sum())
    assert int(r["pane"].min()) == 12
    after = merge_fire(K.AGG_SUM_I64, dk, dr, dc, t, False, E.EMPTY, E.EMPTY, 0, 1,
                       panes=(12, 15))
    o1, o2 = np.argsort(before[0]), np.argsort(after[0])
    for x, y in zip(before, after):
        assert np.array_equal(np.asarray(x)[o1], np.asarray(y)[o2])
    t.purge(15)
    assert t.nrows == int((cols["pane"] >= 15).sum()) and t.pane_range() == (15, 19)
    r = t.rows()
    assert int(r["cnt"].sum()) == int(cols["cnt"][cols["pane"] >= 15].sum())


@pytest.mark.parametrize("piece", [1, 777, 40_000, 10**6])
def test_cxx_window_tier_export_window_pieces(piece):
    """export_window (the GPU export's pieces through a ring of fixed pinned slabs) concatenated
    over [0, total) equals export_rows in the same order -- pane-sorted chunks and a chunk whose
    pane span is too wide to sort (filtered row by row), with a purged (dead) prefix."""
    from mxstream.ops.native import load

    rng = np.random.default_rng(9)
    t = load().WindowTier(K.AGG_SUM_I64)
    for _ in range(3):
        n = 30_000
        t.absorb(rng.integers(0, 50_000, n).astype(np.uint64), rng.integers(10, 20, n),
                 rng.integers(-9, 9, n), rng.integers(1, 4, n), np.zeros(n, np.uint8))
    n = 5_000  # pane span >= 2^20: kept unsorted
    pane = rng.integers(10, 20, n)
    pane[0] = 10 + (1 << 21)
    t.absorb(rng.integers(0, 50_000, n).astype(np.uint64), pane, rng.integers(-9, 9, n),
             rng.integers(1, 4, n), np.zeros(n, np.uint8))
    t.purge(12)
    cap = t.nrows
    k, a, c = np.empty(cap, np.uint64), np.empty(cap, np.int64), np.empty(cap, np.uint32)
    total = t.export_rows(12, 17, k.ctypes.data, a.ctypes.data, c.ctypes.data, cap)
    assert 0 < total <= cap
    parts = [[], [], []]
    r = 0
    while r < total:
        pk, pa, pc = np.empty(piece, np.uint64), np.empty(piece, np.int64), np.empty(piece, np.uint32)
        assert t.export_window(12, 17, pk.ctypes.data, pa.ctypes.data, pc.ctypes.data, r,
                               piece) == total
        m = min(piece, total - r)
        for lst, arr in zip(parts, (pk, pa, pc)):
            lst.append(arr[:m])
        r += m
    for whole, lst in zip((k, a, c), parts):
        assert np.array_equal(whole[:total], np.concatenate(lst))


def test_cxx_window_tier_purge_never_rewinds():
    """A purge with a cutoff below an earlier purge's (15, then 12) leaves the tier as the first
    purge left it: dead rows stay dead, counts do not wrap (csrc/window_tier.h purge)."""
    from mxstream.runtime.window_spill import HostWindowTier

    rng = np.random.default_rng(9)
    t = HostWindowTier(K.AGG_SUM_I64)
    n = 5000
    pane = rng.integers(10, 20, n).astype(np.int64)
    cnt = rng.integers(1, 5, n).astype(np.int64)
    t.absorb(rng.integers(0, 3000, n).astype(np.uint64), pane,
             rng.integers(-9, 9, n).astype(np.int64), cnt, np.zeros(n, np.uint8))
    t.purge(13)  # lazy: below 13 is less than half -> rows marked dead
    keep = int((pane >= 13).sum())
    assert t.nrows == keep
    t.purge(12)
    assert t.nrows == keep and t.pane_range() == (13, 19)
    r = t.copy().rows()
    assert int(r["pane"].min()) == 13 and int(r["cnt"].sum()) == int(cnt[pane >= 13].sum())
    t.purge(17)  # filter branch (more than half below)
    t.purge(15)
    assert t.nrows == int((pane >= 17).sum())
    r = t.rows()
    assert int(r["pane"].min()) == 17 and int(r["cnt"].sum()) == int(cnt[pane >= 17].sum())


def test_cxx_window_tier_export_segments():
    """export_rows (the device-merged tiered firing's upload): pane-sorted chunks give one
    contiguous segment each, a chunk spanning >= 2^20 panes is filtered row by row; the exported
    (key, acc, cnt) multiset equals the live rows of the panes, before and after purges, and
    zero-count rows never leave the tier."""
    from mxstream.runtime.window_spill import HostWindowTier

    rng = np.random.default_rng(11)
    t = HostWindowTier(K.AGG_SUM_I64)
    cols = {k: [] for k in ("key", "pane", "acc", "cnt")}
    for j in range(6):
        n = 300_000 if j % 2 else 7000
        pane = rng.integers(10, 22, n).astype(np.int64)
        if j == 5:
            pane[0] = 10 + (1 << 21)  # one far pane: this chunk stays unsorted
        c = {"key": rng.integers(0, 1 << 40, n).astype(np.uint64), "pane": pane,
             "acc": rng.integers(-1000, 1000, n).astype(np.int64),
             "cnt": rng.integers(0, 4, n).astype(np.int64)}
        t.absorb(c["key"], c["pane"], c["acc"], c["cnt"], np.zeros(n, np.uint8))
        for k in cols:
            cols[k].append(c[k])
    cols = {k: np.concatenate(v) for k, v in cols.items()}

    def check(p0, p1, live_from):
        got = t.export(p0, p1, "cpu")
        sel = ((cols["pane"] >= max(p0, live_from)) & (cols["pane"] <= p1) & (cols["cnt"] > 0))
        if got is None:
            assert not sel.any()
            return
        k, a, c, n, _ = got
        assert n == int(sel.sum())
        want = np.stack([cols["key"][sel].view(np.int64), cols["acc"][sel], cols["cnt"][sel]], 1)
        have = np.stack([k.numpy(), a.numpy(), c.numpy().astype(np.int64)], 1)
        want = want[np.lexsort(want.T[::-1])]
        have = have[np.lexsort(have.T[::-1])]
        assert np.array_equal(want, have)

    check(12, 17, 0)
    check(0, 1 << 30, 0)
    t.purge(14)
    check(12, 17, 14)
    check(20, 21, 14)
    t.purge(21)
    check(0, 1 << 30, 21)
    # (the unsorted chunk -- the last 300K rows -- keeps its zero-count rows)
    unsorted = np.arange(cols["pane"].size) >= cols["pane"].size - 300_000
    assert t.nrows == int(((cols["pane"] >= 21) & ((cols["cnt"] > 0) | unsorted)).sum())


def test_cxx_window_tier_presorted_absorb_equals_sort():
    """absorb_presorted (rows grouped by pane on the device) builds the same tier as absorb's
    host counting sort of the same rows: same rows(), same exports, same purges."""
    from mxstream.runtime.window_spill import HostWindowTier

    rng = np.random.default_rng(12)
    a, b = HostWindowTier(K.AGG_SUM_I64), HostWindowTier(K.AGG_SUM_I64)
    c3 = HostWindowTier(K.AGG_SUM_I64)  # background absorbs, purges deferred to the join
    for j in range(4):
        n = 200_000 if j % 2 else 3000
        p_lo, np_ = 20 + 2 * j, 9
        pane = rng.integers(p_lo + 1, p_lo + np_ - 1, n).astype(np.int64)
        key = rng.integers(0, 1 << 40, n).astype(np.uint64)
        acc = rng.integers(-1000, 1000, n).astype(np.int64)
        cnt = rng.integers(1, 6, n).astype(np.int32)
        dirty = rng.integers(0, 2, n).astype(np.uint8)
        a.absorb(key, pane, acc, cnt.astype(np.int64), dirty)
        o = np.argsort(pane, kind="stable")  # what the device hands over: grouped by pane
        counts = np.bincount(pane - p_lo, minlength=np_).astype(np.uint32)
        b.absorb_presorted(key[o], acc[o], cnt[o], dirty[o], p_lo, counts)
        c3.absorb_presorted(key[o], acc[o], cnt[o], dirty[o], p_lo, counts, background=True)
        if j == 2:
            a.purge(24)
            b.purge(24)
            c3.purge(23)
            c3.purge(24)  # both deferred while the absorb runs; the larger cutoff applies
        assert a.nrows == b.nrows == c3.nrows and a.pane_range() == b.pane_range()
        assert c3.pane_range() == a.pane_range()

    def canon(t, p0, p1):
        k, x, c, n, _ = t.export(p0, p1, "cpu")
        m = np.stack([k.numpy(), x.numpy(), c.numpy().astype(np.int64)], 1)
        return m[np.lexsort(m.T[::-1])]

    for p0, p1 in ((20, 40), (25, 27), (30, 31)):
        assert np.array_equal(canon(a, p0, p1), canon(b, p0, p1))
        assert np.array_equal(canon(a, p0, p1), canon(c3, p0, p1))
    ra, rb = a.rows(), b.rows()
    for k in ("key", "pane", "acc", "cnt", "dirty"):
        assert np.array_equal(ra[k], rb[k])


def test_latency_fire_equals_pipelined():
    """latency_fire (fire in the call of the triggering batch when few windows are due) emits
    exactly the pipelined operator's rows -- sliding windows, allowed lateness, late data."""
    def run(latency_fire):
        op = KeyedWindowOperator(size=6_000, slide=1_000, lateness=3_000, agg=K.AGG_SUM_I64,
                                 device="cpu", max_keys=3000, batch_capacity=8192,
                                 ooo_bound=500, pipeline="stream", latency_fire=latency_fire)
        keys = torch.empty(8192, dtype=torch.int64)
        ts, vals = torch.empty_like(keys), torch.empty_like(keys)
        rows, imm = [], 0
        for i in range(30):
            K.gen_events(keys, ts, vals, seed=3, stream_id=0, idx0=i * 8192, nkeys=3000,
                         ts_base=i * 400, ts_span=400, disorder=500, val_lo=0, val_span=100)
            if i > 8:
                ts[:400] -= 2_500  # late but within the allowed lateness: re-firings
            before = op.metrics.steps
            out = op.process(keys, ts, vals)
            imm += sum(1 for r in out if r.seq == before + 1)
            rows += [(r.window_start, int(k), int(a)) for r in out
                     for k, a in zip(r.keys, r.raw)]
        rows += [(r.window_start, int(k), int(a)) for r in op.finish()
                 for k, a in zip(r.keys, r.raw)]
        return sorted(rows), op.metrics.extra.get("latency_fires", 0), imm

    ref, _, _ = run(0)
    got, n_fast, imm = run(64)
    assert got == ref and len(ref) > 1000
    assert n_fast > 10 and imm > 10  # firings returned by the call of their own batch


@pytest.mark.parametrize("world,exchange", [(2, "partials"), (4, "partials"), (2, "records")])
def test_spill_tier_multirank_matches_unbounded_table(world, exchange):
    """The host-DRAM tier at G > 1 (LoopbackComm ranks): local-global partials (each rank's tier
    rows join its local partials on the device before the owners merge) and the records
    exchange both equal one rank with a table that holds every key."""
    from mxstream.parallel.comm import run_loopback

    batches = _drift_batches(20, 6000, seed=5)
    ref, _ = _run_windows(batches, max_keys=80_000)

    def rank(comm):
        mine = [(k[comm.rank::world].contiguous(), t[comm.rank::world].contiguous(),
                 v[comm.rank::world].contiguous())
                for k, t, v in batches]
        return _run_windows(mine, max_keys=3000, spill=True, spill_check_steps=1,
                            spill_load=0.5, cap_log2=7, spill_keep_panes=1, comm=comm,
                            parallelism=world, exchange=exchange, window_keys=80_000)

    res = run_loopback(world, rank)
    got = sorted(r for rows, _ in res for r in rows)
    assert sum(op.metrics.extra.get("spilled_keys", 0) for _, op in res) > 0
    assert got == ref


@pytest.mark.parametrize("high_bit", [False, True])
def test_partials_merge_table_drops_dead_keys(high_bit):
    """Local-global owners keep a key in the merge table while a fired window inside its allowed
    lateness holds a value for it. With drifting keys the dead ones are compacted away (the
    table is sized for ~one window's keys here, far below the keys of the whole run) and the
    output still equals one rank with an unbounded table. high_bit: every key has its top bit
    set (negative int64); only -1 / -2 are reserved slot markers, so compaction must keep them
    and late re-firings must still see their merge slices."""
    from mxstream.parallel.comm import run_loopback

    batches = _drift_batches(40, 6000, seed=8)  # ~60K distinct keys over the run
    if high_bit:
        batches = [(k + np.iinfo(np.int64).min, t, v) for k, t, v in batches]
    ref, _ = _run_windows(batches, max_keys=120_000)
    world = 2

    def rank(comm):
        mine = [(k[comm.rank::world].contiguous(), t[comm.rank::world].contiguous(),
                 v[comm.rank::world].contiguous()) for k, t, v in batches]
        return _run_windows(mine, max_keys=120_000, comm=comm, parallelism=world,
                            exchange="partials", window_keys=16_000, cap_log2=7)

    res = run_loopback(world, rank)
    got = sorted(r for rows, _ in res for r in rows)
    assert sum(op.metrics.extra.get("merge_compactions", 0) for _, op in res) > 0
    assert got == ref


@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("combine", [True, False])
def test_narrow_records_exchange_equals_one_rank(world, combine):
    """8-byte records across the records exchange (key id < 2^32, int28 value, pane offset < 15;
    anything else widens the step's records): sender-side combiner or raw records, the output
    equals one rank."""
    from mxstream.parallel.comm import run_loopback

    batches = _drift_batches(12, 6000, seed=3)
    ref, _ = _run_windows(batches, max_keys=80_000)

    def rank(comm):
        mine = [(k[comm.rank::world].contiguous(), t[comm.rank::world].contiguous(),
                 v[comm.rank::world].contiguous()) for k, t, v in batches]
        return _run_windows(mine, max_keys=80_000, comm=comm, parallelism=world,
                            exchange="records", compact=True, narrow=True, combine=combine)

    res = run_loopback(world, rank)
    assert all(op.rec_w == 1 for _, op in res)
    assert sorted(r for rows, _ in res for r in rows) == ref
