"""Keyed rolling state (per-record emissions) vs the oracle; GPU vs the C++ twin."""
import numpy as np
import pytest
import torch

from mxstream.ops import expr as E
from mxstream.ops import kernels as K
from mxstream.runtime.rolling_operator import KeyedRollingOperator


def _gen(dev, n, nkeys, seed):
    keys = torch.empty(n, dtype=torch.int64, device=dev)
    ts = torch.empty_like(keys)
    vals = torch.empty_like(keys)
    K.gen_events(keys, ts, vals, seed=seed, stream_id=0, idx0=0, nkeys=nkeys, ts_base=0,
                 ts_span=1000, disorder=0, val_lo=-500, val_span=1000)
    return keys, vals


def _per_key(rows):
    d = {}
    order = np.argsort(rows.tags, kind="stable")
    for i in order:
        d.setdefault(int(rows.keys[i]), []).append(int(rows.values[i]))
    return d


def _oracle(batches, agg):
    state, out = {}, {}
    for keys, vals in batches:
        for k, v in zip(keys.tolist(), vals.tolist()):
            if agg == K.AGG_COUNT:
                state[k] = state.get(k, 0) + 1
            elif k not in state:
                state[k] = v
            elif agg == K.AGG_SUM_I64:
                state[k] += v
            elif agg == K.AGG_MAX_I64:
                state[k] = max(state[k], v)
            else:
                state[k] = min(state[k], v)
            out.setdefault(k, []).append(state[k])
    return out


@pytest.mark.parametrize("agg", [K.AGG_SUM_I64, K.AGG_MAX_I64, K.AGG_MIN_I64, K.AGG_COUNT])
def test_rolling_cpu_matches_oracle(agg):
    batches = [_gen("cpu", 3000, 97, s) for s in range(4)]
    op = KeyedRollingOperator(agg=agg, device="cpu", max_keys=200, batch_capacity=3000, cap_log2=8)
    got = {}
    for keys, vals in batches:
        for k, v in _per_key(op.process(keys, vals)).items():
            got.setdefault(k, []).extend(v)
    assert got == _oracle(batches, agg)


def test_rolling_filter_epilogue_cpu():
    batches = [_gen("cpu", 2000, 10, s) for s in range(3)]
    f = E.compile_expr(E.var(E.VAR_COUNT) % 100 == 0)
    op = KeyedRollingOperator(agg=K.AGG_COUNT, device="cpu", max_keys=16, batch_capacity=2000,
                              cap_log2=6, filter_prog=f)
    n = 0
    for keys, vals in batches:
        rows = op.process(keys, vals)
        assert all(int(v) % 100 == 0 for v in rows.values)
        n += len(rows.keys)
    assert n == sum(c // 100 for c in np.bincount(torch.cat([b[0] for b in batches]).numpy()))


@pytest.mark.gpu
@pytest.mark.parametrize("agg", [K.AGG_SUM_I64, K.AGG_MAX_I64, K.AGG_COUNT])
@pytest.mark.parametrize("nkeys", [10, 10_000])
@pytest.mark.parametrize("direct", [True, False])
def test_rolling_gpu_equals_cpu(gpu_device, agg, nkeys, direct):
    """direct=True: single-rank lookup from the source columns + slot-bits sort;
    direct=False: the partitioned path every rank takes at world size > 1."""
    res = {}
    for d in (gpu_device, torch.device("cpu")):
        op = KeyedRollingOperator(agg=agg, device=d, max_keys=nkeys, batch_capacity=1 << 16)
        op.direct_single_rank = direct
        got = {}
        for s in range(3):
            keys, vals = _gen(d, 1 << 16, nkeys, s)
            for k, v in _per_key(op.process(keys, vals)).items():
                got.setdefault(k, []).extend(v)
        res[d.type] = got
        if d.type == "cuda":
            tags = op.process(*_gen(d, 1 << 16, nkeys, 9)).tags
            assert len(tags) == 1 << 16 and len(np.unique(tags)) == 1 << 16
    assert res["cuda"] == res["cpu"]


@pytest.mark.gpu
@pytest.mark.parametrize("n,nkeys,zipf", [(1, 10, 0.0), (777, 50, 0.0), (70_001, 10_000, 0.0),
                                          (3_000_000, 10_000, 0.0), (1 << 20, 5_000, 1.2),
                                          (1 << 18, 11_000, 0.0)])
@pytest.mark.parametrize("filt", ["none", "count", "key", "stack", "ge", "k1000"])
def test_rolling_sort_free_count(gpu_device, n, nkeys, zipf, filt):
    """Sort-free COUNT (csrc/rolling_hist_hip.hip: chunk histograms, cross-chunk prefix, tile
    ranking by lane masks or, for rarely passing filters, the select path) == the sort path on
    the GPU == the C++ twin, per record, over several batches (state carried), chunk counts > 16
    (two-level prefix) and a Zipf hot key (its chunks fall back to ranking)."""
    fp = {"none": E.EMPTY, "count": E.compile_expr(E.var(E.VAR_COUNT) % 7 == 0),
          "key": E.compile_expr(E.var(E.VAR_KEY) % 3 == 1),
          # integer-mode chain (remainder, then an integer compare)
          "ge": E.compile_expr(E.var(E.VAR_COUNT) % 1000 >= 997),
          # config 2's alert: few passing counts per chunk (the emit pass's select path)
          "k1000": E.compile_expr(E.var(E.VAR_COUNT) % 1000 == 0),
          # not a chain program: the operator falls back to the sort path
          "stack": E.compile_expr((E.var(E.VAR_KEY) % 3 == 1) & (E.var(E.VAR_COUNT) > 2))}[filt]
    res = {}
    for d, sort_free in ((gpu_device, True), (gpu_device, False), (torch.device("cpu"), False)):
        op = KeyedRollingOperator(agg=K.AGG_COUNT, device=d, max_keys=nkeys, batch_capacity=n,
                                  filter_prog=fp)
        op.sort_free = sort_free
        if d.type == "cuda":
            assert op.nslots <= 16384
        got = {}
        for s in range(3):
            keys = torch.empty(n, dtype=torch.int64, device=d)
            K.gen_events(keys, torch.empty_like(keys), torch.empty_like(keys), seed=s, stream_id=0,
                         idx0=s * n, nkeys=nkeys, ts_base=0, ts_span=1000, disorder=0, val_lo=0,
                         val_span=10, zipf=zipf)
            rows = op.process(keys, keys)
            order = np.lexsort((rows.tags, rows.keys))
            got[s] = (rows.keys[order].tolist(), rows.values[order].tolist(),
                      rows.tags[order].tolist())
        res[(d.type, sort_free)] = got
        res[(d.type, sort_free, "state")] = sorted(
            (int(k), int(c)) for k, c in zip(op.keys_g.cpu().tolist(), op.cnt_g.cpu().tolist())
            if k != -1)
    assert res[("cuda", True)] == res[("cpu", False)]
    assert res[("cuda", False)] == res[("cpu", False)]
    assert res[("cuda", True, "state")] == res[("cpu", False, "state")]


@pytest.mark.gpu
@pytest.mark.parametrize("zipf", [0.0, 1.1])
def test_rolling_dense_keys(gpu_device, zipf):
    """Dictionary-id keys (slot = id, no probe) give the hashed CPU twin's rows and state; a
    snapshot restores into a fresh dense operator; an id >= max_keys raises."""
    n, nkeys = 200_003, 9_000
    fp = E.compile_expr(E.var(E.VAR_COUNT) % 5 == 0)
    ops = {"dense": KeyedRollingOperator(agg=K.AGG_COUNT, device=gpu_device, max_keys=nkeys,
                                         batch_capacity=n, filter_prog=fp, dense_keys=True),
           "cpu": KeyedRollingOperator(agg=K.AGG_COUNT, device="cpu", max_keys=nkeys,
                                       batch_capacity=n, filter_prog=fp)}
    res = {}
    for name, op in ops.items():
        d = op.device
        got = []
        for s in range(3):
            keys = torch.empty(n, dtype=torch.int64, device=d)
            K.gen_events(keys, torch.empty_like(keys), torch.empty_like(keys), seed=s, stream_id=0,
                         idx0=s * n, nkeys=nkeys, ts_base=0, ts_span=1000, disorder=0, val_lo=0,
                         val_span=10, zipf=zipf)
            rows = op.process(keys, keys)
            order = np.lexsort((rows.tags, rows.keys))
            got.append((rows.keys[order].tolist(), rows.values[order].tolist()))
        res[name] = got
    assert res["dense"] == res["cpu"]
    snap = ops["dense"].snapshot_state()
    fresh = KeyedRollingOperator(agg=K.AGG_COUNT, device=gpu_device, max_keys=nkeys,
                                 batch_capacity=n, filter_prog=fp, dense_keys=True)
    fresh.restore_state(snap.columns, snap.meta)
    for k in (0, 17, nkeys - 1):
        assert fresh.state_of(k)[1] == ops["cpu"].state_of(k)[1]  # counts (COUNT keeps no acc)
    bad = torch.full((10,), 1 << 20, dtype=torch.int64, device=gpu_device)
    with pytest.raises(ValueError, match="dense"):
        fresh.process(bad, bad)


def _count_oracle(batches, agg, n):
    """Tumbling count windows per key (countWindow(n)): one row per n elements."""
    win, out = {}, {}
    for keys, vals in batches:
        for k, v in zip(keys.tolist(), vals.tolist()):
            w = win.setdefault(k, [])
            w.append(v)
            if len(w) == n:
                r = {K.AGG_SUM_I64: sum(w), K.AGG_MAX_I64: max(w), K.AGG_MIN_I64: min(w),
                     K.AGG_COUNT: n, K.AGG_AVG_I64: sum(w)}[agg]
                out.setdefault(k, []).append(r)
                win[k] = []
    return out


@pytest.mark.parametrize("agg", [K.AGG_SUM_I64, K.AGG_MAX_I64, K.AGG_MIN_I64, K.AGG_COUNT,
                                 K.AGG_AVG_I64])
@pytest.mark.parametrize("n", [1, 7, 64, 150])
def test_count_window_cpu_matches_oracle(agg, n):
    batches = [_gen("cpu", 3000, 97, s) for s in range(4)]
    op = KeyedRollingOperator(agg=agg, device="cpu", max_keys=200, batch_capacity=3000,
                              cap_log2=8, count_window=n)
    got = {}
    for keys, vals in batches:
        for k, v in _per_key(op.process(keys, vals)).items():
            got.setdefault(k, []).extend(v)
    assert got == _count_oracle(batches, agg, n)
    with pytest.raises(ValueError):
        KeyedRollingOperator(agg=K.AGG_AVG_I64, device="cpu")  # avg only with count windows


@pytest.mark.gpu
@pytest.mark.parametrize("agg", [K.AGG_SUM_I64, K.AGG_MAX_I64, K.AGG_COUNT, K.AGG_AVG_I64])
@pytest.mark.parametrize("n", [1, 5, 64, 100, 300])
@pytest.mark.parametrize("direct", [True, False])
def test_count_window_gpu_equals_cpu(gpu_device, agg, n, direct):
    """The segmented wave scan (window boundaries inside and across 64-element chunks and
    batches) emits exactly the C++ twin's windows."""
    res = {}
    for d in (gpu_device, torch.device("cpu")):
        op = KeyedRollingOperator(agg=agg, device=d, max_keys=300, batch_capacity=1 << 15,
                                  count_window=n)
        op.direct_single_rank = direct
        got = {}
        for s in range(3):
            keys, vals = _gen(d, 1 << 15, 300, s)
            for k, v in _per_key(op.process(keys, vals)).items():
                got.setdefault(k, []).extend(v)
        res[d.type] = got
    assert res["cuda"] == res["cpu"]
    assert sum(len(v) for v in res["cpu"].values()) > 0


def _drifting_batches(dev, nbatches, per, window, drift, seed):
    """Keys from a moving id window, plus a few revisits of long-gone keys (spilled state that
    must come back with its value)."""
    g = torch.Generator().manual_seed(seed)
    out = []
    for b in range(nbatches):
        k = torch.randint(0, window, (per,), generator=g, dtype=torch.int64) + b * drift
        if b >= 6:
            k[::17] = torch.randint(0, drift, (k[::17].numel(),), generator=g) + (b - 6) * drift
        v = torch.randint(-500, 500, (per,), generator=g, dtype=torch.int64)
        out.append((k.to(dev), v.to(dev)))
    return out


def _spill_run(dev, batches, agg, spill, max_keys):
    op = KeyedRollingOperator(agg=agg, device=dev, max_keys=max_keys, batch_capacity=4096,
                              spill=spill)
    rows = [op.process(k, v) for k, v in batches]
    got = {}
    for r in rows:
        for k, val in _per_key(r).items():
            got.setdefault(k, []).extend(val)
    return got, op


@pytest.mark.parametrize("agg", [K.AGG_SUM_I64, K.AGG_MAX_I64, K.AGG_COUNT])
def test_rolling_spill_tier_matches_unbounded_cpu(agg):
    """Keyed rolling state over a key space ~4x the table: LRU keys move to host DRAM and come
    back with their values when they reappear; emissions equal an unbounded table's and the
    oracle's."""
    dev = torch.device("cpu")
    batches = _drifting_batches(dev, 14, 600, 120, 80, 3)
    got, op = _spill_run(dev, batches, agg, True, 256)
    ref, _ = _spill_run(dev, batches, agg, False, 1 << 13)
    assert got == ref == _oracle(batches, agg)
    assert op.spill_stats["spilled_keys"] > 0 and op.spill_stats["promoted_keys"] > 0
    assert len(op.store) > 0 and op.host_bytes() > 0
    # checkpoint with spilled keys restores into an operator of the same (small) table
    snap = op.snapshot_state()
    fresh = KeyedRollingOperator(agg=agg, device=dev, max_keys=256, batch_capacity=4096,
                                 spill=True)
    fresh.restore_state(dict(snap.columns), snap.meta)
    more = _drifting_batches(dev, 3, 600, 120, 80, 9)
    a = [fresh.process(k, v) for k, v in more]
    b = [op.process(k, v) for k, v in more]
    for x, y in zip(a, b):
        assert _per_key(x) == _per_key(y)


@pytest.mark.gpu
@pytest.mark.parametrize("agg", [K.AGG_SUM_I64, K.AGG_COUNT])
def test_rolling_spill_tier_gpu_matches_unbounded(gpu_device, agg):
    batches = _drifting_batches(gpu_device, 14, 600, 120, 80, 4)
    got, op = _spill_run(gpu_device, batches, agg, True, 256)
    ref, _ = _spill_run(gpu_device, batches, agg, False, 1 << 13)
    cpu = [(k.cpu(), v.cpu()) for k, v in batches]
    assert got == ref == _oracle(cpu, agg)
    assert op.spill_stats["spilled_keys"] > 0 and op.spill_stats["promoted_keys"] > 0
