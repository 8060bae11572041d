"""gfx950 kernels vs the C++ twins and plain PyTorch references (needs an MI355X)."""
import numpy as np
import pytest
import torch

from mxstream.ops import expr as E
from mxstream.ops import kernels as K
from mxstream.runtime.window_operator import KeyedWindowOperator

pytestmark = pytest.mark.gpu


def _gen(dev, n, nkeys, span=10_000, disorder=300, seed=3, f64=False):
    keys = torch.empty(n, dtype=torch.int64, device=dev)
    ts = torch.empty_like(keys)
    vals = torch.empty_like(keys)
    K.gen_events(keys, ts, vals, seed=seed, stream_id=1, idx0=17, nkeys=nkeys, ts_base=1000,
                 ts_span=span, disorder=disorder, val_lo=0, val_span=1000, val_f64=f64)
    return keys, ts, vals


def test_native_module_is_loaded(native, gpu_device):
    assert native.gpu_device_count() >= 1
    assert native.__file__.endswith(".so")


def test_gen_events_bit_exact(gpu_device):
    g = _gen(gpu_device, 100_003, 777)
    c = _gen("cpu", 100_003, 777)
    for a, b in zip(g, c):
        assert torch.equal(a.cpu(), b)


def test_partition_matches_cpu_as_multisets(gpu_device):
    n = 200_000
    g = _gen(gpu_device, n, 50_000)
    c = _gen("cpu", n, 50_000)
    outs = {}
    for dev, (keys, ts, vals) in (("gpu", g), ("cpu", c)):
        d = keys.device
        plan = K.PartitionPlan(max_parallelism=128, nsub_log2=6, nranks=4, window_mode=1,
                               drop_late=1, hash_mode=0, bucket_cap=2048, late_ts=3000,
                               tbase=500, pane=500)
        kg = torch.tensor([(k * 4) // 128 for k in range(128)], dtype=torch.int32, device=d)
        cursor = torch.zeros(plan.nbuckets, dtype=torch.int32, device=d)
        out = torch.zeros(plan.nbuckets * plan.bucket_cap * 3, dtype=torch.int64, device=d)
        stats = K.new_stats(d)
        K.partition(keys, ts, vals, plan, kg, cursor, out, stats)
        outs[dev] = (cursor.cpu(), out.cpu().view(plan.nbuckets, plan.bucket_cap, 3), stats.cpu())
    cg, og, sg = outs["gpu"]
    cc, oc, sc = outs["cpu"]
    assert torch.equal(sg, sc)
    assert sg[K.STAT_OVERFLOW] == 0
    hole = np.int64(-1)  # t = aux = 0xFFFFFFFF: padding of the write-combined scatter
    for b in range(cg.numel()):
        a = og[b, :int(cg[b])].numpy()
        a = a[a[:, 2] != hole]
        e = oc[b, :int(cc[b])].numpy()
        assert len(a) == len(e)
        assert np.array_equal(a[np.lexsort(a.T[::-1])], e[np.lexsort(e.T[::-1])])


def _results(out):
    return {(r.window_start, int(k)): (int(a), int(c))
            for r in out for k, a, c in zip(r.keys, r.raw, r.counts)}


@pytest.mark.parametrize("size,slide,lateness", [(2000, 2000, 0), (3000, 1000, 0), (2000, 500, 700)])
def test_window_operator_gpu_equals_cpu(gpu_device, size, slide, lateness):
    res = {}
    for d in (gpu_device, torch.device("cpu")):
        op = KeyedWindowOperator(size=size, slide=slide, lateness=lateness, agg=K.AGG_SUM_I64,
                                 device=d, max_keys=20_000, batch_capacity=1 << 16,
                                 ooo_bound=300, cap_log2=9)
        out = []
        for step in range(6):
            keys, ts, vals = _gen(d, 1 << 16, 20_000, span=2500, disorder=1500, seed=step)
            ts += step * 2500
            out += op.process(keys, ts, vals)
        out += op.finish()
        res[d.type] = (_results(out), op.metrics.num_late_records_dropped)
    assert res["cuda"] == res["cpu"]


def test_window_sum_vs_torch_reference(gpu_device):
    """Tumbling window sums vs a plain PyTorch (index_add) reference of the same op."""
    n = 1 << 20
    keys, ts, vals = _gen(gpu_device, n, 100_000, span=4000, disorder=0)
    op = KeyedWindowOperator(size=1000, agg=K.AGG_SUM_I64, device=gpu_device, max_keys=100_000,
                             batch_capacity=n)
    out = op.process(keys, ts, vals) + op.finish()
    got = _results(out)
    win = torch.div(ts, 1000, rounding_mode="floor")
    comp = win * 1_000_000 + keys
    uniq, inv = torch.unique(comp, return_inverse=True)
    sums = torch.zeros(uniq.numel(), dtype=torch.int64, device=gpu_device).index_add_(0, inv, vals)
    cnts = torch.zeros(uniq.numel(), dtype=torch.int64, device=gpu_device).index_add_(
        0, inv, torch.ones_like(vals))
    exp = {(int(u) // 1_000_000 * 1000, int(u) % 1_000_000): (int(s), int(c))
           for u, s, c in zip(uniq.cpu(), sums.cpu(), cnts.cpu())}
    assert got == exp


@pytest.mark.parametrize("agg", [K.AGG_SUM_I64, K.AGG_AVG_I64])
def test_packed_int_sums_extreme_values(gpu_device, agg):
    """Packed (48-bit sum, 16-bit count) LDS accumulators: int32 extremes of both signs and hot
    keys with thousands of records per slot per step, vs a PyTorch int64 reference."""
    n = 1 << 18
    g = torch.Generator(device="cpu").manual_seed(7)
    keys = torch.randint(0, 64, (n,), generator=g, dtype=torch.int64)  # ~4K records per key
    keys[: n // 2] = torch.randint(0, 50_000, (n // 2,), generator=g, dtype=torch.int64)
    ts = torch.randint(0, 3000, (n,), generator=g, dtype=torch.int64)
    vals = torch.randint(-(2**31), 2**31, (n,), generator=g, dtype=torch.int64)
    vals[::7] = 2**31 - 1
    vals[::11] = -(2**31)
    op = KeyedWindowOperator(size=1000, agg=agg, device=gpu_device, max_keys=60_000,
                             batch_capacity=n)
    out = op.process(keys.to(gpu_device), ts.to(gpu_device), vals.to(gpu_device)) + op.finish()
    got = _results(out)
    comp = torch.div(ts, 1000, rounding_mode="floor") * 1_000_000 + keys
    uniq, inv = torch.unique(comp, return_inverse=True)
    sums = torch.zeros(uniq.numel(), dtype=torch.int64).index_add_(0, inv, vals)
    cnts = torch.zeros(uniq.numel(), dtype=torch.int64).index_add_(0, inv, torch.ones_like(vals))
    exp = {(int(u) // 1_000_000 * 1000, int(u) % 1_000_000): (int(s), int(c))
           for u, s, c in zip(uniq, sums, cnts)}
    assert got == exp


@pytest.mark.parametrize("agg", [K.AGG_SUM_F64, K.AGG_MIN_F64, K.AGG_MAX_F64, K.AGG_AVG_F64])
def test_float_aggregates_vs_torch(gpu_device, agg):
    n = 1 << 18
    keys, ts, vals = _gen(gpu_device, n, 3000, span=1000, disorder=0, f64=True)
    op = KeyedWindowOperator(size=10_000, agg=agg, device=gpu_device, max_keys=3000,
                             batch_capacity=n)
    out = op.process(keys, ts, vals) + op.finish()
    v = vals.view(torch.float64)
    uniq, inv = torch.unique(keys, return_inverse=True)
    if agg in (K.AGG_SUM_F64, K.AGG_AVG_F64):
        ref = torch.zeros(uniq.numel(), dtype=torch.float64, device=gpu_device).index_add_(0, inv, v)
        if agg == K.AGG_AVG_F64:
            ref = ref / torch.bincount(inv).double()
    else:
        red = "amin" if agg == K.AGG_MIN_F64 else "amax"
        ref = torch.zeros(uniq.numel(), dtype=torch.float64, device=gpu_device).scatter_reduce_(
            0, inv, v, red, include_self=False)
    exp = dict(zip(uniq.cpu().tolist(), ref.cpu().tolist()))
    got = {int(k): float(x) for r in out for k, x in zip(r.keys, r.values)}
    assert set(got) == set(exp)
    for k, x in exp.items():
        assert got[k] == pytest.approx(x, rel=1e-12)


def test_fire_epilogue_bit_exact(gpu_device):
    n = 1 << 18
    m = E.compile_expr(E.var(E.VAR_RESULT) * 8.0 / 60 / 1024 / 1024)
    f = E.compile_expr(E.var(E.VAR_MAPPED) < 1.5)
    res = {}
    for d in (gpu_device, torch.device("cpu")):
        keys, ts, vals = _gen(d, n, 4000, span=3000, disorder=0)
        op = KeyedWindowOperator(size=1000, agg=K.AGG_SUM_I64, device=d, max_keys=4000,
                                 batch_capacity=n, map_prog=m, filter_prog=f)
        out = op.process(keys, ts, vals) + op.finish()
        res[d.type] = {(r.window_start, int(k)): float(v) for r in out for k, v in zip(r.keys, r.values)}
    assert res["cuda"] == res["cpu"] and len(res["cpu"]) > 0


def test_expr_filter_gpu(gpu_device):
    x = torch.linspace(0, 100, 10_001, dtype=torch.float64, device=gpu_device)
    prog = E.compile_expr(E.var(0) > 90)
    keep = K.expr_filter(x, prog)
    assert torch.equal(keep, x > 90)


@pytest.mark.parametrize("nsub_log2,nranks", [(9, 1), (6, 8), (3, 2)])
def test_partition_staged_variant_matches_plain(native, gpu_device, nsub_log2, nranks):
    """The write-combined partition (variant 4) holds the same records per bucket as the plain
    scatter (variant 0); its padding holes carry t == 0xFFFFFFFF."""
    n = 300_001
    keys, ts, vals = _gen(gpu_device, n, 70_000)
    nb = nranks << nsub_log2
    bcap = (int(n / nb * 1.5) + 8 * 1024 + 7) & ~7
    kg = torch.tensor([(k * nranks) // 128 for k in range(128)], dtype=torch.int32,
                      device=gpu_device)
    plan = K.PartitionPlan(max_parallelism=128, nsub_log2=nsub_log2, nranks=nranks, window_mode=1,
                           drop_late=1, hash_mode=0, bucket_cap=bcap, late_ts=2000, tbase=500,
                           pane=500)
    res = {}
    for var in (0, 4):
        cursor = torch.zeros(nb, dtype=torch.int32, device=gpu_device)
        out = torch.zeros(nb * bcap * 3, dtype=torch.int64, device=gpu_device)
        stats = K.new_stats(gpu_device)
        native.gpu_partition_variant(keys.data_ptr(), ts.data_ptr(), vals.data_ptr(), 0, n,
                                     plan.as_dict(), kg.data_ptr(), cursor.data_ptr(),
                                     out.data_ptr(), stats.data_ptr(),
                                     torch.cuda.current_stream().cuda_stream, var)
        res[var] = (cursor.cpu(), out.cpu().view(nb, bcap, 3), stats.cpu())
    c0, o0, s0 = res[0]
    c4, o4, s4 = res[4]
    assert torch.equal(s0, s4)
    for b in range(nb):
        a = o0[b, :int(c0[b])].numpy()
        e = o4[b, :int(c4[b])].numpy()
        e = e[e[:, 2] != np.int64(-1)]
        assert len(a) == len(e)
        assert np.array_equal(a[np.lexsort(a.T[::-1])], e[np.lexsort(e.T[::-1])])
        assert int(c4[b]) % 8 == 0


@pytest.mark.parametrize("agg", [K.AGG_SUM_I64, K.AGG_MAX_I64, K.AGG_COUNT, K.AGG_AVG_F64])
def test_window_combine_matches_cpu(gpu_device, agg):
    """Sender-side combiner (G > 1 path) on the GPU vs its C++ twin on the same send buckets."""
    n = 200_000
    outs = {}
    for dev in (gpu_device, "cpu"):
        keys, ts, vals = _gen(dev, n, 20_000, f64=agg in K.AGG_IS_F64)
        plan = K.PartitionPlan(max_parallelism=128, nsub_log2=4, nranks=2, window_mode=1,
                               drop_late=0, hash_mode=0, bucket_cap=16384, tbase=1000, pane=500)
        kg = torch.tensor([(k * 2) // 128 for k in range(128)], dtype=torch.int32, device=dev)
        cursor = torch.zeros(plan.nbuckets, dtype=torch.int32, device=dev)
        send = torch.zeros(plan.nbuckets * plan.bucket_cap * 3, dtype=torch.int64, device=dev)
        stats = K.new_stats(dev)
        K.partition(keys, ts, vals, plan, kg, cursor, send, stats)
        qmin, qmax = int(stats[K.STAT_MINPANE]), int(stats[K.STAT_MAXPANE])
        ccap = 2048 * (qmax - qmin + 1)
        out = torch.zeros(plan.nbuckets * ccap * 3, dtype=torch.int64, device=dev)
        oc = torch.zeros(plan.nbuckets, dtype=torch.int32, device=dev)
        flags = torch.zeros(1, dtype=torch.int32, device=dev)
        cp = K.AggPlan(cap_log2=11, nsub=plan.nbuckets, ring=1, agg=agg, nsrc=1,
                       bucket_cap=plan.bucket_cap, np_step=qmax - qmin + 1, pg=2, pane_base=0,
                       p_lo=qmin, fired_hi=0)
        K.window_combine(send, cursor, cp, out, ccap, oc, flags)
        assert int(flags[0]) == 0
        outs[str(dev)] = (oc.cpu(), out.cpu().view(plan.nbuckets, ccap, 3))
    (cg, og), (cc, occ) = outs[str(gpu_device)], outs["cpu"]
    assert torch.equal(cg, cc)
    for b in range(cg.numel()):
        a = og[b, :int(cg[b])].numpy()
        e = occ[b, :int(cc[b])].numpy()
        sa = a[np.lexsort((a[:, 2], a[:, 0]))]
        se = e[np.lexsort((e[:, 2], e[:, 0]))]
        assert np.array_equal(sa[:, [0, 2]], se[:, [0, 2]])  # key, (t | count << 32)
        if agg == K.AGG_AVG_F64:  # f64 sums: order-dependent rounding
            assert np.allclose(sa[:, 1].view(np.float64), se[:, 1].view(np.float64), rtol=1e-12)
        else:
            assert np.array_equal(sa[:, 1], se[:, 1])


def test_segment_median_vs_numpy(gpu_device):
    rng = np.random.default_rng(9)
    n = 300_000
    keys = rng.integers(0, 5000, n)
    vals = rng.normal(0, 100, n)
    vals[::977] = -0.0
    vals[::1301] = 0.0
    kt = torch.from_numpy(keys).to(gpu_device)
    vt = torch.from_numpy(vals).to(gpu_device).view(torch.int64)
    uniq, ids = torch.unique(kt, return_inverse=True)
    ordv = K.f64_order_bits(vt.contiguous())
    ordv, ids = K.sort_pairs(ordv, ids.contiguous(), bits=64)
    ids, ordv = K.sort_pairs(ids.contiguous(), ordv, bits=13)
    heads = torch.nonzero(torch.cat([torch.ones(1, dtype=torch.bool, device=gpu_device),
                                     ids[1:] != ids[:-1]])).flatten()
    med = K.segment_median(heads.contiguous(), ordv).cpu().numpy()
    got = dict(zip(uniq[ids[heads]].cpu().tolist(), med.tolist()))
    for k in range(0, 5000, 97):
        v = np.sort(vals[keys == k])
        if not len(v):
            continue
        exp = v[len(v) // 2] if len(v) % 2 else (v[len(v) // 2] + v[len(v) // 2 - 1]) / 2
        assert got[k] == exp


def test_compact_partition_matches_cpu(gpu_device):
    """16-byte record partition (keys-only histogram pass, hole-filled reservations) vs the C++
    twin, including late records (their reserved slots become holes)."""
    n = 300_000
    outs = {}
    for dev in (gpu_device, "cpu"):
        keys, ts, vals = _gen(dev, n, 40_000, span=6000, disorder=2000)
        plan = K.PartitionPlan(max_parallelism=128, nsub_log2=7, nranks=2, window_mode=1,
                               drop_late=1, hash_mode=0, bucket_cap=4096, late_ts=2500,
                               tbase=1000, pane=500, rec_words=2)
        kg = torch.tensor([(k * 2) // 128 for k in range(128)], dtype=torch.int32, device=dev)
        cursor = torch.zeros(plan.nbuckets, dtype=torch.int32, device=dev)
        out = torch.zeros(plan.nbuckets * plan.bucket_cap * 3, dtype=torch.int64, device=dev)
        stats = K.new_stats(dev)
        K.partition(keys, ts, vals, plan, kg, cursor, out, stats)
        outs[str(dev)] = (cursor.cpu(), out.cpu()[: plan.nbuckets * plan.bucket_cap * 2]
                          .view(plan.nbuckets, plan.bucket_cap, 2), stats.cpu())
    (cg, og, sg), (cc, oc, sc) = outs[str(gpu_device)], outs["cpu"]
    # The compact kernel also reports the largest (padded) bucket fill; the C++ twin does not.
    assert int(sg[K.STAT_MAXBUCKET]) == int(cg.max())
    sg[K.STAT_MAXBUCKET] = 0
    assert torch.equal(sg, sc) and int(sg[K.STAT_LATE]) > 0 and int(sg[K.STAT_OVERFLOW]) == 0
    for b in range(cg.numel()):
        a = og[b, :int(cg[b])].numpy()
        a = a[(a[:, 1] >> 32) != -1]  # drop holes (t = 0xFFFFFFFF)
        e = oc[b, :int(cc[b])].numpy()
        assert np.array_equal(a[np.lexsort(a.T[::-1])], e[np.lexsort(e.T[::-1])])


@pytest.mark.parametrize("narrow", [False, True])
def test_late_refires_at_scale_equal_cpu(gpu_device, narrow):
    """Sliding windows with allowed lateness and 5 % late events at full sub-table size
    (4096 slots: packed accumulators + the LDS touched-slot list): every re-firing row equals
    the C++ twin's. A touched-slot list truncated by an undersized LDS image drops re-fired keys
    (config 4 once emitted 1.45M instead of 5.08M alerts)."""

    def run(dev):
        op = KeyedWindowOperator(size=6000, slide=1000, lateness=3000, agg=K.AGG_SUM_I64,
                                 device=dev, max_keys=200_000, batch_capacity=400_000,
                                 ooo_bound=500, narrow=narrow if dev != "cpu" else False)
        rows = []
        for step in range(14):
            k = torch.empty(400_000, dtype=torch.int64, device=dev)
            t = torch.empty_like(k)
            v = torch.empty_like(k)
            K.gen_events(k, t, v, seed=5, stream_id=0, idx0=step * 400_000, nkeys=150_000,
                         ts_base=step * 1000, ts_span=1000, disorder=500, val_lo=0,
                         val_span=1000)
            if step > 6:
                t[:20_000] -= 2500  # late, within the allowed lateness
            rows += op.process(k, t, v)
        rows += op.finish()
        return sorted((r.window_start, r.refire, int(a), int(b), int(c))
                      for r in rows for a, b, c in zip(r.keys, r.raw, r.counts))

    g, c = run(gpu_device), run("cpu")
    assert sum(1 for x in c if x[1]) > 10_000  # many re-fired rows
    assert g == c


@pytest.mark.parametrize("narrow,compact", [(True, True), (False, True), (False, False)])
def test_int32_keys_gpu_match_cpu(gpu_device, narrow, compact):
    """int32 key ids through the GPU partition (read as 4-byte keys by the 8- and 16-byte record
    kernels, widened for the 24-byte path) fire exactly the C++ twin's rows from int64 keys."""

    def run(dev, dtype):
        op = KeyedWindowOperator(size=3000, slide=1000, agg=K.AGG_SUM_I64, device=dev,
                                 max_keys=100_000, batch_capacity=300_000, ooo_bound=400,
                                 dense_keys=True, narrow=narrow if dev != "cpu" else False,
                                 compact=compact if dev != "cpu" else None)
        rows = []
        for step in range(8):
            k = torch.empty(300_000, dtype=dtype, device=dev)
            t = torch.empty(300_000, dtype=torch.int64, device=dev)
            v = torch.empty_like(t)
            K.gen_events(k, t, v, seed=11, stream_id=0, idx0=step * 300_000, nkeys=90_000,
                         ts_base=step * 1000, ts_span=1000, disorder=400, val_lo=0,
                         val_span=5000)
            rows += op.process(k, t, v)
        rows += op.finish()
        return sorted((r.window_start, int(a), int(b), int(c))
                      for r in rows for a, b, c in zip(r.keys, r.raw, r.counts))

    assert run(gpu_device, torch.int32) == run("cpu", torch.int64)


@pytest.mark.parametrize("zipf,narrow", [(1.2, True), (1.2, False), (0.9, True)])
def test_hot_keys_gpu_match_cpu(gpu_device, zipf, narrow):
    """Power-law keys (key 0 carries ~14 % of the events at s = 1.2): LDS atomics on one hot
    slot, one bucket far above the mean (bucket regrow + step redo) -- the fired rows equal the
    C++ twin's. The batches are generated once on the CPU and copied to the device."""
    batches = []
    for step in range(6):
        k = torch.empty(400_000, dtype=torch.int64)
        t = torch.empty_like(k)
        v = torch.empty_like(k)
        K.gen_events(k, t, v, seed=21, stream_id=0, idx0=step * 400_000, nkeys=200_000,
                     ts_base=step * 1000, ts_span=1000, disorder=300, val_lo=0, val_span=3000,
                     zipf=zipf)
        batches.append((k, t, v))

    def run(dev):
        op = KeyedWindowOperator(size=2000, slide=1000, agg=K.AGG_SUM_I64, device=dev,
                                 max_keys=200_000, batch_capacity=400_000, ooo_bound=300,
                                 dense_keys=True, narrow=narrow if dev != "cpu" else False)
        rows = []
        for k, t, v in batches:
            rows += op.process(k.to(dev), t.to(dev), v.to(dev))
        rows += op.finish()
        return sorted((r.window_start, int(a), int(b), int(c))
                      for r in rows for a, b, c in zip(r.keys, r.raw, r.counts)), op

    (g, gop), (c, _) = run(gpu_device), run("cpu")
    assert g == c
    top = max(x[3] for x in c)
    assert top > 20_000  # the hot key really is hot (mean count per key and window: ~4)


@pytest.mark.parametrize("dense", [False, True])
def test_deterministic_f64_sums_gpu_bit_exact(gpu_device, dense):
    """deterministic=True: the GPU's LDS fixed-point accumulation (two 64-bit atomics per add)
    gives f64 window sums bit-identical to the C++ twin's, run after run."""
    import sys

    sys.path.insert(0, __import__("os").path.dirname(__file__))
    from test_window_operator_cpu import _f64_batches

    batches = _f64_batches(200_000, 5, 11)

    def run(dev):
        op = KeyedWindowOperator(size=2000, agg=K.AGG_SUM_F64, device=dev, max_keys=600,
                                 batch_capacity=200_000, deterministic=True, dense_keys=dense)
        rows = {}
        for k, t, v in batches:
            for r in op.process(k.to(dev), t.to(dev), v.to(dev)) + []:
                rows.update({(r.window_start, a): b for a, b in zip(r.keys.tolist(), r.raw.tolist())})
        for r in op.finish():
            rows.update({(r.window_start, a): b for a, b in zip(r.keys.tolist(), r.raw.tolist())})
        return rows

    g1, g2, c = run(gpu_device), run(gpu_device), run("cpu")
    assert g1 == c and g2 == c and len(c) > 1000


@pytest.mark.parametrize("pane_sort", [True, False])
def test_spill_tier_gpu_matches_unbounded_cpu(gpu_device, pane_sort, monkeypatch):
    """window_compact on the GPU (LDS rehash of every sub-table, eviction rows to the host
    tier, grouped by pane on the device or by the tier's host sort) + tiered firings == an
    unbounded C++-twin table."""
    import sys

    monkeypatch.setenv("MXS_EVICT_PANE_SORT", "1" if pane_sort else "0")

    sys.path.insert(0, __import__("os").path.dirname(__file__))
    from test_window_operator_cpu import _drift_batches, _run_windows

    batches = _drift_batches(26, 6000)
    ref, _ = _run_windows(batches, max_keys=80_000)
    got, op = _run_windows(batches, device=gpu_device, max_keys=3000, spill=True,
                           spill_check_steps=1, spill_load=0.5, cap_log2=7, spill_keep_panes=1)
    assert op.metrics.extra.get("spilled_keys", 0) > 0
    # evictions went to host DRAM asynchronously; firings merged the tier on the device
    assert op.metrics.extra.get("async_evictions", 0) > 0
    assert got == ref


@pytest.mark.parametrize("exchange", ["partials", "records"])
def test_spill_tier_gpu_loopback_g4_matches_unbounded_cpu(gpu_device, exchange):
    """The host-DRAM tier at G = 4 (virtual ranks on one MI355X): asynchronous eviction, tier
    rows merged on the device into each rank's local partials (local-global) or into the
    owner's tiered firing (records exchange) == one unbounded C++-twin table."""
    import sys

    from mxstream.parallel.comm import run_loopback

    sys.path.insert(0, __import__("os").path.dirname(__file__))
    from test_window_operator_cpu import _drift_batches, _run_windows

    batches = _drift_batches(20, 6000, seed=5)
    ref, _ = _run_windows(batches, max_keys=80_000)

    def rank(comm):
        mine = [(k[comm.rank::4].contiguous(), t[comm.rank::4].contiguous(),
                 v[comm.rank::4].contiguous()) for k, t, v in batches]
        return _run_windows(mine, device=gpu_device, max_keys=3000, spill=True,
                            spill_check_steps=1, spill_load=0.5, cap_log2=7, spill_keep_panes=1,
                            comm=comm, parallelism=4, exchange=exchange, window_keys=80_000)

    res = run_loopback(4, rank, device=gpu_device)
    got = sorted(r for rows, _ in res for r in rows)
    assert sum(op.metrics.extra.get("spilled_keys", 0) for _, op in res) > 0
    assert got == ref


def test_segment_median_select_gpu_matches_cpu(gpu_device):
    """Median of unsorted segments: LDS bitonic path (<= 2048 values) and radix-select path
    (longer segments, odd and even lengths) equal numpy's median and the C++ twin."""
    rng = np.random.default_rng(1)
    lens = [1, 2, 3, 63, 64, 65, 1000, 2047, 2048, 2049, 5000, 10_001, 7]
    vals = rng.standard_normal(sum(lens)) * 1e3
    vals[:20] = 5.0  # ties
    heads = torch.tensor(np.r_[0, np.cumsum(lens)[:-1]], dtype=torch.int64)
    ordb = K.f64_order_bits(torch.from_numpy(vals).view(torch.int64))
    g = K.segment_median(heads.to(gpu_device), ordb.to(gpu_device), sorted_values=False).cpu()
    c = K.segment_median(heads, ordb, sorted_values=False)
    ref = [np.median(vals[a:a + n]) for a, n in zip(heads.tolist(), lens)]
    assert torch.equal(g, c) and np.allclose(c.numpy(), ref, rtol=0, atol=0)


def test_h2d_kernel_copies_pinned_bytes(gpu_device):
    """gpu_h2d_kernel: the copy kernel reads a pinned host buffer over PCIe (16-byte granules);
    misaligned sizes are refused, not truncated."""
    from mxstream.ops.native import load

    m = load()
    st = torch.cuda.current_stream(gpu_device).cuda_stream
    for nb in (16, 4096, (3 << 20) + 48):
        src = torch.randint(0, 256, (nb,), dtype=torch.uint8).pin_memory()
        dst = torch.zeros(nb, dtype=torch.uint8, device=gpu_device)
        assert m.gpu_h2d_kernel(dst.data_ptr(), src.data_ptr(), nb, st, 64) == 0
        torch.cuda.synchronize()
        assert torch.equal(dst.cpu(), src)
    src = torch.zeros(64, dtype=torch.uint8).pin_memory()
    dst = torch.zeros(64, dtype=torch.uint8, device=gpu_device)
    assert m.gpu_h2d_kernel(dst.data_ptr(), src.data_ptr(), 40, st, 64) != 0


@pytest.mark.parametrize("emit", ["full", "key_value"])
def test_batched_fire_gpu_equals_cpu(gpu_device, emit):
    """Watermark jumps over many slides fire a group of windows in one window_fire_many call
    (blockIdx.y = window, staging regions, pack kernel): the rows per window -- full 28-byte or
    compact 12-byte (uint32 key id + value) -- equal the C++ twin's, window by window."""
    from mxstream.ops import expr as E

    prog = E.compile_expr(E.var(E.VAR_RESULT) * 0.25)

    def run(dev):
        op = KeyedWindowOperator(size=60_000, slide=1_000, lateness=0, agg=K.AGG_SUM_I64,
                                 device=dev, max_keys=4096, batch_capacity=100_000,
                                 ooo_bound=100, dense_keys=True, map_prog=prog, emit=emit)
        rows = []
        for step in range(6):
            k = torch.empty(100_000, dtype=torch.int64, device=dev)
            t = torch.empty_like(k)
            v = torch.empty_like(k)
            # 30 s of event time per step: every step fires ~30 windows at once
            K.gen_events(k, t, v, seed=23, stream_id=0, idx0=step * 100_000, nkeys=3000,
                         ts_base=step * 30_000, ts_span=30_000, disorder=50, val_lo=0,
                         val_span=1000)
            rows += op.process(k, t, v)
        rows += op.finish()
        return [(r.window_start, sorted(zip(r.keys.tolist(), r.values.tolist()))) for r in rows]

    g, c = run(gpu_device), run("cpu")
    assert len(c) > 100
    assert g == c


def test_counted_d2h_copies_device_count(gpu_device):
    """gpu_d2h_counted: the copy kernel reads the row count on the device and moves only those
    rows (rounded to 16 bytes) of each column; fixed tensors travel whole."""
    from mxstream.runtime.window_operator import CountedHostRows, PinnedSlabPool

    cap = 4096
    a = torch.arange(cap, dtype=torch.int64, device=gpu_device) * 3
    b = torch.arange(cap, dtype=torch.int32, device=gpu_device) - 7
    flags = torch.tensor([5, 0, 1234, 0], dtype=torch.int32, device=gpu_device)
    n = torch.tensor([1234, 0, 0, 0], dtype=torch.int32, device=gpu_device)
    pool = PinnedSlabPool()
    t, arr = pool.take(1 << 16)
    arr[:] = 0xAB  # sentinel: rows past the count must stay untouched
    del t, arr
    rows = CountedHostRows(pool, [a, b], n[:1], [flags])
    rows.wait()
    assert rows.fixed(0).tolist() == [5, 0, 1234, 0]
    ca, cb = rows.columns(1234)
    assert np.array_equal(ca, a[:1234].cpu().numpy())
    assert np.array_equal(cb, b[:1234].cpu().numpy())
    # 1234 int64 rows = 9872 bytes (a 16-byte multiple): the next row was not copied
    off_a = rows.cols_meta[0][0]
    assert (rows.arr[off_a + 9872:off_a + 9880] == 0xAB).all()


@pytest.mark.parametrize("emit", ["full", "key_value"])
@pytest.mark.parametrize("pipeline", [False, "stream", True])
def test_async_fire_equals_sync_fire(gpu_device, emit, pipeline, monkeypatch):
    """Firings resolved later (device-counted copy, no host sync per firing; pipelined calls
    return only what has reached the host and queue the rest in order) emit exactly the
    synchronous path's firings and re-firings, in the same order, with batch tags that never
    precede the batch that triggered them."""

    def run(async_fire):
        monkeypatch.setenv("MXS_ASYNC_FIRE", "1" if async_fire else "0")
        op = KeyedWindowOperator(size=6000, slide=1000, lateness=3000, agg=K.AGG_SUM_I64,
                                 device=gpu_device, max_keys=100_000, batch_capacity=200_000,
                                 ooo_bound=500, dense_keys=True, emit=emit, pipeline=pipeline)
        assert op.async_fire == async_fire
        rows, tags = [], []
        for step in range(16):
            k = torch.empty(200_000, dtype=torch.int64, device=gpu_device)
            t = torch.empty_like(k)
            v = torch.empty_like(k)
            K.gen_events(k, t, v, seed=31, stream_id=0, idx0=step * 200_000, nkeys=80_000,
                         ts_base=step * 1000, ts_span=1000, disorder=500, val_lo=0,
                         val_span=1000)
            if step > 6:
                t[:10_000] -= 2500
            out = op.process(k, t, v)
            tags += [(step + 1, r.seq) for r in out]
            rows += out
        rows += op.finish()
        assert all(seq <= call for call, seq in tags)
        return [(r.window_start, r.refire, sorted(zip(r.keys.tolist(), r.values.tolist())))
                for r in rows]

    a, s = run(True), run(False)
    assert sum(1 for r in s if r[1]) > 5  # re-firings happened
    assert a == s


@pytest.mark.parametrize("emit", ["full", "key_value"])
def test_fused_refire_equals_per_window(gpu_device, emit, monkeypatch):
    """All windows a step re-fires in one pass over the touched-slot list (union of their panes
    loaded once per slot, map/filter epilogue per window) == one sweep per window."""
    prog = E.compile_expr(E.var(E.VAR_RESULT) * 0.5)
    filt = E.compile_expr(E.var(E.VAR_MAPPED) > 40.0)

    def run(fused):
        monkeypatch.setenv("MXS_FUSED_REFIRE", "1" if fused else "0")
        op = KeyedWindowOperator(size=6000, slide=1000, lateness=4000, agg=K.AGG_SUM_I64,
                                 device=gpu_device, max_keys=50_000, batch_capacity=100_000,
                                 ooo_bound=300, dense_keys=True, emit=emit, map_prog=prog,
                                 filter_prog=filt)
        rows = []
        for step in range(14):
            k = torch.empty(100_000, dtype=torch.int64, device=gpu_device)
            t = torch.empty_like(k)
            v = torch.empty_like(k)
            K.gen_events(k, t, v, seed=41, stream_id=0, idx0=step * 100_000, nkeys=40_000,
                         ts_base=step * 1000, ts_span=1000, disorder=300, val_lo=0, val_span=100)
            if step > 7:
                t[:8_000] -= 3500  # re-fires 3-4 already fired windows per step
            rows += op.process(k, t, v)
        rows += op.finish()
        return [(r.window_start, r.refire, sorted(zip(r.keys.tolist(), r.values.tolist())))
                for r in rows], op

    (f, fop), (u, _) = run(True), run(False)
    assert sum(1 for r in u if r[1]) > 10
    assert f == u
    assert fop.metrics.extra.get("refire_unfused", 0) == 0


@pytest.mark.parametrize("narrow", [True, False])
def test_sparse_pane_rows_equal_dense(gpu_device, narrow, monkeypatch):
    """A step whose records fall into a late pane and the current panes (empty panes between
    them) aggregates only the panes that have records (partition pane mask -> sparse LDS rows):
    every firing and re-firing equals the dense pane range's, and both equal the C++ twin."""

    def run(dev, sparse):
        monkeypatch.setenv("MXS_SPARSE_PANES", "1" if sparse else "0")
        op = KeyedWindowOperator(size=8000, slide=1000, lateness=6000, agg=K.AGG_SUM_I64,
                                 device=dev, max_keys=60_000, batch_capacity=150_000,
                                 ooo_bound=200, dense_keys=True,
                                 narrow=narrow if dev != "cpu" else False)
        rows = []
        for step in range(16):
            k = torch.empty(150_000, dtype=torch.int64, device=dev)
            t = torch.empty_like(k)
            v = torch.empty_like(k)
            K.gen_events(k, t, v, seed=43, stream_id=0, idx0=step * 150_000, nkeys=50_000,
                         ts_base=step * 1000, ts_span=1000, disorder=200, val_lo=0,
                         val_span=500)
            if step > 8:
                t[:9_000] -= 5200   # 5 panes back
                t[9_000:12_000] -= 3100  # and 3 panes back
            rows += op.process(k, t, v)
        rows += op.finish()
        return sorted((r.window_start, r.refire, int(a), int(b), int(c))
                      for r in rows for a, b, c in zip(r.keys, r.raw, r.counts))

    s, d, c = run(gpu_device, True), run(gpu_device, False), run("cpu", False)
    assert sum(1 for x in c if x[1]) > 1000
    assert s == d == c


@pytest.mark.parametrize("key_dtype", [torch.int32, torch.int64])
def test_two_level_partition_equals_plain(gpu_device, key_dtype, monkeypatch):
    """More than 512 sub-tables with 8-byte records: the two-level partition (LDS-staged compact
    kernel into 512 coarse buckets + per-coarse-bucket split into the fine buckets) fires
    exactly the plain scatter's rows, re-firings included; int32 key ids go through the
    compact kernel natively."""

    def run(two_level):
        monkeypatch.setenv("MXS_TWO_LEVEL", "1" if two_level else "0")
        op = KeyedWindowOperator(size=4000, slide=1000, lateness=2000, agg=K.AGG_SUM_I64,
                                 device=gpu_device, max_keys=3_000_000, batch_capacity=1 << 20,
                                 ooo_bound=300, dense_keys=True, narrow=True)
        assert op.nbuckets > 512 and op.two_level == two_level
        rows = []
        for step in range(9):
            k = torch.empty(1 << 20, dtype=key_dtype, device=gpu_device)
            t = torch.empty(1 << 20, dtype=torch.int64, device=gpu_device)
            v = torch.empty_like(t)
            K.gen_events(k, t, v, seed=47, stream_id=0, idx0=step << 20, nkeys=2_000_000,
                         ts_base=step * 1000, ts_span=1000, disorder=300, val_lo=0,
                         val_span=2000)
            if step > 4:
                t[:30_000] -= 2500
            rows += op.process(k, t, v)
        rows += op.finish()
        return sorted((r.window_start, r.refire, int(a), int(b), int(c))
                      for r in rows for a, b, c in zip(r.keys, r.raw, r.counts)), op

    (a, aop), (b, _) = run(True), run(False)
    assert len(a) > 100_000 and sum(1 for x in a if x[1]) > 1000
    assert a == b
    assert aop.metrics.bucket_regrows == 0


def test_window_rows_pane_sort(gpu_device):
    """window_rows_pane_sort: the first min(n, cap) rows grouped by pane (counts per pane), each
    pane's (key, acc, cnt, dirty) multiset unchanged; rows past n are ignored."""
    from mxstream.ops.native import load

    m = load()
    g = torch.Generator().manual_seed(7)
    cap, n, p_lo, np_ = 300_000, 271_113, 40, 11
    key = torch.randint(0, 1 << 40, (cap,), generator=g)
    pane = torch.randint(p_lo, p_lo + np_, (cap,), generator=g)
    pane[n:] = p_lo + 99  # beyond the count: must not be read as rows
    acc = torch.randint(-1000, 1000, (cap,), generator=g)
    cnt = torch.randint(1, 9, (cap,), generator=g, dtype=torch.int32)
    dirty = torch.randint(0, 2, (cap,), generator=g, dtype=torch.uint8)
    d = [t.to(gpu_device) for t in (key, pane, acc, cnt, dirty)]
    n_dev = torch.tensor([n], dtype=torch.int32, device=gpu_device)
    ok, oa = torch.empty_like(d[0]), torch.empty_like(d[2])
    oc, od = torch.empty_like(d[3]), torch.empty_like(d[4])
    counts = torch.empty(128, dtype=torch.int32, device=gpu_device)
    m.gpu_window_rows_pane_sort(d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(),
                                d[3].data_ptr(), d[4].data_ptr(), n_dev.data_ptr(), cap, p_lo,
                                np_, ok.data_ptr(), oa.data_ptr(), oc.data_ptr(), od.data_ptr(),
                                counts.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    c = counts[:np_].cpu().numpy()
    want_c = np.bincount(pane[:n].numpy() - p_lo, minlength=np_)
    assert np.array_equal(c, want_c)
    off = np.concatenate([[0], np.cumsum(c)])
    got = np.stack([ok.cpu().numpy()[:n], oa.cpu().numpy()[:n], oc.cpu().numpy()[:n],
                    od.cpu().numpy()[:n]], 1)
    src = np.stack([key.numpy()[:n], acc.numpy()[:n], cnt.numpy()[:n], dirty.numpy()[:n]], 1)
    for j in range(np_):
        a = got[off[j]:off[j + 1]]
        b = src[pane[:n].numpy() == p_lo + j]
        assert np.array_equal(a[np.lexsort(a.T[::-1])], b[np.lexsort(b.T[::-1])])


def test_hashed_narrow_steps_over_wide_table_keys_equal_cpu(gpu_device):
    """8-byte records fold against 32-bit LDS keys; a sub-table holding a key >= 2^32 - 1
    (restored from a checkpoint written by 16-byte steps) keeps 64-bit keys. Steps 1.. run
    narrow on a table restored with wide keys in most sub-tables: results equal the CPU twin's."""
    res = {}
    for d in (gpu_device, torch.device("cpu")):
        def op_for():
            return KeyedWindowOperator(size=2000, agg=K.AGG_SUM_I64, device=d, max_keys=20_000,
                                       batch_capacity=1 << 16, ooo_bound=300, cap_log2=9)
        op = op_for()
        keys, ts, vals = _gen(d, 1 << 16, 20_000, span=2500, disorder=300, seed=11)
        wide = torch.arange(keys.numel(), device=d) % 16 == 0
        keys = torch.where(wide, keys + (1 << 33), keys)  # ~4K wide keys: most sub-tables
        out = op.process(keys, ts, vals)
        snap = op.snapshot_state()
        op = op_for()
        op.restore_state(snap.columns, snap.meta)
        if d.type == "cuda":
            assert op.rec_w == 1  # the restored operator runs 8-byte records again
        for step in range(1, 5):
            keys, ts, vals = _gen(d, 1 << 16, 20_000, span=2500, disorder=300, seed=11 + step)
            ts += step * 2500
            out += op.process(keys, ts, vals)
        out += op.finish()
        res[d.type] = _results(out)
    assert res["cuda"] == res["cpu"]


@pytest.mark.parametrize("split", [2, 4])
def test_forced_agg_split_equals_default(gpu_device, split, monkeypatch):
    """MXS_AGG_FORCE_SPLIT (A/B knob): every dense sub-table folded by `split` workgroups whose
    partial sums merge with atomics (and the packed accumulators each share allows) gives the
    same windows as one workgroup per sub-table."""
    res = {}
    for n_split in (0, split):
        monkeypatch.setenv("MXS_AGG_FORCE_SPLIT", str(n_split))
        op = KeyedWindowOperator(size=2000, agg=K.AGG_SUM_I64, device=gpu_device,
                                 max_keys=1 << 16, batch_capacity=1 << 18, ooo_bound=300,
                                 dense_keys=True)
        out = []
        for step in range(4):
            keys, ts, vals = _gen(gpu_device, 1 << 18, 1 << 16, span=2500, disorder=300,
                                  seed=21 + step)
            ts += step * 2500
            out += op.process(keys, ts, vals)
        out += op.finish()
        res[n_split] = _results(out)
    assert res[0] == res[split]


@pytest.mark.gpu
def test_step_comm_stream_is_the_steps_stream():
    """The native step's collectives run on the step's own stream: for the legacy default stream
    (handle 0) that is torch's default stream, not whatever torch makes of ExternalStream(0)."""
    from mxstream.parallel.comm import LocalComm
    from mxstream.runtime.window_operator import _StepCommAdapter

    dev = torch.device("cuda", 0)
    ad = _StepCommAdapter(LocalComm(), dev)
    with ad._stream(0):
        assert torch.cuda.current_stream(dev).cuda_stream == \
            torch.cuda.default_stream(dev).cuda_stream
    s = torch.cuda.Stream(dev)
    with ad._stream(s.cuda_stream):
        assert torch.cuda.current_stream(dev).cuda_stream == s.cuda_stream
