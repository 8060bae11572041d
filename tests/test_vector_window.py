"""Vector-metric keyed windows (runtime/vector_window_operator.py, csrc/vector_*.{hip,cpp}).

Reference semantics: per (key, window) sum / average of the D-float metric vectors of the window's
elements (ComputeCpuAvg.java:27-59 generalised to per-core vectors), compared against a plain
numpy float64 reference. The GPU tests compare the MFMA kernel (and its VALU twin) against the same
reference and against the C++ twin.
"""
import numpy as np
import pytest
import torch

from mxstream.ops import kernels as K
from mxstream.ops import vector as V
from mxstream.runtime.vector_window_operator import VectorWindowOperator


def _events(dev, n, nkeys, dim, *, seed, span, disorder, t0=0, skew=False):
    keys = torch.empty(n, dtype=torch.int64, device=dev)
    ts = torch.empty_like(keys)
    vals = torch.empty_like(keys)
    K.gen_events(keys, ts, vals, seed=seed, stream_id=0, idx0=seed * n, nkeys=nkeys, ts_base=t0,
                 ts_span=span, disorder=disorder, val_lo=0, val_span=1)
    if skew:  # a hot key holding ~1/3 of the events (long runs across MFMA tiles)
        keys[::3] = 7
    vec = torch.empty(n, dim, dtype=torch.float32, device=dev)
    V.gen_vectors(vec, seed=seed, stream_id=0, idx0=seed * n, lo=-50.0, span=150.0)
    return keys, ts, vec


def _reference(batches, size, slide, avg):
    """{(window start, key): (vector f64, count)} with Flink window assignment (no lateness:
    the streams below are in order up to the watermark bound)."""
    acc = {}
    for keys, ts, vec in batches:
        k, t, v = keys.cpu().numpy(), ts.cpu().numpy(), vec.cpu().numpy().astype(np.float64)
        for i in range(len(k)):
            last = t[i] - (t[i] % slide)
            s = last
            while s > t[i] - size:
                a = acc.setdefault((s, int(k[i])), [np.zeros(v.shape[1]), 0])
                a[0] += v[i]
                a[1] += 1
                s -= slide
    return {key: (a / c if avg else a, c) for key, (a, c) in acc.items()}


def _collect(out):
    res = {}
    for r in out:
        for k, vec, c in zip(r.keys.tolist(), r.values, r.counts.tolist()):
            res[(r.window_start, int(k))] = (np.asarray(vec, dtype=np.float64), int(c))
    return res


def _run(dev, batches, *, size, slide, dim, avg=True, mfma=True, threshold=None):
    op = VectorWindowOperator(dim=dim, size=size, slide=slide, device=dev, max_keys=5000,
                              batch_capacity=max(b[0].numel() for b in batches), ooo_bound=400,
                              avg=avg, mfma=mfma, threshold=threshold)
    out = []
    for keys, ts, vec in batches:
        out += op.process(keys.to(dev), ts.to(dev), vec.to(dev))
    out += op.finish()
    return _collect(out), op


def _assert_close(got, ref, rtol=2e-5):
    assert got.keys() == ref.keys()
    for key, (v, c) in ref.items():
        gv, gc = got[key]
        assert gc == c, key
        scale = np.maximum(np.abs(v), 1.0)
        assert np.all(np.abs(gv - v) <= rtol * scale * max(1.0, np.sqrt(c))), key


def _batches(dev, dim, nb=4, n=6000, nkeys=700, skew=False):
    out = []
    for b in range(nb):
        out.append(_events(dev, n, nkeys, dim, seed=b + 1, span=1000, disorder=300,
                           t0=b * 1000 + 1000, skew=skew))
    return out


@pytest.mark.parametrize("size,slide", [(1000, 1000), (1500, 500)])
@pytest.mark.parametrize("avg", [True, False])
def test_cpu_twin_matches_reference(size, slide, avg):
    batches = _batches("cpu", 32)
    got, op = _run("cpu", batches, size=size, slide=slide, dim=32, avg=avg)
    _assert_close(got, _reference(batches, size, slide, avg))
    assert op.metrics.num_late_records_dropped == 0


def test_cpu_wide_vectors_and_threshold():
    batches = _batches("cpu", 64, nb=2)
    ref = _reference(batches, 1000, 1000, True)
    got, _ = _run("cpu", batches, size=1000, slide=1000, dim=64, threshold=55.0)
    want = {k: v for k, v in ref.items() if v[0].max() > 55.0}
    assert 0 < len(want) < len(ref)
    _assert_close(got, want)


def test_dim_validation():
    with pytest.raises(ValueError):
        VectorWindowOperator(dim=48, size=1000, device="cpu")
    with pytest.raises(TypeError):
        VectorWindowOperator(dim=32, size=1000, device="cpu", agg=K.AGG_SUM_F64)


def test_checkpoint_roundtrip_cpu(tmp_path):
    from mxstream.runtime.checkpoint import read_operator_rows, write_operator_file

    batches = _batches("cpu", 32, nb=2)
    op = VectorWindowOperator(dim=32, size=3000, device="cpu", max_keys=5000,
                              batch_capacity=6000, ooo_bound=400)
    op.process(*batches[0])
    snap = op.snapshot_state()
    # the async freeze (D2D clones of the vector state) exports the same rows
    frozen = op.snapshot_state_async()
    op.process(*batches[1])  # mutate the live state after the freeze
    snap_a = frozen()
    for c in snap.columns:
        assert snap.columns[c].tobytes() == snap_a.columns[c].tobytes(), c
    op = VectorWindowOperator(dim=32, size=3000, device="cpu", max_keys=5000,
                              batch_capacity=6000, ooo_bound=400)
    op.process(*batches[0])
    name = write_operator_file(tmp_path, "vec", 0, snap, 128)
    rows = read_operator_rows(tmp_path, [name], 0, 127)
    op2 = VectorWindowOperator(dim=32, size=3000, device="cpu", max_keys=5000,
                               batch_capacity=6000, ooo_bound=400)
    op2.restore_state(rows, snap.meta)
    a = _collect(op.process(*batches[1]) + op.finish())
    b = _collect(op2.process(*batches[1]) + op2.finish())
    assert a.keys() == b.keys()
    for k in a:
        assert a[k][1] == b[k][1]
        np.testing.assert_allclose(a[k][0], b[k][0], rtol=1e-6)


# ---- GPU: MFMA kernel ------------------------------------------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("dim", [32, 96])
@pytest.mark.parametrize("mfma", [True, False])
def test_gpu_matches_reference_and_twin(gpu_device, dim, mfma):
    batches = _batches(gpu_device, dim)
    ref = _reference(batches, 1500, 500, True)
    got, _ = _run(gpu_device, batches, size=1500, slide=500, dim=dim, mfma=mfma)
    _assert_close(got, ref)
    cpu_b = [tuple(t.cpu() for t in b) for b in batches]
    twin, _ = _run("cpu", cpu_b, size=1500, slide=500, dim=dim)
    _assert_close(got, {k: v for k, v in twin.items()})


@pytest.mark.gpu
def test_gpu_hot_key_runs_span_tiles(gpu_device):
    """A key with 1/3 of the events: its run covers many 32-record tiles and LDS rounds."""
    batches = _batches(gpu_device, 32, nb=2, n=40_000, skew=True)
    ref = _reference(batches, 1000, 1000, False)
    got, _ = _run(gpu_device, batches, size=1000, slide=1000, dim=32, avg=False)
    _assert_close(got, ref, rtol=1e-4)


@pytest.mark.gpu
def test_gpu_gen_vectors_bit_exact(gpu_device):
    a = torch.empty(1000, 32, dtype=torch.float32, device=gpu_device)
    b = torch.empty(1000, 32, dtype=torch.float32)
    V.gen_vectors(a, seed=5, stream_id=2, idx0=77)
    V.gen_vectors(b, seed=5, stream_id=2, idx0=77)
    assert torch.equal(a.cpu(), b)
