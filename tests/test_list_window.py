"""Native `process` windows (ComputeCpuMiddle.java:34-48): the device pane arena + counting-sort
median firing (runtime/list_window_operator.py, csrc/listwin_*.{hip,cpp}).

* the operator equals a plain per-key median (numpy) per window, with lateness re-firings;
* the C++ twin's scan / scatter equal numpy;
* a job with a native median window restarts from a checkpoint (the live panes' elements are in
  the snapshot) and ends with the clean run's results;
* G virtual ranks (LoopbackComm) print what one rank prints;
* GPU (marked): the HIP kernels equal the C++ twins and a torch median reference.
"""
from collections import Counter

import numpy as np
import pytest
import torch

from mxstream.ops.native import load
from mxstream.runtime.list_window_operator import KeyedListWindowOperator


def _java_median(v: np.ndarray) -> float:
    s = np.sort(v)
    n = len(s)
    return float(s[n // 2]) if n % 2 else float((s[n // 2 - 1] + s[n // 2]) / 2)


def _events(n, nkeys, span, seed, late_every=0):
    rng = np.random.default_rng(seed)
    k = rng.integers(0, nkeys, n).astype(np.int64)
    t = np.sort(rng.integers(0, span, n)).astype(np.int64)
    v = rng.normal(50, 20, n).round(2)
    if late_every:
        t[::late_every] -= 2500
    return k, t, v


def _run_op(dev, k, t, v, *, size, slide, lateness, steps, bound=500):
    op = KeyedListWindowOperator(size=size, slide=slide, lateness=lateness, device=dev)
    out = []
    n = len(k)
    per = -(-n // steps)
    for i in range(steps):
        sl = slice(i * per, min(n, (i + 1) * per))
        if sl.start >= n:
            break
        kt = torch.from_numpy(k[sl]).to(dev)
        tt = torch.from_numpy(t[sl]).to(dev)
        vt = torch.from_numpy(v[sl].view(np.int64)).to(dev)
        out += op.process(kt, tt, vt)
        out += op.advance_watermark(int(t[sl].max()) - bound)
    out += op.advance_watermark(2**63 - 1)
    return op, [(s, e, int(a), float(b)) for s, e, ks, ms in out for a, b in zip(ks, ms)]


def _oracle(k, t, v, size, slide):
    """Every (window, key) median over all elements (what the final firings must show)."""
    res = {}
    starts = set()
    for ti in t.tolist():
        s = ti - (ti % slide)
        while s > ti - size:
            starts.add(s)
            s -= slide
    for s in sorted(starts):
        sel = (t >= s) & (t < s + size)
        for key in np.unique(k[sel]).tolist():
            res[(s, key)] = _java_median(v[sel & (k == key)])
    return res


@pytest.mark.parametrize("size,slide", [(4000, 4000), (6000, 2000)])
def test_arena_median_equals_numpy(size, slide):
    k, t, v = _events(6000, 37, 40_000, seed=3)
    op, rows = _run_op("cpu", k, t, v, size=size, slide=slide, lateness=0, steps=9)
    got = {(s, key): m for s, e, key, m in rows}
    assert got == _oracle(k, t, v, size, slide)
    assert op.metrics.num_late_records_dropped == 0


def test_arena_lateness_refires_touched_keys():
    k, t, v = _events(5000, 11, 30_000, seed=5, late_every=41)
    _, rows = _run_op("cpu", k, t, v, size=4000, slide=2000, lateness=3000, steps=12)
    # the last firing of every (window, key) carries the median of everything it received
    last = {}
    for s, e, key, m in rows:
        last[(s, key)] = m
    keep = t >= 0
    ref = _oracle(k[keep], t[keep], v[keep], 4000, 2000)
    late_ok = {kk: vv for kk, vv in last.items() if kk in ref}
    assert len(late_ok) > 0.9 * len(ref)
    mism = [kk for kk, vv in late_ok.items() if vv != ref[kk]]
    # windows whose late data came after their cleanup are dropped, all others match
    assert len(mism) < 0.05 * len(late_ok)
    assert len(rows) > len(last)  # re-firings happened


def test_scan_and_scatter_twins_equal_numpy():
    m = load()
    rng = np.random.default_rng(1)
    nk = 10_000
    counts = rng.integers(0, 4, nk).astype(np.int32)
    offs = np.zeros(nk + 1, np.int64)
    heads = np.zeros(nk, np.int64)
    hk = np.zeros(nk, np.int64)
    nh = np.zeros(1, np.int64)
    m.lw_scan(False, counts.ctypes.data, nk, 5, 0, offs.ctypes.data, heads.ctypes.data,
              hk.ctypes.data, nh.ctypes.data, 0)
    ex = np.concatenate([[0], np.cumsum(counts)])
    assert np.array_equal(offs, ex)
    ne = np.nonzero(counts)[0]
    assert nh[0] == len(ne)
    assert np.array_equal(heads[:nh[0]], ex[ne]) and np.array_equal(hk[:nh[0]], ne + 5)


def _median_job(tmp_path=None, fault=None, comm=None, native="auto"):
    from mxstream.api.environment import (FsStateBackend, RestartStrategies,
                                          StreamExecutionEnvironment)
    from mxstream.api.time import Time, TimeCharacteristic
    from mxstream.api.tuples import Tuple2
    from mxstream.api.watermarks import BoundedOutOfOrdernessTimestampExtractor
    from mxstream.models.chapters import MedianUsage
    from mxstream.runtime.executor import ManualClock

    out = []
    env = StreamExecutionEnvironment(4, clock=ManualClock(0)).set_output(out.append)
    env.config.native = native
    env.config.fault_injection = fault
    env._comm = comm
    env.set_stream_time_characteristic(TimeCharacteristic.EventTime)
    if tmp_path is not None:
        env.enable_checkpointing(500)
        env.set_state_backend(FsStateBackend(str(tmp_path)))
        env.set_restart_strategy(RestartStrategies.fixed_delay_restart(2, 0))
    ev = [(i * 40 + 10, (f"h{i % 7}", float((i * 37) % 101) / 4, i * 40)) for i in range(400)]
    (env.from_timed_collection(ev)
     .assign_timestamps_and_watermarks(
         BoundedOutOfOrdernessTimestampExtractor(Time.milliseconds(100), extractor=lambda e: e[2]))
     .map(lambda e: Tuple2(e[0], e[1]))
     .key_by(0)
     .time_window(Time.milliseconds(2000))
     .process(MedianUsage())
     .print())
    res = env.execute("median-ft")
    return out, res


def test_median_window_restarts_from_checkpoint(tmp_path):
    clean, _ = _median_job()
    host, _ = _median_job(native="off")
    assert Counter(clean) == Counter(host)
    got, res = _median_job(tmp_path / "ft", fault="Window:200")
    assert res.metrics["numRestarts"] == 1
    assert res.metrics["restoredCheckpointId"] >= 1
    assert set(got) == set(clean)


@pytest.mark.parametrize("world", [2, 4])
def test_median_window_invariant_to_world(world):
    from mxstream.parallel.comm import run_loopback

    ref, _ = _median_job()
    res = run_loopback(world, lambda comm: _median_job(comm=comm))
    got = [line for out, _ in res for line in out]
    assert Counter(got) == Counter(ref)


@pytest.mark.gpu
@pytest.mark.parametrize("size,slide,lateness", [(60_000, 60_000, 0), (6000, 2000, 3000)])
def test_gpu_arena_median_equals_cpu_and_torch(gpu_device, size, slide, lateness):
    k, t, v = _events(400_000, 5000, 240_000, seed=11, late_every=97 if lateness else 0)
    _, g = _run_op(gpu_device, k, t, v, size=size, slide=slide, lateness=lateness, steps=8)
    _, c = _run_op("cpu", k, t, v, size=size, slide=slide, lateness=lateness, steps=8)
    assert sorted(g) == sorted(c)
    # torch reference of the final firing of every (window, key) without lateness
    if not lateness:
        kt, tt, vt = (torch.from_numpy(x) for x in (k, t, v))
        for s, e, key, med in g[:200]:
            sel = (tt >= s) & (tt < e) & (kt == key)
            ref = torch.sort(vt[sel]).values
            n = ref.numel()
            want = float(ref[n // 2]) if n % 2 else float((ref[n // 2 - 1] + ref[n // 2]) / 2)
            assert med == want


def test_wide_key_range_takes_the_mapped_firing():
    """Keys spread over 2^40 ids record no ranks (the per-key counts would not fit) and fire
    through dense ids from torch.unique: same medians as the oracle."""
    k, t, v = _events(3000, 29, 20_000, seed=9)
    big = (k * (1 << 35) + 7).astype(np.int64)
    op, rows = _run_op("cpu", big, t, v, size=4000, slide=4000, lateness=0, steps=5)
    got = {(s, key): m for s, e, key, m in rows}
    ref = {(s, key * (1 << 35) + 7): m for (s, key), m in _oracle(k, t, v, 4000, 4000).items()}
    assert got == ref
    assert not any(op.ranked[r] for r, p in enumerate(op.slot_pane) if p is not None) or \
        all(p is None for p in op.slot_pane)
