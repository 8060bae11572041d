"""C ABI (csrc/mxs_c.h) of the native window pipeline (csrc/pipeline.cpp): golden chapter3 stream
from C, and a ctypes differential test against the Python KeyedWindowOperator (same kernels, same
state geometry -> identical firings)."""
import ctypes
import subprocess
from pathlib import Path

import numpy as np
import pytest
import torch

from mxstream.ops import kernels as K
from mxstream.runtime.window_operator import KeyedWindowOperator

ROOT = Path(__file__).resolve().parent.parent


class Cfg(ctypes.Structure):
    _fields_ = [("size_ms", ctypes.c_int64), ("slide_ms", ctypes.c_int64),
                ("offset_ms", ctypes.c_int64), ("lateness_ms", ctypes.c_int64),
                ("ooo_bound_ms", ctypes.c_int64), ("agg", ctypes.c_int32),
                ("device", ctypes.c_int32), ("device_index", ctypes.c_int32),
                ("max_parallelism", ctypes.c_int32), ("max_keys", ctypes.c_int64),
                ("batch_capacity", ctypes.c_int64)]


class Res(ctypes.Structure):
    _fields_ = [("window_start", ctypes.c_int64), ("window_end", ctypes.c_int64),
                ("key", ctypes.c_uint64), ("value", ctypes.c_double), ("raw", ctypes.c_int64),
                ("count", ctypes.c_uint32), ("refire", ctypes.c_int32)]


@pytest.fixture(scope="module")
def lib():
    from mxstream.build import build_capi

    path = build_capi()
    L = ctypes.CDLL(str(path))
    L.mxs_pipeline_create.restype = ctypes.c_void_p
    L.mxs_pipeline_create.argtypes = [ctypes.POINTER(Cfg)]
    L.mxs_pipeline_destroy.argtypes = [ctypes.c_void_p]
    L.mxs_pipeline_process.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                       ctypes.c_void_p, ctypes.c_int64]
    L.mxs_pipeline_finish.argtypes = [ctypes.c_void_p]
    L.mxs_pipeline_take_results.restype = ctypes.c_int64
    L.mxs_pipeline_take_results.argtypes = [ctypes.c_void_p, ctypes.POINTER(Res), ctypes.c_int64]
    L.mxs_pipeline_late_dropped.restype = ctypes.c_int64
    L.mxs_pipeline_late_dropped.argtypes = [ctypes.c_void_p]
    L.mxs_last_error.restype = ctypes.c_char_p
    L.mxs_window_config_default.argtypes = [ctypes.POINTER(Cfg)]
    return L


def _drain(L, p, out):
    buf = (Res * 4096)()
    while True:
        n = L.mxs_pipeline_take_results(p, buf, 4096)
        assert n >= 0
        if n == 0:
            return
        for r in buf[:n]:
            out[(r.window_start, r.key, r.refire)] = out.get((r.window_start, r.key, r.refire), []) \
                + [(r.raw, r.count)]


def _stream(steps=8, n=4000, nkeys=1500):
    out = []
    for s in range(steps):
        keys = torch.empty(n, dtype=torch.int64)
        ts = torch.empty_like(keys)
        vals = torch.empty_like(keys)
        K.gen_events(keys, ts, vals, seed=9, stream_id=0, idx0=s * n, nkeys=nkeys,
                     ts_base=s * 1500, ts_span=1500, disorder=2500, val_lo=0, val_span=1000)
        if s > 3:
            ts[::17] -= 4000  # late: dropped or (within the lateness) re-fired
        out.append((keys, ts, vals))
    return out


def _run_capi(L, stream, device, size, slide, lateness):
    cfg = Cfg()
    L.mxs_window_config_default(ctypes.byref(cfg))
    cfg.size_ms, cfg.slide_ms, cfg.lateness_ms, cfg.ooo_bound_ms = size, slide, lateness, 1000
    cfg.agg, cfg.device, cfg.max_keys, cfg.batch_capacity = K.AGG_SUM_I64, device, 1500, 4000
    p = L.mxs_pipeline_create(ctypes.byref(cfg))
    assert p, L.mxs_last_error()
    got = {}
    try:
        for keys, ts, vals in stream:
            k, t, v = (np.ascontiguousarray(x.numpy()) for x in (keys, ts, vals))
            rc = L.mxs_pipeline_process(p, k.ctypes.data, t.ctypes.data, v.ctypes.data, len(k))
            assert rc == 0, L.mxs_last_error()
            _drain(L, p, got)
        assert L.mxs_pipeline_finish(p) == 0
        _drain(L, p, got)
        late = L.mxs_pipeline_late_dropped(p)
    finally:
        L.mxs_pipeline_destroy(p)
    return got, late


@pytest.mark.parametrize("size,slide,lateness", [(3000, 3000, 0), (3000, 1000, 2000)])
def test_capi_equals_python_operator(lib, size, slide, lateness):
    stream = _stream()
    got, late = _run_capi(lib, stream, 0, size, slide, lateness)
    op = KeyedWindowOperator(size=size, slide=slide, lateness=lateness, agg=K.AGG_SUM_I64,
                             device="cpu", max_keys=1500, batch_capacity=4000, ooo_bound=1000)
    ref = {}
    for keys, ts, vals in stream:
        for r in op.process(keys, ts, vals):
            for k, a, c in zip(r.keys.tolist(), r.raw.tolist(), r.counts.tolist()):
                ref.setdefault((r.window_start, k, int(r.refire)), []).append((a, c))
    for r in op.finish():
        for k, a, c in zip(r.keys.tolist(), r.raw.tolist(), r.counts.tolist()):
            ref.setdefault((r.window_start, k, int(r.refire)), []).append((a, c))
    assert got == ref
    assert late == op.metrics.num_late_records_dropped


def test_capi_c_program_golden_chapter3(lib):
    libdir = Path(lib._name).parent
    exe = libdir / "capi_main"
    subprocess.run(["gcc", "-O1", "-Wall", f"-I{ROOT / 'csrc'}", str(ROOT / "csrc/tests/capi_main.c"),
                    f"-L{libdir}", "-lmxstream", f"-Wl,-rpath,{libdir}", "-o", str(exe)], check=True)
    res = subprocess.run([str(exe), "0"], capture_output=True, text=True, timeout=120)
    assert res.returncode == 0, res.stdout + res.stderr
    assert "12 x 10000" in res.stdout and "36 x 10200" in res.stdout


def test_capi_rejects_bad_config(lib):
    cfg = Cfg()
    lib.mxs_window_config_default(ctypes.byref(cfg))
    cfg.size_ms = 0
    assert not lib.mxs_pipeline_create(ctypes.byref(cfg))
    assert b"positive" in lib.mxs_last_error()


@pytest.mark.gpu
def test_capi_gpu_equals_host(lib, gpu_device):
    stream = _stream()
    a, la = _run_capi(lib, stream, 0, 3000, 1000, 2000)
    b, lb = _run_capi(lib, stream, 1, 3000, 1000, 2000)
    assert a == b and la == lb


class RCfg(ctypes.Structure):
    _fields_ = [("agg", ctypes.c_int32), ("device", ctypes.c_int32),
                ("device_index", ctypes.c_int32), ("reserved", ctypes.c_int32),
                ("max_keys", ctypes.c_int64), ("batch_capacity", ctypes.c_int64),
                ("count_window", ctypes.c_int64)]


class RRow(ctypes.Structure):
    _fields_ = [("key", ctypes.c_uint64), ("raw", ctypes.c_int64), ("index", ctypes.c_int64)]


def _rolling_lib(L):
    L.mxs_rolling_create.restype = ctypes.c_void_p
    L.mxs_rolling_create.argtypes = [ctypes.POINTER(RCfg)]
    L.mxs_rolling_destroy.argtypes = [ctypes.c_void_p]
    L.mxs_rolling_process.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                      ctypes.c_int64]
    L.mxs_rolling_take_rows.restype = ctypes.c_int64
    L.mxs_rolling_take_rows.argtypes = [ctypes.c_void_p, ctypes.POINTER(RRow), ctypes.c_int64]
    L.mxs_rolling_config_default.argtypes = [ctypes.POINTER(RCfg)]
    return L


def _run_rolling_capi(L, batches, device, agg, count_window):
    L = _rolling_lib(L)
    cfg = RCfg()
    L.mxs_rolling_config_default(ctypes.byref(cfg))
    cfg.agg, cfg.device, cfg.max_keys, cfg.batch_capacity = agg, device, 2000, 1024
    cfg.count_window = count_window
    r = L.mxs_rolling_create(ctypes.byref(cfg))
    assert r, L.mxs_last_error()
    out = []
    buf = (RRow * 8192)()
    try:
        for step, (keys, vals) in enumerate(batches):
            k, v = (np.ascontiguousarray(x.numpy()) for x in (keys, vals))
            assert L.mxs_rolling_process(r, k.ctypes.data, v.ctypes.data, len(k)) == 0, L.mxs_last_error()
            while True:
                n = L.mxs_rolling_take_rows(r, buf, 8192)
                if n <= 0:
                    break
                out += [(step, x.index, x.key, x.raw) for x in buf[:n]]
    finally:
        L.mxs_rolling_destroy(r)
    return out


@pytest.mark.parametrize("agg,count_window", [(K.AGG_SUM_I64, 0), (K.AGG_MAX_I64, 0),
                                              (K.AGG_COUNT, 0), (K.AGG_SUM_I64, 7),
                                              (K.AGG_AVG_I64, 16)])
def test_capi_rolling_equals_python_operator(lib, agg, count_window):
    """mxs_rolling_* (C++ control loop over the C++ twins) emits exactly the Python
    KeyedRollingOperator's rows, in input order (keyed rolling state and count windows)."""
    from mxstream.runtime.rolling_operator import KeyedRollingOperator

    batches = []
    for s in range(4):
        keys = torch.empty(5000, dtype=torch.int64)
        ts = torch.empty_like(keys)
        vals = torch.empty_like(keys)
        K.gen_events(keys, ts, vals, seed=3, stream_id=0, idx0=s * 5000, nkeys=1200,
                     ts_base=0, ts_span=1000, disorder=0, val_lo=-300, val_span=1000)
        batches.append((keys, vals))
    got = _run_rolling_capi(lib, batches, 0, agg, count_window)
    op = KeyedRollingOperator(agg=agg, device="cpu", max_keys=2000, batch_capacity=1024,
                              count_window=count_window)
    ref = []
    for step, (keys, vals) in enumerate(batches):
        rows = op.process(keys, vals)
        order = np.argsort(rows.tags & 0xFFFFFFFF, kind="stable")
        ref += [(step, int(rows.tags[i]) & 0xFFFFFFFF, int(rows.keys[i]), int(rows.values[i]))
                for i in order]
    assert got == ref and len(ref) > 0


@pytest.mark.gpu
@pytest.mark.parametrize("agg,count_window", [(K.AGG_SUM_I64, 0), (K.AGG_AVG_I64, 16)])
def test_capi_rolling_gpu_equals_host(lib, gpu_device, agg, count_window):
    batches = []
    for s in range(3):
        keys = torch.empty(40_000, dtype=torch.int64)
        ts = torch.empty_like(keys)
        vals = torch.empty_like(keys)
        K.gen_events(keys, ts, vals, seed=5, stream_id=0, idx0=s * 40_000, nkeys=1500,
                     ts_base=0, ts_span=1000, disorder=0, val_lo=0, val_span=1000)
        batches.append((keys, vals))
    assert _run_rolling_capi(lib, batches, 1, agg, count_window) == \
        _run_rolling_capi(lib, batches, 0, agg, count_window)


class SCfg(ctypes.Structure):
    _fields_ = [("gap_ms", ctypes.c_int64), ("lateness_ms", ctypes.c_int64),
                ("ooo_bound_ms", ctypes.c_int64), ("agg", ctypes.c_int32),
                ("reserved", ctypes.c_int32)]


class SRes(ctypes.Structure):
    _fields_ = [("key", ctypes.c_uint64), ("start", ctypes.c_int64), ("end", ctypes.c_int64),
                ("value", ctypes.c_double), ("raw", ctypes.c_int64), ("count", ctypes.c_uint32),
                ("refire", ctypes.c_int32)]


@pytest.mark.parametrize("agg", [K.AGG_SUM_I64, K.AGG_MAX_I64, K.AGG_COUNT])
@pytest.mark.parametrize("lateness", [0, 3_000])
def test_capi_sessions_equal_python_operator(lib, agg, lateness):
    """mxs_session_* (C ABI over the C++ session store core) emits exactly the Python
    KeyedSessionOperator's sessions (EventTimeSessionWindows, chapter3/README.md:412-428),
    including late-but-allowed re-firings."""
    from mxstream.runtime.session_operator import KeyedSessionOperator

    L = lib
    L.mxs_session_create.restype = ctypes.c_void_p
    L.mxs_session_create.argtypes = [ctypes.POINTER(SCfg)]
    L.mxs_session_destroy.argtypes = [ctypes.c_void_p]
    L.mxs_session_process.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                      ctypes.c_void_p, ctypes.c_int64]
    L.mxs_session_finish.argtypes = [ctypes.c_void_p]
    L.mxs_session_take_results.restype = ctypes.c_int64
    L.mxs_session_take_results.argtypes = [ctypes.c_void_p, ctypes.POINTER(SRes), ctypes.c_int64]
    L.mxs_session_late_dropped.restype = ctypes.c_int64
    L.mxs_session_late_dropped.argtypes = [ctypes.c_void_p]
    L.mxs_session_config_default.argtypes = [ctypes.POINTER(SCfg)]
    rng = np.random.default_rng(agg + lateness)
    n = 6000
    ts = np.sort(rng.integers(0, 120_000, n)) + rng.integers(-2_500, 2_500, n)  # disorder
    keys = rng.integers(0, 40, n)
    vals = rng.integers(0, 100, n)
    cfg = SCfg()
    L.mxs_session_config_default(ctypes.byref(cfg))
    cfg.gap_ms, cfg.lateness_ms, cfg.ooo_bound_ms, cfg.agg = 1_500, lateness, 1_000, agg
    s = L.mxs_session_create(ctypes.byref(cfg))
    assert s, L.mxs_last_error()
    op = KeyedSessionOperator(gap=1_500, lateness=lateness, agg=agg, device="cpu",
                              max_keys=64, batch_capacity=512, ooo_bound=1_000)
    got, want = [], []
    buf = (SRes * 4096)()

    def take():
        while True:
            m = L.mxs_session_take_results(s, buf, 4096)
            if m <= 0:
                break
            got.extend((x.key, x.start, x.end, x.raw, x.count) for x in buf[:m])

    def rows(r):
        want.extend((int(k), int(a), int(b), int(w), int(c))
                    for k, a, b, w, c in zip(r.keys, r.start, r.end, r.raw, r.counts))

    try:
        for i in range(0, n, 500):
            k, t, v = (np.ascontiguousarray(x[i:i + 500], dtype=np.int64) for x in (keys, ts, vals))
            assert L.mxs_session_process(s, k.ctypes.data, t.ctypes.data, v.ctypes.data,
                                         len(k)) == 0, L.mxs_last_error()
            take()
            rows(op.process(torch.from_numpy(k), torch.from_numpy(t), torch.from_numpy(v)))
        assert L.mxs_session_finish(s) == 0
        take()
        rows(op.finish())
        assert L.mxs_session_late_dropped(s) == op.metrics.num_late_records_dropped
    finally:
        L.mxs_session_destroy(s)
    assert len(want) > 100 and sorted(got) == sorted(want)
