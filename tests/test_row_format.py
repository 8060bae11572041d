"""Device row formatter (csrc/row_format.h + csrc/format_hip.hip, ops/rowfmt.py) against the host
formatter (csrc/javafmt.h: Double.toString shortest digits, Long / String, Tuple.toString,
subtask prefixes). The C++ twin runs here; the gfx950 kernels in the gpu-marked test."""
import numpy as np
import pytest
import torch

from mxstream.ops.ingest import DeviceDict, TextIngest
from mxstream.ops.native import load
from mxstream.ops.rowfmt import RowFormatter
from mxstream.ops.text import FK_DOUBLE, FK_LONG, FK_STR
from mxstream.runtime.columnar import DeviceColumnBatch


def _host_format(cols, kinds, names, sub, prefixes, as_tuple):
    """The host formatter's bytes for numpy columns (the print sink's host path)."""
    keep, spec = [], []
    for c, k in zip(cols, kinds):
        if k == FK_STR:
            a = np.ascontiguousarray(c, dtype=np.int64)
            spec.append((0, a.ctypes.data))
        elif k == FK_DOUBLE:
            a = np.ascontiguousarray(c, dtype=np.float64)
            spec.append((1, a.ctypes.data))
        else:
            a = np.ascontiguousarray(c, dtype=np.int64)
            spec.append((2, a.ctypes.data))
        keep.append(a)
    s = np.ascontiguousarray(sub, dtype=np.int32)
    return load().java_format_bytes(spec, len(cols[0]), names, s.ctypes.data, prefixes, as_tuple, 1)


def _decimals(rng, n):
    """Parsed-metric style doubles: short decimals in plain notation, signs, integers."""
    ip = rng.integers(0, 10_000_000, n)
    fd = rng.integers(0, 7, n)
    frac = rng.integers(0, 10 ** 6, n) // 10 ** (6 - fd)
    txt = [f"{'-' if s else ''}{i}.{str(f).zfill(d) if d else '0'}"
           for s, i, f, d in zip(rng.integers(0, 2, n), ip, frac, fd)]
    v = np.array([float(t) for t in txt])
    v = v[(np.abs(v) >= 1e-3) & (np.abs(v) < 1e7) | (v == 0)]
    small = rng.integers(1, 1000, 200) / 1000.0  # 0.001 .. 0.999
    return np.concatenate([v, small, -small, [0.0, -0.0, 1.0, 9999999.5, 0.001]])


def _batch(cols, kinds, strings=None, sub=None):
    return DeviceColumnBatch(len(cols[0]), [torch.as_tensor(c) for c in cols], kinds, strings,
                             None, sub_dev=None if sub is None else torch.as_tensor(sub))


@pytest.mark.parametrize("as_tuple", [True, False])
def test_doubles_equal_host_formatter(as_tuple):
    rng = np.random.default_rng(3)
    v = _decimals(rng, 20_000)
    sub = rng.integers(0, 4, v.size).astype(np.int32)
    pfx = ["1> ", "2> ", "3> ", "4> "]
    cb = _batch([v], (FK_DOUBLE,), sub=sub)
    got = RowFormatter().format(cb, pfx, as_tuple)
    assert got is not None
    assert bytes(got) == _host_format([v], (FK_DOUBLE,), None, sub, pfx, as_tuple)


def test_long_digit_doubles_go_to_the_host():
    """17-digit doubles and scientific notation are flagged (the batch is formatted on the host)."""
    f = RowFormatter()
    for x in (0.1 + 0.2, 1e7, 1.5e-4, 123456.78901234567, float("inf"), float("nan")):
        cb = _batch([np.array([1.5, x])], (FK_DOUBLE,))
        got = f.format(cb, [""], True)
        special = x != x or x in (float("inf"),)
        if special:  # NaN / Infinity have fixed texts
            assert bytes(got) == _host_format([np.array([1.5, x])], (FK_DOUBLE,), None,
                                              np.zeros(2, np.int32), [""], True)
        else:
            assert got is None


def test_strings_longs_prefixes_equal_host_formatter():
    rng = np.random.default_rng(5)
    d = DeviceDict("cpu")
    names = [f"10.8.{i}.{i % 7}" for i in range(300)] + ["www.ch%d.com" % i for i in range(50)]
    ids = TextIngest([(0, FK_STR)], sep="\n", device="cpu", dictionary=d).parse(
        ("\n".join(names) + "\n").encode()).cols[0].to(torch.int64).numpy()
    assert ids.tolist() == list(range(len(names)))
    n = 5000
    k = rng.integers(0, len(names), n).astype(np.int32)
    lv = rng.integers(-(1 << 62), 1 << 62, n)
    lv[:3] = [np.iinfo(np.int64).min, 0, np.iinfo(np.int64).max]
    dv = _decimals(rng, n)[:n]
    sub = rng.integers(0, 3, n).astype(np.int32)
    pfx = ["1> ", "2> ", "3> "]
    cb = _batch([k, lv, dv], (FK_STR, FK_LONG, FK_DOUBLE), strings=d, sub=sub)
    got = RowFormatter().format(cb, pfx, True)
    want = _host_format([k, lv, dv], (FK_STR, FK_LONG, FK_DOUBLE), names, sub, pfx, True)
    assert bytes(got) == want
    bad = _batch([np.array([0, len(names) + 5], np.int32)], (FK_STR,), strings=d)
    assert RowFormatter().format(bad, [""], True) is None  # id outside the dictionary


def test_print_sink_uses_device_formatter(monkeypatch):
    """A reference job with device ingest prints through the device formatter (C++ twin here),
    with the golden output of the host path."""
    from mxstream.ops import rowfmt
    from mxstream.runtime import operators as O

    used = {"n": 0}
    orig = rowfmt.RowFormatter.format

    def spy(self, *a, **k):
        r = orig(self, *a, **k)
        used["n"] += r is not None
        return r

    def run(device_format):
        from mxstream.api.environment import StreamExecutionEnvironment
        from mxstream.models import chapters as C
        from mxstream.runtime.executor import ManualClock

        monkeypatch.setattr(O, "_DEVICE_FORMAT", device_format)
        out = []
        env = StreamExecutionEnvironment(4, clock=ManualClock(0)).set_output(out.append)
        env.config.native = "auto"
        env.config.text_ingest = "device"
        lines = [f"{1563452000 + i} 10.8.{i % 9}.{i % 3} cpu{i % 4} {((i * 37) % 400) / 4.0}"
                 for i in range(400)]
        C.build_compute_cpu_max(env, env.from_collection(lines, batch_size=64))
        env.execute("ComputeCpuMax")
        return out

    monkeypatch.setattr(rowfmt.RowFormatter, "format", spy)
    a = run(True)
    assert used["n"] > 0
    b = run(False)
    assert a == b and len(a) == 400


@pytest.mark.gpu
def test_gpu_row_format_equals_host(gpu_device):
    rng = np.random.default_rng(9)
    d = DeviceDict("cuda")
    names = [f"host-{i}" for i in range(1000)]
    TextIngest([(0, FK_STR)], sep="\n", device="cuda", dictionary=d).parse(
        ("\n".join(names) + "\n").encode())
    n = 300_000
    k = rng.integers(0, len(names), n).astype(np.int32)
    dv = _decimals(rng, n)[:n]
    lv = rng.integers(-(1 << 40), 1 << 40, dv.size)
    k = k[:dv.size]
    sub = rng.integers(0, 4, dv.size).astype(np.int32)
    pfx = ["1> ", "2> ", "3> ", "4> "]
    cb = DeviceColumnBatch(dv.size, [torch.as_tensor(c).cuda() for c in (k, lv, dv)],
                           (FK_STR, FK_LONG, FK_DOUBLE), d, None,
                           sub_dev=torch.as_tensor(sub).cuda())
    got = RowFormatter().format(cb, pfx, True)
    assert got is not None
    assert bytes(got) == _host_format([k, lv, dv], (FK_STR, FK_LONG, FK_DOUBLE), names, sub,
                                      pfx, True)
