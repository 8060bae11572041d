"""Device text ingest + device string dictionary (ops/ingest.py, csrc/ingest*.{h,hip,cpp}).

CPU tests run the C++ twins; the GPU tests (marked gpu) run the gfx950 kernels and compare them
with the twins and with the host parser (``parse_lines`` + ``StringDict``), which is the
reference for Java parse semantics and for dictionary ids (first appearance order).
"""
import numpy as np
import pytest
import torch

from mxstream.ops import expr as E
from mxstream.ops.ingest import DeviceDict, DictionaryError, TextIngest, count_lines
from mxstream.ops.native import load

SPEC_CPU = [(1, 0), (2, 0), (3, 1), (0, 2)]       # host, cpu, usage (double), ts (long)
SPEC_BW = [(1, 0), (2, 2), (0, 3)]                # channel, bytes, ISO ts (int seconds * 1000)


def _cpu_lines(n, hosts, seed=0):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        h = hosts[int(rng.integers(0, len(hosts)))]
        u = rng.uniform(0, 100)
        fmt = rng.integers(0, 4)
        us = f"{u:.1f}" if fmt == 0 else f"{u:.17g}" if fmt == 1 else f"{int(u)}" if fmt == 2 else f"{u:.3e}"
        out.append(f"{1563452000 + i} {h} cpu{int(rng.integers(0, 8))} {us}")
    return out


def _host_parse(text, spec, d=None, offset_s=0):
    m = load()
    d = d if d is not None else m.StringDict()
    cols, n, ei, err = m.parse_lines(text, spec, " ", d, offset_s, 1)
    assert not err, err
    return cols, d


def _check_equal(res, host_cols, spec):
    for j, (_, k) in enumerate(spec):
        got = res.cols[j].cpu().numpy()
        want = host_cols[j]
        if k == 1:
            assert np.array_equal(got.view(np.int64), np.asarray(want, np.float64).view(np.int64))
        else:
            assert np.array_equal(got.astype(np.int64), np.asarray(want).astype(np.int64))


def _run_batches(device, batches, spec, ts_field=-1, offset_s=0):
    ing = TextIngest(spec, " ", offset_s=offset_s, ts_field=ts_field, device=device)
    m = load()
    d = m.StringDict()
    for text in batches:
        res = ing.parse(text)
        cols, _ = _host_parse(text, spec, d, offset_s)
        _check_equal(res, cols, spec)
    assert ing.dict.strings() == d.strings()
    assert np.array_equal(ing.dict.jhash_table(), d.jhash_table())
    return ing


def test_count_lines():
    assert count_lines(b"") == 0
    assert count_lines(b"a") == 1 and count_lines(b"a\n") == 1 and count_lines(b"a\n\nb") == 3
    assert count_lines(np.frombuffer(b"x\ny\n", np.uint8)) == 2


def test_ids_and_columns_equal_host_parser_over_batches():
    hosts = [f"10.8.{i // 256}.{i % 256}" for i in range(300)] + ["ü-host", "主机-1", "host\U0001F600"]
    batches = []
    for b in range(5):
        lines = _cpu_lines(700, hosts[: 60 * (b + 1)], seed=b)
        batches.append(("\n".join(lines) + ("\n" if b % 2 else "")).encode())
    ing = _run_batches("cpu", batches, SPEC_CPU, ts_field=3)
    assert ing.stats["flagged_lines"] > 0  # %.17g values leave the exact fast path


def test_bandwidth_iso_timestamps_and_max_ts():
    lines = [f"2019-08-28T10:{m:02d}:{s:02d} www.{c}.com {m * 100 + s}"
             for m in range(3) for s in range(0, 60, 7) for c in ("163", "qq", "sina")]
    text = "\n".join(lines).encode()
    ing = TextIngest(SPEC_BW, " ", offset_s=8 * 3600, ts_field=2, device="cpu")
    res = ing.parse(text)
    cols, _ = _host_parse(text, SPEC_BW, offset_s=8 * 3600)
    _check_equal(res, cols, SPEC_BW)
    assert res.max_ts == int(np.max(cols[2]))


def test_filter_compaction_in_input_order():
    lines = _cpu_lines(3000, ["a", "b", "c"], seed=3)
    text = "\n".join(lines).encode()
    prog = E.compile_expr((E.var(2) > 90) | (E.var(2) < 2.5))
    ing = TextIngest(SPEC_CPU, " ", ts_field=3, device="cpu", filter_prog=prog)
    res = ing.parse(text)
    cols, _ = _host_parse(text, SPEC_CPU)
    u = np.asarray(cols[2])
    keep = np.flatnonzero((u > 90) | (u < 2.5))
    assert res.n == keep.size and np.array_equal(res.line_idx.numpy(), keep)
    assert np.array_equal(res.cols[2].numpy(), u[keep])
    assert res.max_ts == int(np.max(cols[3]))  # the watermark sees every line


def test_parse_errors_raise_java_exceptions():
    from mxstream.api import java as J

    ing = TextIngest(SPEC_CPU, " ", ts_field=3, device="cpu")
    with pytest.raises(J.ArrayIndexOutOfBoundsException):
        ing.parse(b"1563452056 10.8.22.1 cpu0 1.0\n1563452056 10.8.22.1\n")
    with pytest.raises(J.NumberFormatException):
        ing.parse(b"1563452056 10.8.22.1 cpu0 abc\n")


def test_dictionary_growth_and_intern_many():
    d = DeviceDict("cpu", cap=8, id_cap=4, arena_cap=16)
    ing = TextIngest([(0, 0)], " ", device="cpu", dictionary=d)
    names = [f"key-{i}" for i in range(5000)]
    for lo in range(0, 5000, 1000):
        res = ing.parse(("\n".join(names[lo:lo + 1000] + names[:10])).encode())
        assert res.cols[0].tolist() == list(range(lo, lo + 1000)) + list(range(10))
    assert d.cap >= 2 * 5000 and len(d) == 5000 and d.strings() == names
    assert d.intern_many(["key-7", "fresh"]).tolist() == [7, 5000]
    assert d.get(5000) == "fresh"


def test_empty_batch_and_empty_strings():
    ing = TextIngest([(0, 0), (1, 2)], ",", device="cpu")
    assert ing.parse(b"").n == 0
    res = ing.parse(b",1\n,2\nx,3\n")
    assert res.cols[0].tolist() == [0, 0, 1] and ing.dict.strings() == ["", "x"]


def test_golden_jobs_through_device_ingest(monkeypatch):
    """The reference jobs' README outputs with the device ingest path (C++ twins here)."""
    import test_reference_jobs as R

    monkeypatch.setenv("MXS_TEXT_INGEST", "device")
    R.test_chapter1_map_print_readme()
    R.test_chapter1_filter_readme()
    R.test_chapter1_malformed_line_fails_job()
    R.test_compute_cpu_max_readme()
    R.test_compute_cpu_avg_readme()
    R.test_compute_cpu_middle_readme()
    R.test_bandwidth_monitor_tumbling_readme()
    R.test_bandwidth_event_time_readme("auto")


# ---- GPU --------------------------------------------------------------------------------------
@pytest.mark.gpu
def test_gpu_ingest_equals_host_parser_and_twins(gpu_device):
    hosts = [f"10.8.{i // 256}.{i % 256}" for i in range(2000)] + ["ü-host", "主机-1"]
    batches = []
    for b in range(4):
        lines = _cpu_lines(20_000, hosts[: 500 * (b + 1)], seed=10 + b)
        batches.append(("\n".join(lines) + "\n").encode())
    g = _run_batches(gpu_device, batches, SPEC_CPU, ts_field=3)
    c = _run_batches("cpu", batches, SPEC_CPU, ts_field=3)
    assert g.dict.strings() == c.dict.strings()
    assert g.stats["flagged_lines"] == c.stats["flagged_lines"] > 0


@pytest.mark.gpu
def test_gpu_ingest_filter_and_bandwidth(gpu_device):
    lines = [f"2019-08-28T10:{(i // 60) % 60:02d}:{i % 60:02d} ch{i % 977}.example.com {i * 37 % 100000}"
             for i in range(200_000)]
    text = "\n".join(lines).encode()
    prog = E.compile_expr(E.var(1) < 5000)
    for dev in (gpu_device, "cpu"):
        ing = TextIngest(SPEC_BW, " ", offset_s=8 * 3600, ts_field=2, device=dev, filter_prog=prog)
        res = ing.parse(text)
        cols, _ = _host_parse(text, SPEC_BW, offset_s=8 * 3600)
        keep = np.flatnonzero(np.asarray(cols[1]) < 5000)
        assert res.n == keep.size
        assert np.array_equal(res.line_idx.cpu().numpy(), keep)
        assert np.array_equal(res.cols[0].cpu().numpy().astype(np.int64), np.asarray(cols[0])[keep].astype(np.int64))
        assert np.array_equal(res.cols[1].cpu().numpy(), np.asarray(cols[1])[keep])
        assert res.max_ts == int(np.max(cols[2]))


@pytest.mark.gpu
def test_gpu_dictionary_growth_pinned_input(gpu_device):
    from mxstream.ops.text import pinned_text_batch

    d = DeviceDict(gpu_device, cap=16, id_cap=8, arena_cap=64)
    ing = TextIngest([(0, 0)], " ", device=gpu_device, dictionary=d)
    names = [f"key-{i}" for i in range(100_000)]
    for lo in range(0, 100_000, 25_000):
        res = ing.parse(pinned_text_batch(("\n".join(names[lo:lo + 25_000] + names[:10])).encode()))
        got = res.cols[0].cpu().tolist()
        assert got == list(range(lo, lo + 25_000)) + list(range(10))
    assert d.strings() == names
    assert d.intern_many(["key-7", "fresh"]).tolist() == [7, 100_000]


@pytest.mark.gpu
def test_golden_jobs_gpu_device_ingest(monkeypatch, gpu_device):
    import test_reference_jobs as R

    monkeypatch.setenv("MXS_DEVICE", "cuda")
    monkeypatch.setenv("MXS_TEXT_INGEST", "device")
    R.test_chapter1_map_print_readme()
    R.test_chapter1_filter_readme()
    R.test_chapter1_malformed_line_fails_job()
    R.test_compute_cpu_max_readme()
    R.test_compute_cpu_avg_readme()
    R.test_compute_cpu_middle_readme()
    R.test_bandwidth_monitor_tumbling_readme()
    R.test_bandwidth_monitor_sliding_readme()
    R.test_bandwidth_event_time_readme("auto")


_ = DictionaryError
