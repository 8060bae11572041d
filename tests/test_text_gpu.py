"""GPU text parsing (K1/K2) vs the C++ runtime's Java-semantics parser (host reference)."""
import numpy as np
import pytest
import torch

from mxstream.ops import text as T
from mxstream.ops.native import load


def test_fnv_reserved_keys_and_ascii():
    assert T.fnv1a64(b"") == np.int64(np.uint64(0xcbf29ce484222325).astype(np.int64))
    assert T.fnv1a64(b"www.163.com") not in (-1, -2)


@pytest.mark.gpu
def test_parse_cpu_metrics_lines_bit_exact(gpu_device):
    rng = np.random.default_rng(5)
    n = 50_000
    hosts = [f"10.0.{i // 256}.{i % 256}" for i in range(500)] + ["主机-1", "srv"]
    usage = rng.uniform(0, 100, n)
    fmts = ["{:.1f}", "{:.3f}", "{}", "{:.0f}", "{:.2e}", "{:.4f}\t"]
    lines = []
    for i in range(n):
        u = fmts[i % len(fmts)].format(usage[i])
        if i % 997 == 0:
            u = "87.5d"          # Java suffix: host path
        if i % 1499 == 0:
            u = "123456789.123456789"  # > 15 significant digits: host path
        lines.append(f"{1563452056 + i} {hosts[i % len(hosts)]} cpu{i % 64} {u}")
    data = ("\n".join(lines) + "\r\n").encode()
    spec = [(0, T.FK_LONG), (1, T.FK_STR), (2, T.FK_STR), (3, T.FK_DOUBLE)]
    got = T.parse_text_gpu(data, spec, " ", 0, gpu_device)
    m = load()
    d = m.StringDict()
    ref, nref, err_idx, err = m.parse_lines(data, spec, " ", d, 0)
    assert not err and nref == n
    assert np.array_equal(got[0].cpu().numpy(), ref[0])
    assert np.array_equal(got[3].cpu().numpy().view(np.int64), np.asarray(ref[3]).view(np.int64))
    strings = d.strings()
    keys, jh = got[1]
    exp_keys = np.array([T.fnv1a64(strings[i].encode()) for i in ref[1].tolist()], dtype=np.int64)
    exp_jh = np.array([m.java_string_hash(strings[i]) for i in ref[1].tolist()], dtype=np.int32)
    assert np.array_equal(keys.cpu().numpy(), exp_keys)
    assert np.array_equal(jh.cpu().numpy(), exp_jh)


@pytest.mark.gpu
def test_parse_bandwidth_iso_lines(gpu_device):
    lines = ["2019-07-18T20:14:16 www.163.com 1024", "2019-07-18T20:14:16.250 www.qq.com 99",
             "2020-02-29T23:59:59 a 9223372036854775807", "1999-12-31T00:00 b -5"]
    data = "\n".join(lines).encode()
    spec = [(0, T.FK_TS_INTSEC), (0, T.FK_TS_MS), (2, T.FK_LONG)]
    got = T.parse_text_gpu(data, spec, " ", 8 * 3600, gpu_device)
    m = load()
    ref, *_ = m.parse_lines(data, spec, " ", m.StringDict(), 8 * 3600)
    for g, r in zip(got, ref):
        assert np.array_equal(g.cpu().numpy(), r)


@pytest.mark.gpu
def test_parse_error_has_java_text(gpu_device):
    data = b"1 h cpu1 12.5\n2 h cpu2 abc\n"
    with pytest.raises(T.ParseError, match="NumberFormatException"):
        T.parse_text_gpu(data, [(3, T.FK_DOUBLE)], " ", 0, gpu_device)
    with pytest.raises(T.ParseError, match="ArrayIndexOutOfBounds"):
        T.parse_text_gpu(b"1 h\n", [(3, T.FK_DOUBLE)], " ", 0, gpu_device)


@pytest.mark.gpu
def test_pinned_batch_matches_bytes(gpu_device):
    """A pinned host batch (the socket ring's slot) parses identically to the bytes path,
    including lines the kernel hands back to the host runtime."""
    lines = [f"{1563452056 + i} 10.8.{i % 7}.{i % 251} cpu{i % 64} {(i * 7.31) % 100:.2f}"
             for i in range(5000)]
    lines[17] = "1 h cpu1 87.5d"  # Java suffix: host patch path
    data = ("\n".join(lines) + "\n").encode()
    spec = [(0, T.FK_LONG), (1, T.FK_STR), (3, T.FK_DOUBLE)]
    a = T.parse_text_gpu(data, spec, " ", 0, gpu_device)
    pinned = T.pinned_text_batch(data)
    assert pinned.is_pinned()
    b = T.parse_text_gpu(pinned, spec, " ", 0, gpu_device)
    assert torch.equal(a[0], b[0]) and torch.equal(a[2], b[2])
    assert torch.equal(a[1][0], b[1][0]) and torch.equal(a[1][1], b[1][1])
