"""Multi-threaded host parse (csrc/runtime.cpp parse_lines, threads > 1) == the serial parse:
same columns, same dictionary ids (first-appearance order over the batch), same error line."""
import numpy as np
import pytest

from mxstream.ops.native import load


def _text(n, seed=3, bad_at=None):
    rng = np.random.default_rng(seed)
    hosts = [f"10.8.{i // 256}.{i % 256}" for i in range(300)]
    lines = [f"1563452056 {hosts[rng.integers(0, 300)]} cpu{rng.integers(0, 64)} "
             f"{rng.uniform(0, 100):.1f}" for _ in range(n)]
    if bad_at is not None:
        lines[bad_at] = "1563452056 10.8.22.1"  # too few fields
    return ("\r\n".join(lines[: n // 2]) + "\n" + "\n".join(lines[n // 2:]) + "\n").encode()


@pytest.mark.parametrize("threads", [2, 3, 8, 64])
def test_parse_threads_equal_serial(threads):
    m = load()
    data = _text(20_000)
    spec = [(1, 0), (2, 0), (3, 1), (0, 2)]
    d1, d2 = m.StringDict(), m.StringDict()
    d1.intern("preexisting")
    d2.intern("preexisting")
    c1, n1, e1, _ = m.parse_lines(data, spec, " ", d1, 0)
    c2, n2, e2, _ = m.parse_lines(data, spec, " ", d2, 0, threads)
    assert (n1, e1) == (n2, e2) == (20_000, -1)
    for a, b in zip(c1, c2):
        assert np.array_equal(a, b)
    assert d1.strings() == d2.strings()


@pytest.mark.parametrize("bad_at", [0, 7_777, 19_999])
def test_parse_threads_first_error(bad_at):
    m = load()
    data = _text(20_000, bad_at=bad_at)
    spec = [(1, 0), (3, 1)]
    d1, d2 = m.StringDict(), m.StringDict()
    c1, n1, e1, msg1 = m.parse_lines(data, spec, " ", d1, 0)
    c2, n2, e2, msg2 = m.parse_lines(data, spec, " ", d2, 0, 8)
    assert (n1, e1, msg1) == (n2, e2, msg2) == (bad_at, bad_at, msg1)
    assert "ArrayIndexOutOfBoundsException" in msg1
    for a, b in zip(c1, c2):
        assert np.array_equal(a[:bad_at], b[:bad_at])
    assert d1.strings() == d2.strings()
