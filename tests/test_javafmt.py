"""Java Double.toString / Tuple.toString formatting of print sinks (SURVEY.md F-ser, F-print;
golden values chapter2/README.md:162, chapter3/README.md:295-296)."""
import math
import random
import struct

from mxstream.utils.javafmt import (_shortest_digits, _shortest_digits_numpy, java_double_str,
                                    java_str)


def test_golden_values():
    assert java_double_str(86.26666666666667) == "86.26666666666667"
    assert java_double_str(0.0012715657552083333) == "0.0012715657552083333"
    assert java_double_str(0.0012969970703125) == "0.0012969970703125"
    assert java_double_str(1e7) == "1.0E7" and java_double_str(9999999.0) == "9999999.0"
    assert java_double_str(1e-3) == "0.001" and java_double_str(9.99e-4) == "9.99E-4"
    assert java_double_str(100.0) == "100.0" and java_double_str(-0.0) == "-0.0"
    assert java_double_str(float("nan")) == "NaN" and java_double_str(-math.inf) == "-Infinity"
    assert java_str(("www.163.com", 11200)) == "(www.163.com,11200)"


def test_repr_digits_equal_dragon4_unique():
    """The fast repr()-based digits equal numpy's unique-mode Dragon4 on random doubles."""
    rng = random.Random(5)
    vals = [5e-324, 1.7976931348623157e308, 1e22, 1e23, 0.1, 123456789.0]
    while len(vals) < 50_000:
        x = struct.unpack("d", struct.pack("Q", rng.getrandbits(64)))[0]
        if math.isfinite(x) and x != 0.0:
            vals.append(abs(x))
        vals.append(round(rng.uniform(0, 1000), rng.randint(0, 8)) or 1.0)
    for x in vals:
        assert _shortest_digits(x) == _shortest_digits_numpy(x), x


def test_native_bulk_format_equals_python():
    """csrc/javafmt.h (the print sink's columnar path) formats exactly like javafmt.py."""
    import numpy as np

    from mxstream.ops.native import load

    m = load()
    rng = random.Random(11)
    vals = [86.26666666666667, 0.0012715657552083333, 1e7, 9999999.0, 1e-3, 9.99e-4, 100.0,
            -0.0, 0.0, float("nan"), math.inf, -math.inf, 5e-324, 1.7976931348623157e308, 1e22,
            1e23, 0.1, -123456789.0, 12.5]
    while len(vals) < 20_000:
        x = struct.unpack("d", struct.pack("Q", rng.getrandbits(64)))[0]
        vals.append(x if not math.isnan(x) else 1.5)
        vals.append(round(rng.uniform(-1000, 1000), rng.randint(0, 8)))
    for x in vals:
        assert m.java_double_str(x) == java_double_str(x), x
    n = 1000
    d = np.array(vals[:n], dtype=np.float64)
    ids = np.array([i % 3 for i in range(n)], dtype=np.int64)
    longs = np.array([rng.randint(-2**63, 2**63 - 1) for _ in range(n)], dtype=np.int64)
    sub = np.array([i % 4 for i in range(n)], dtype=np.int32)
    names = ["www.a.com", "b", "ü-utf8"]
    pre = [f"{k + 1}> " for k in range(4)]
    got = m.java_format_rows([(0, ids.ctypes.data), (1, d.ctypes.data), (2, longs.ctypes.data)],
                             n, names, sub.ctypes.data, pre, True)
    want = [pre[i % 4] + java_str((names[i % 3], float(d[i]), int(longs[i]))) for i in range(n)]
    assert got == want


def test_print_sink_columnar_path_equals_records():
    """A native window job's fired rows reach print() as one column batch: the printed lines
    equal the per-record path (native off) line for line."""
    from mxstream.api.environment import StreamExecutionEnvironment
    from mxstream.models import chapters as C

    lines = []
    for i in range(3000):
        c = (i * 7) % 23
        v = 40 + (i % 11) if c % 7 == 0 else 5_000_000 + (i * 7919) % 1_000_000
        lines.append(f"2019-08-28T{10 + i // 3600:02d}:{(i // 60) % 60:02d}:{i % 60:02d} "
                     f"www.ch{c}.com {v}")

    def run(native):
        out = []
        env = StreamExecutionEnvironment(4).set_output(out.append)
        env.config.native = native
        C.build_bandwidth_event_time(env, env.from_collection(lines, batch_size=500))
        env.execute("bw")
        return out

    ref = run("off")
    got = run("auto")
    assert len(ref) > 20 and sorted(got) == sorted(ref)
