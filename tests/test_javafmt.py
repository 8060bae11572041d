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
