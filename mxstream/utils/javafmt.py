"""Java-compatible text formatting for print() sinks.

Flink's PrintSinkFunction writes ``prefix + record.toString()`` (SURVEY.md F-print):
  * ``Tuple.toString()`` = ``(f0,f1,...)`` with no spaces;
  * ``Double.toString`` = shortest round-trip digits, plain notation for 1e-3 <= |x| < 1e7,
    otherwise ``d.dddE<exp>`` — e.g. ``86.26666666666667``, ``0.0012715657552083333``, ``1.0E7``;
  * the ``"{subtask+1}> "`` prefix appears only when the sink parallelism is > 1.
Golden outputs: chapter1/README.md:81-83,122; chapter2/README.md:63-65,162-163,246-247;
chapter3/README.md:295-296.
"""
from __future__ import annotations

import math

import numpy as np


class JDouble(float):
    """A float that prints like java.lang.Double (used for Double-typed tuple fields)."""

    def __str__(self):
        return java_double_str(float(self))

    __repr__ = __str__


class JLong(int):
    def __str__(self):
        return str(int(self))

    __repr__ = __str__


def java_double_str(x: float) -> str:
    if math.isnan(x):
        return "NaN"
    if math.isinf(x):
        return "Infinity" if x > 0 else "-Infinity"
    if x == 0.0:
        return "-0.0" if math.copysign(1.0, x) < 0 else "0.0"
    sign = "-" if x < 0 else ""
    ax = abs(x)
    digits, e10 = _shortest_digits(ax)
    if 1e-3 <= ax < 1e7:
        point = e10 + 1  # digits before the decimal point
        if point <= 0:
            return sign + "0." + "0" * (-point) + digits
        if point >= len(digits):
            return sign + digits + "0" * (point - len(digits)) + ".0"
        return sign + digits[:point] + "." + digits[point:]
    frac = digits[1:] or "0"
    return f"{sign}{digits[0]}.{frac}E{e10}"


def _shortest_digits(ax: float) -> tuple[str, int]:
    """Shortest round-trip decimal digits of ax > 0 and the exponent of the first digit, from
    repr() (CPython's correctly rounded shortest repr: the same digits as a unique-mode Dragon4,
    at a fraction of numpy.format_float_scientific's cost -- print sinks format every alert)."""
    r = repr(ax)
    e = 0
    if "e" in r:
        r, ex = r.split("e")
        e = int(ex)
    ip, _, fp = r.partition(".")
    d = ip + fp
    lead = len(d) - len(d.lstrip("0"))
    d = d[lead:].rstrip("0") or "0"
    return d, len(ip) + e - lead - 1


def _shortest_digits_numpy(ax: float) -> tuple[str, int]:
    s = np.format_float_scientific(ax, unique=True, trim="-")
    mant, exp = s.split("e")
    return mant.replace(".", ""), int(exp)


def java_str(v) -> str:
    """String.valueOf(v) for the value types the engine emits."""
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, (float, np.floating)) and not isinstance(v, JLong):
        return java_double_str(float(v))
    if isinstance(v, tuple):
        return tuple_str(v)
    return str(v)


def tuple_str(t) -> str:
    return "(" + ",".join(java_str(x) for x in t) + ")"


def print_prefix(subtask: int, parallelism: int) -> str:
    return f"{subtask + 1}> " if parallelism > 1 else ""
