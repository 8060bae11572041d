"""Flink ``TupleN`` equivalents: Python tuples with ``f0..fN`` accessors and Java ``toString``.

``Tuple.toString()`` prints ``(f0,f1,...)`` and ``Tuple1<String>.hashCode() == f0.hashCode()``
— what keyBy(0) hashes (ComputeCpuMax.java:26).
"""
from __future__ import annotations

from ..utils.javafmt import JDouble, JLong, java_str


class Tuple(tuple):
    def __getattr__(self, name):
        if len(name) > 1 and name[0] == "f" and name[1:].isdigit():
            i = int(name[1:])
            if i < len(self):
                return self[i]
        raise AttributeError(name)

    def set_field(self, pos: int, value) -> "Tuple":
        return type(self)(self[:pos] + (value,) + self[pos + 1:])

    def __str__(self):
        return "(" + ",".join(java_str(x) for x in self) + ")"

    __repr__ = __str__

    def arity(self) -> int:
        return len(self)


def Tuple1(a):
    return Tuple((a,))


def Tuple2(a, b):
    return Tuple((a, b))


def Tuple3(a, b, c):
    return Tuple((a, b, c))


def Tuple4(a, b, c, d):
    return Tuple((a, b, c, d))


def Tuple5(a, b, c, d, e):
    return Tuple((a, b, c, d, e))


class Types:
    """Java boxed types used to make Python values print/hash like the reference's fields."""

    @staticmethod
    def DOUBLE(x) -> JDouble:
        return JDouble(x)

    @staticmethod
    def LONG(x) -> JLong:
        return JLong(x)

    @staticmethod
    def INT(x) -> int:
        return int(x)

    @staticmethod
    def STRING(x) -> str:
        return str(x)
