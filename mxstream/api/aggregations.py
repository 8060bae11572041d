"""Builtin AggregateFunctions that the planner can run natively.

Each behaves exactly like the equivalent hand-written Flink AggregateFunction on the host path
(e.g. ``AvgAggregate(1)`` is ComputeCpuAvg.java:31-58: accumulator (count, sum), result
``sum / count`` or 0.0) and carries a ``native`` descriptor (kind, field) for the GPU/C++ path.
"""
from __future__ import annotations

from .functions import AggregateFunction


class BuiltinAggregate(AggregateFunction):
    native: tuple[str, int]


class SumAggregate(BuiltinAggregate):
    def __init__(self, field: int):
        self.field = field
        self.native = ("sum", field)

    def create_accumulator(self):
        return None

    def add(self, value, acc):
        x = value[self.field]
        return x if acc is None else acc + x

    def get_result(self, acc):
        return acc

    def merge(self, a, b):
        return b if a is None else (a if b is None else a + b)


class CountAggregate(BuiltinAggregate):
    def __init__(self, field: int = 0):
        self.native = ("count", field)

    def create_accumulator(self):
        return 0

    def add(self, value, acc):
        return acc + 1

    def get_result(self, acc):
        return acc

    def merge(self, a, b):
        return a + b


class AvgAggregate(BuiltinAggregate):
    """Tuple2<Integer count, Double sum> accumulator; result sum/count (0.0 when empty)."""

    def __init__(self, field: int):
        self.field = field
        self.native = ("avg", field)

    def create_accumulator(self):
        return (0, 0.0)

    def add(self, value, acc):
        return (acc[0] + 1, acc[1] + value[self.field])

    def get_result(self, acc):
        return 0.0 if acc[0] == 0 else acc[1] / acc[0]

    def merge(self, a, b):
        return (a[0] + b[0], a[1] + b[1])


class MinAggregate(BuiltinAggregate):
    def __init__(self, field: int):
        self.field = field
        self.native = ("min", field)

    def create_accumulator(self):
        return None

    def add(self, value, acc):
        x = value[self.field]
        return x if acc is None or x < acc else acc

    def get_result(self, acc):
        return acc

    def merge(self, a, b):
        if a is None:
            return b
        if b is None:
            return a
        return a if a <= b else b


class MaxAggregate(MinAggregate):
    def __init__(self, field: int):
        self.field = field
        self.native = ("max", field)

    def add(self, value, acc):
        x = value[self.field]
        return x if acc is None or x > acc else acc

    def merge(self, a, b):
        if a is None:
            return b
        if b is None:
            return a
        return a if a >= b else b


class VectorSumAggregate(BuiltinAggregate):
    """Element-wise sum of a metric-vector field (list/tuple of floats, e.g. one usage value
    per CPU core). Host path: a list accumulator; native path: the MFMA vector-window kernel
    (runtime/vector_window_operator.py). The result is a list of floats."""

    kind = "vsum"

    def __init__(self, field: int):
        self.field = field
        self.native = (self.kind, field)

    def create_accumulator(self):
        return (0, None)

    def add(self, value, acc):
        x = [float(v) for v in value[self.field]]
        n, s = acc
        if s is None:
            return (n + 1, x)
        if len(x) != len(s):
            raise ValueError("metric vectors of one key must have the same length")
        return (n + 1, [a + b for a, b in zip(s, x)])

    def get_result(self, acc):
        return [] if acc[1] is None else list(acc[1])

    def merge(self, a, b):
        if a[1] is None:
            return b
        if b[1] is None:
            return a
        return (a[0] + b[0], [x + y for x, y in zip(a[1], b[1])])


class VectorAvgAggregate(VectorSumAggregate):
    """Element-wise average of a metric-vector field (ComputeCpuAvg.java:31-58 per vector
    component: accumulator (count, sums), result sums / count)."""

    kind = "vavg"

    def get_result(self, acc):
        n, s = acc
        return [] if s is None else [v / n for v in s]
