"""Expression tracing and the bytecode of the in-kernel expression VM.

User map/filter lambdas over numeric fields (e.g. the Mbps conversion and the `< 100` alert of
``BandwidthMonitorWithEventTime.java:48-55``, the ``value.f2 > 90`` filter of ``Main.java:31``)
are traced by calling them with proxy objects. The resulting expression tree is compiled to
(op, arg) pairs + a constant pool and evaluated per row inside the fused HIP kernels
(``csrc/mxs_common.h: expr_eval``) with Java double semantics: one rounding per operation, no
contraction. A numpy evaluator with identical semantics serves host-side fallbacks and tests.
"""
from __future__ import annotations

import math
import operator
from dataclasses import dataclass
from typing import Any, Callable, Sequence

import numpy as np

# Opcodes — keep in sync with csrc/mxs_common.h (ExprOp).
OP_END, OP_VAR, OP_CONST = 0, 1, 2
OP_ADD, OP_SUB, OP_MUL, OP_DIV = 3, 4, 5, 6
OP_LT, OP_LE, OP_GT, OP_GE, OP_EQ, OP_NE = 7, 8, 9, 10, 11, 12
OP_AND, OP_OR, OP_NOT, OP_NEG, OP_ABS, OP_MIN, OP_MAX, OP_MOD, OP_TOINT = range(13, 22)

MAX_CODE = 64
MAX_CONST = 16

# Variables visible to window epilogues (csrc/mxs_common.h).
VAR_RESULT, VAR_COUNT, VAR_WSTART, VAR_WEND, VAR_KEY, VAR_RAW, VAR_MAPPED = range(7)
NVARS = 8


class TraceError(Exception):
    """The function cannot be expressed in the expression VM (host fallback is used)."""


_BINOPS = {
    "+": OP_ADD, "-": OP_SUB, "*": OP_MUL, "/": OP_DIV, "<": OP_LT, "<=": OP_LE, ">": OP_GT,
    ">=": OP_GE, "==": OP_EQ, "!=": OP_NE, "&": OP_AND, "|": OP_OR, "%": OP_MOD,
    "min": OP_MIN, "max": OP_MAX,
}
_UNOPS = {"!": OP_NOT, "neg": OP_NEG, "abs": OP_ABS, "toint": OP_TOINT}


class Expr:
    """Node of a traced numeric expression."""

    __slots__ = ("op", "args", "value")

    def __init__(self, op: str, args: tuple = (), value: Any = None):
        self.op = op
        self.args = args
        self.value = value

    # -- construction helpers -------------------------------------------------------------
    @staticmethod
    def lift(x) -> "Expr":
        if isinstance(x, Expr):
            return x
        if isinstance(x, bool):
            return Expr("const", value=1.0 if x else 0.0)
        if isinstance(x, (int, float, np.integer, np.floating)):
            return Expr("const", value=float(x))
        raise TraceError(f"cannot lift {type(x).__name__} into an expression")

    def _bin(self, op, other, swap=False):
        a, b = (Expr.lift(other), self) if swap else (self, Expr.lift(other))
        return Expr(op, (a, b))

    __add__ = lambda s, o: s._bin("+", o)
    __radd__ = lambda s, o: s._bin("+", o, True)
    __sub__ = lambda s, o: s._bin("-", o)
    __rsub__ = lambda s, o: s._bin("-", o, True)
    __mul__ = lambda s, o: s._bin("*", o)
    __rmul__ = lambda s, o: s._bin("*", o, True)
    __truediv__ = lambda s, o: s._bin("/", o)
    __rtruediv__ = lambda s, o: s._bin("/", o, True)
    __mod__ = lambda s, o: s._bin("%", o)
    __rmod__ = lambda s, o: s._bin("%", o, True)
    __lt__ = lambda s, o: s._bin("<", o)
    __le__ = lambda s, o: s._bin("<=", o)
    __gt__ = lambda s, o: s._bin(">", o)
    __ge__ = lambda s, o: s._bin(">=", o)
    __and__ = lambda s, o: s._bin("&", o)
    __rand__ = lambda s, o: s._bin("&", o, True)
    __or__ = lambda s, o: s._bin("|", o)
    __ror__ = lambda s, o: s._bin("|", o, True)

    def __eq__(self, o):  # type: ignore[override]
        return self._bin("==", o)

    def __ne__(self, o):  # type: ignore[override]
        return self._bin("!=", o)

    def __neg__(self):
        return Expr("neg", (self,))

    def __pos__(self):
        return self

    def __abs__(self):
        return Expr("abs", (self,))

    def __invert__(self):
        return Expr("!", (self,))

    def __float__(self):
        raise TraceError("float() of a traced value (use the value directly)")

    def __bool__(self):
        raise TraceError("data-dependent control flow (and/or/if) cannot be traced; use & | ~")

    def __hash__(self):
        return id(self)

    def __floordiv__(self, o):
        raise TraceError("// has Python floor semantics; use / or mxstream.functions.to_long")

    def __repr__(self):
        if self.op == "var":
            return f"v{self.value}"
        if self.op == "const":
            return repr(self.value)
        return f"({self.op} {' '.join(map(repr, self.args))})"


def var(i: int) -> Expr:
    return Expr("var", value=int(i))


def const(c: float) -> Expr:
    return Expr.lift(c)


def emin(a, b) -> Expr:
    return Expr("min", (Expr.lift(a), Expr.lift(b)))


def emax(a, b) -> Expr:
    return Expr("max", (Expr.lift(a), Expr.lift(b)))


def to_long(a) -> Expr:
    """Java `(long)` cast of a double (truncation toward zero)."""
    return Expr("toint", (Expr.lift(a),))


def substitute(e: Expr, mapping: dict[int, Expr]) -> Expr:
    """Replace variables (used to compose map -> filter chains)."""
    if e.op == "var":
        return mapping.get(e.value, e)
    if e.op == "const":
        return e
    return Expr(e.op, tuple(substitute(a, mapping) for a in e.args), e.value)


@dataclass(frozen=True)
class Program:
    code: tuple[int, ...]
    consts: tuple[float, ...]

    @property
    def empty(self) -> bool:
        return len(self.code) == 0

    def as_args(self) -> tuple[list[int], list[float]]:
        return list(self.code), list(self.consts)


EMPTY = Program((), ())


def compile_expr(e: Expr | None) -> Program:
    if e is None:
        return EMPTY
    code: list[int] = []
    consts: list[float] = []

    def emit(n: Expr):
        if n.op == "var":
            code.extend((OP_VAR, n.value))
        elif n.op == "const":
            v = float(n.value)
            for i, c in enumerate(consts):
                if c == v and math.copysign(1.0, c) == math.copysign(1.0, v):
                    code.extend((OP_CONST, i))
                    break
            else:
                consts.append(v)
                code.extend((OP_CONST, len(consts) - 1))
        elif n.op in _UNOPS:
            emit(n.args[0])
            code.extend((_UNOPS[n.op], 0))
        elif n.op in _BINOPS:
            emit(n.args[0])
            emit(n.args[1])
            code.extend((_BINOPS[n.op], 0))
        else:
            raise TraceError(f"unknown node {n.op}")

    emit(e)
    if len(code) // 2 > MAX_CODE or len(consts) > MAX_CONST:
        raise TraceError("expression too large for the kernel VM")
    return Program(tuple(code), tuple(consts))


_NP_BIN: dict[int, Callable] = {
    OP_ADD: np.add, OP_SUB: np.subtract, OP_MUL: np.multiply,
    OP_LT: np.less, OP_LE: np.less_equal, OP_GT: np.greater, OP_GE: np.greater_equal,
    OP_EQ: np.equal, OP_NE: np.not_equal, OP_MIN: np.minimum, OP_MAX: np.maximum,
}


def eval_numpy(prog: Program, vars_: Sequence[np.ndarray | float]) -> np.ndarray | float:
    """Evaluate a program over numpy columns with the kernel VM's semantics."""
    st: list = []
    code = prog.code
    with np.errstate(all="ignore"):
        for i in range(0, len(code), 2):
            op, arg = code[i], code[i + 1]
            if op == OP_VAR:
                st.append(np.asarray(vars_[arg], dtype=np.float64))
            elif op == OP_CONST:
                st.append(np.float64(prog.consts[arg]))
            elif op == OP_NOT:
                st[-1] = (st[-1] == 0.0).astype(np.float64)
            elif op == OP_NEG:
                st[-1] = -st[-1]
            elif op == OP_ABS:
                st[-1] = np.abs(st[-1])
            elif op == OP_TOINT:
                st[-1] = np.trunc(st[-1])
            else:
                b = st.pop()
                a = st[-1]
                if op == OP_DIV:
                    r = np.divide(a, b)
                elif op == OP_MOD:
                    r = np.fmod(a, b)
                elif op == OP_AND:
                    r = np.logical_and(a != 0.0, b != 0.0)
                elif op == OP_OR:
                    r = np.logical_or(a != 0.0, b != 0.0)
                else:
                    r = _NP_BIN[op](a, b)
                st[-1] = np.asarray(r, dtype=np.float64)
    return st[-1] if st else np.float64(0.0)


# ---- tuple tracing --------------------------------------------------------------------------

class FieldRef:
    """A non-numeric passthrough field of a traced row (e.g. the String key)."""

    __slots__ = ("name",)

    def __init__(self, name: str):
        self.name = name

    def __repr__(self):
        return f"<field {self.name}>"

    def __bool__(self):
        raise TraceError("non-numeric field used in a condition")

    def _no(self, *a):
        raise TraceError(f"arithmetic on non-numeric field {self.name}")

    __add__ = __radd__ = __sub__ = __rsub__ = __mul__ = __rmul__ = _no
    __truediv__ = __rtruediv__ = __lt__ = __le__ = __gt__ = __ge__ = _no


class RowProxy(tuple):
    """Tuple of Expr/FieldRef handed to user lambdas during tracing; supports t[i] and t.fN."""

    def __new__(cls, fields):
        return super().__new__(cls, fields)

    def __getattr__(self, name):
        if name.startswith("f") and name[1:].isdigit():
            return self[int(name[1:])]
        raise AttributeError(name)


def trace_row_fn(fn: Callable, row: Sequence) -> Any:
    try:
        return fn(RowProxy(row))
    except TraceError:
        raise
    except Exception as e:  # any python-level failure means "not traceable"
        raise TraceError(f"tracing failed: {type(e).__name__}: {e}") from e


_ = operator  # re-exported for callers composing expressions
