"""Stack-free chain evaluation of traced epilogues (csrc/mxs_common.h expr_eval_chain): same
double ops in the same order as the stack VM, so results are bit-identical."""
import random

from mxstream.ops import expr as E
from mxstream.ops.native import load


def _args(prog):
    code, consts = prog.as_args()
    return list(code), list(consts)


def test_reference_epilogues_are_chains():
    m = load()
    mbps = E.compile_expr(E.var(E.VAR_RESULT) * 8.0 / 60 / 1024 / 1024)
    flt = E.compile_expr(E.var(E.VAR_MAPPED) < 100.0)
    assert m.expr_is_chain(*_args(mbps)) and m.expr_is_chain(*_args(flt))
    # not a chain: the running value is the right operand of a nested sub-expression
    nested = E.compile_expr((E.var(0) + 1.0) * (E.var(1) - 2.0))
    assert not m.expr_is_chain(*_args(nested))


def test_chain_equals_vm_bitwise():
    m = load()
    rng = random.Random(7)
    ops = [lambda a, c: a * c, lambda a, c: a / c, lambda a, c: a + c, lambda a, c: a - c]
    for _ in range(300):
        e = E.var(rng.randrange(7))
        for _ in range(rng.randrange(1, 6)):
            c = rng.choice([8.0, 60.0, 1024.0, 0.1, 3.0, rng.uniform(-5, 5)])
            e = rng.choice(ops)(e, c)
        if rng.random() < 0.5:
            e = e < rng.uniform(-100, 100)
        code, consts = _args(E.compile_expr(e))
        if not m.expr_is_chain(code, consts):
            continue
        vars_ = [rng.uniform(-1e6, 1e6) for _ in range(8)]
        a = m.expr_eval(code, consts, vars_)
        b = m.expr_eval_chain(code, consts, vars_)
        assert a == b or (a != a and b != b)
