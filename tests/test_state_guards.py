"""Keyed-state guards: a full table, the reserved key ids and mis-shaped inputs fail loudly.

A key that finds no slot used to be dropped silently (the sticky flags[0] bit was never read);
the reserved ids -1 / -2 (empty-slot and tombstone markers) used to be "stored" in an empty slot
and lost. Every operator now reports both through the step's one host sync.
"""
import pytest
import torch

from mxstream.ops import kernels as K
from mxstream.runtime.rolling_operator import KeyedRollingOperator
from mxstream.runtime.window_operator import KeyedWindowOperator


def _devs():
    return [pytest.param("cpu", id="cpu"), pytest.param("cuda", id="gpu", marks=pytest.mark.gpu)]


def _skip(dev):
    if dev == "cuda" and not torch.cuda.is_available():
        pytest.skip("no GPU")


def _cols(dev, keys, t0=0):
    d = torch.device(dev)
    k = torch.as_tensor(keys, dtype=torch.int64, device=d)
    ts = torch.arange(k.numel(), dtype=torch.int64, device=d) + t0
    v = torch.ones_like(k)
    return k, ts, v


@pytest.mark.parametrize("dev", _devs())
@pytest.mark.parametrize("pipeline", [False, True])
def test_window_table_full_raises(dev, pipeline):
    _skip(dev)
    # 1 sub-table of 64 slots: 500 distinct keys cannot fit.
    op = KeyedWindowOperator(size=1000, agg=K.AGG_SUM_I64, device=dev, max_keys=16,
                             batch_capacity=4096, cap_log2=6, pipeline=pipeline)
    assert op.nslots < 500
    with pytest.raises(RuntimeError, match="table full"):
        op.process(*_cols(dev, range(500)))
        op.process(*_cols(dev, range(500), t0=600))
        op.finish()


@pytest.mark.parametrize("dev", _devs())
@pytest.mark.parametrize("bad", [-1, -2])
def test_window_reserved_key_raises(dev, bad):
    _skip(dev)
    op = KeyedWindowOperator(size=1000, agg=K.AGG_SUM_I64, device=dev, max_keys=1000,
                             batch_capacity=4096, cap_log2=8)
    with pytest.raises(ValueError, match="reserved"):
        op.process(*_cols(dev, [1, 2, bad, 3]))
        op.finish()


@pytest.mark.parametrize("dev", _devs())
def test_rolling_table_full_raises(dev):
    _skip(dev)
    op = KeyedRollingOperator(agg=K.AGG_COUNT, device=dev, max_keys=16, batch_capacity=4096,
                              cap_log2=6)
    k, _, v = _cols(dev, range(op.nslots + 200))
    with pytest.raises(RuntimeError, match="table full"):
        op.process(k, v)


@pytest.mark.parametrize("dev", _devs())
@pytest.mark.parametrize("bad", [-1, -2])
def test_rolling_reserved_key_raises(dev, bad):
    _skip(dev)
    op = KeyedRollingOperator(agg=K.AGG_SUM_I64, device=dev, max_keys=100, batch_capacity=64,
                              cap_log2=8)
    k, _, v = _cols(dev, [5, bad, 7])
    with pytest.raises(ValueError, match="reserved"):
        op.process(k, v)


@pytest.mark.gpu
def test_rolling_direct_path_validates_inputs():
    """The single-rank GPU path reads the columns by pointer: wrong dtype / device / length must
    raise before the kernel launch (it used to be a GPU fault)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    d = torch.device("cuda", 0)
    op = KeyedRollingOperator(agg=K.AGG_SUM_I64, device=d, max_keys=100, batch_capacity=64)
    k = torch.arange(10, dtype=torch.int64, device=d)
    with pytest.raises(TypeError):
        op.process(k, torch.ones(10, dtype=torch.int32, device=d))
    with pytest.raises(ValueError):
        op.process(k, torch.ones(10, dtype=torch.int64))  # host tensor
    with pytest.raises(ValueError):
        op.process(k, torch.ones(5, dtype=torch.int64, device=d))


def test_session_reserved_key_raises():
    from mxstream.runtime.session_operator import KeyedSessionOperator

    op = KeyedSessionOperator(gap=10, agg=K.AGG_SUM_I64, device="cpu", max_keys=100,
                              batch_capacity=64, cap_log2=8)
    with pytest.raises(ValueError, match="reserved"):
        op.process(*_cols("cpu", [1, -2, 3]))
