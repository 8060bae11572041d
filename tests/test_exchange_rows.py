"""parallel/exchange.py exchange_rows: the packed-row exchange of the keyed operators without a
record partition of their own (the median pane arena at G > 1, ComputeCpuMiddle.java:34-48).

Every rank sends random rows of several columns (int64, float64, and a 2-wide int32 column) to
random destinations; each rank must receive exactly the rows addressed to it, in (source rank,
source row) order -- the stable order that keeps every key's rows in arrival order. Checked
against a plain PyTorch reference of the routing, on the C++ twin (CPU) and on the gfx950 kernels.
"""
import pytest
import torch

from mxstream.parallel.comm import run_loopback
from mxstream.parallel.exchange import exchange_rows


def _rows(rank, world, n, dev):
    g = torch.Generator().manual_seed(1000 + rank)
    dest = torch.randint(0, world, (n,), generator=g)
    a = torch.arange(n, dtype=torch.int64) + rank * 1_000_000
    b = torch.randn(n, generator=g, dtype=torch.float64)
    c = torch.randint(-5, 5, (n, 2), generator=g, dtype=torch.int32)
    return dest.to(dev), [a.to(dev), b.to(dev), c.to(dev)]


def _expected(me, world, sizes):
    outs = [[], [], []]
    for r in range(world):
        dest, cols = _rows(r, world, sizes[r], "cpu")
        sel = dest == me
        for k in range(3):
            outs[k].append(cols[k][sel])
    return [torch.cat(o) for o in outs]


def _check(world, sizes, dev):
    def rank(comm):
        dest, cols = _rows(comm.rank, world, sizes[comm.rank], dev)
        return [t.cpu() for t in exchange_rows(comm, dest, cols)]

    res = run_loopback(world, rank, device=torch.device(dev) if dev != "cpu" else None)
    for me, got in enumerate(res):
        want = _expected(me, world, sizes)
        for g, w in zip(got, want):
            assert g.dtype == w.dtype and g.shape == w.shape
            assert torch.equal(g, w)


@pytest.mark.parametrize("world,sizes", [(2, [500, 700]), (3, [0, 2500, 40]),
                                         (4, [3000, 3000, 1, 0]), (8, [300] * 8)])
def test_exchange_rows_routes_stably_cpu(world, sizes):
    _check(world, sizes, "cpu")


def test_exchange_rows_no_rows_anywhere():
    def rank(comm):
        dest = torch.empty(0, dtype=torch.int64)
        return exchange_rows(comm, dest, [torch.empty(0, dtype=torch.int64)])

    for got in run_loopback(2, rank):
        assert got[0].numel() == 0


def test_exchange_rows_rejects_bad_destination():
    def rank(comm):
        dest = torch.tensor([0, 5], dtype=torch.int64)
        return exchange_rows(comm, dest, [torch.zeros(2, dtype=torch.int64)])

    with pytest.raises(ValueError, match="destination"):
        run_loopback(2, rank)


@pytest.mark.gpu
@pytest.mark.parametrize("world,sizes", [(2, [5000, 7000]), (4, [70_000, 1, 0, 33_333]),
                                         (8, [4096] * 8)])
def test_gpu_exchange_rows_routes_stably(world, sizes, gpu_device):
    _check(world, sizes, "cuda")
