"""Order-preserving filter compaction (chapter1 `filter(usage > 90)`,
reference chapter1/src/main/java/me/zjy/Main.java:31): indices of the passing rows in input
order, GPU (mask/scan/write kernels) and C++ twin against a NumPy reference."""
import numpy as np
import pytest
import torch

from mxstream.ops import expr as E
from mxstream.ops import kernels as K


def _ref(x, thr):
    return np.nonzero(x > thr)[0]


@pytest.mark.parametrize("n", [0, 1, 1023, 1024, 1025, 100_003])
def test_filter_compact_cpu(n):
    x = np.random.default_rng(n).uniform(0, 100, n)
    idx, total = K.expr_filter_compact(torch.from_numpy(x), E.compile_expr(E.var(0) > 90))
    c = int(total.item())
    assert np.array_equal(idx[:c].numpy(), _ref(x, 90))


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 1000, 1024, 4097, 1 << 20, 3_000_001])
@pytest.mark.parametrize("thr", [-1.0, 50.0, 99.9, 200.0])
def test_filter_compact_gpu(n, thr):
    x = np.random.default_rng(n).uniform(0, 100, n)
    idx, total = K.expr_filter_compact(torch.from_numpy(x).cuda(),
                                       E.compile_expr(E.var(0) > thr))
    c = int(total.item())
    assert np.array_equal(idx[:c].cpu().numpy(), _ref(x, thr))
