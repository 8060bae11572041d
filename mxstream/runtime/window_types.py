"""Result records of the keyed window operator (runtime/window_operator.py) and the aggregate
helpers of its checkpoint half (window_state.py).
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np
import torch

from ..ops import kernels as K

I64_MIN = K.I64_MIN
I64_MAX = K.I64_MAX


def _agg_identity(agg: int) -> int:
    """agg_identity (csrc/mxs_common.h) as an int64 bit pattern."""
    if agg == K.AGG_MIN_I64:
        return I64_MAX
    if agg == K.AGG_MAX_I64:
        return I64_MIN
    if agg == K.AGG_MIN_F64:
        return 0x7FF0000000000000
    if agg == K.AGG_MAX_F64:
        return 0xFFF0000000000000 - (1 << 64)
    return 0


def combine_partials(agg: int, acc: torch.Tensor, inv: torch.Tensor, n: int) -> torch.Tensor:
    """Fold rows of exported accumulators (int64 bit patterns) into n groups (`inv`: group of
    each row) with the aggregate's combine: sum / min / max over int64 or float64 values."""
    f64 = agg in (K.AGG_SUM_F64, K.AGG_AVG_F64, K.AGG_MIN_F64, K.AGG_MAX_F64)
    x = acc.view(torch.float64) if f64 else acc
    if agg in (K.AGG_MIN_I64, K.AGG_MIN_F64, K.AGG_MAX_I64, K.AGG_MAX_F64):
        is_min = agg in (K.AGG_MIN_I64, K.AGG_MIN_F64)
        init = (float("inf") if is_min else float("-inf")) if f64 else (I64_MAX if is_min else I64_MIN)
        out = torch.full((n,), init, dtype=x.dtype, device=x.device)
        out.scatter_reduce_(0, inv, x, "amin" if is_min else "amax")
    else:
        out = torch.zeros(n, dtype=x.dtype, device=x.device).index_add_(0, inv, x)
    return out.view(torch.int64) if f64 else out


@dataclass
class FireResult:
    window_start: int
    window_end: int
    keys: np.ndarray        # uint64 key ids (dictionary ids for string keys; uint32 ids for
                            # emit="key_value")
    values: np.ndarray      # float64 (result after the fused map epilogue)
    raw: np.ndarray | None  # int64 raw accumulator (exact integer sums / f64 bit pattern)
    counts: np.ndarray | None  # int32 element counts (raw / counts: None for emit="key_value")
    refire: bool = False
    seq: int = 0            # the operator's batch count when the firing was triggered (1-based
                            # process() call; latency accounting of deferred results)


@dataclass
class OperatorMetrics:
    num_records_in: int = 0
    num_late_records_dropped: int = 0
    num_records_out: int = 0
    num_fires: int = 0
    current_watermark: int = I64_MIN
    steps: int = 0
    bucket_regrows: int = 0
    ring_regrows: int = 0
    extra: dict = field(default_factory=dict)
