"""Validated launch wrappers of the vector-metric window kernels (csrc/vector_hip.hip: MFMA
segmented sums on gfx950; csrc/vector_cpu.cpp: C++ twins).

Same contract as ``ops/kernels.py``: every operand's dtype, device, contiguity and the sizes the
kernel grid assumes are checked before a launch; CUDA(HIP) tensors go to the gfx950 kernels, CPU
tensors to the twins; there is no Python fallback.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch

from .kernels import REC_WORDS, _check, _is_gpu, _p, _stream
from .native import load

MODE_MFMA = 0   # one-hot x vectors GEMM on v_mfma_f32_32x32x16_bf16 (production)
MODE_VALU = 1   # same sorted tiles, lanes walk the runs sequentially (A/B reference)


def check_dim(dim: int) -> None:
    if dim <= 0 or dim % 32 or dim > 256:
        raise ValueError("metric vector width must be a multiple of 32 in [32, 256]")


@dataclass
class VecAggPlan:
    cap_log2: int
    nsub: int
    ring: int
    dim: int
    nsrc: int
    bucket_cap: int
    np_step: int
    positional: int
    rec_words: int
    mode: int
    pane_base: int
    p_lo: int
    fired_hi: int

    def as_dict(self) -> dict:
        return dict(self.__dict__)


def gen_vectors(vec: torch.Tensor, *, seed: int, stream_id: int, idx0: int, lo: float = 0.0,
                span: float = 100.0) -> None:
    """Synthetic metric vectors (row i = event idx0 + i), identical on GPU and CPU."""
    if vec.dim() != 2:
        raise ValueError("vec must be [n, dim]")
    n, dim = vec.shape
    check_dim(dim)
    _check(vec, torch.float32, n * dim, "vec", vec.device)
    m = load()
    args = (_p(vec), n, dim, seed & (2**64 - 1), stream_id & (2**64 - 1), idx0, float(lo),
            float(span))
    if _is_gpu(vec):
        m.gpu_gen_vectors(*args, _stream(vec))
    else:
        m.cpu_gen_vectors(*args)


def vec_window_agg(recs, counts, plan: VecAggPlan, vec, keys_g, acc_g, cnt_g, dirty_g, occ,
                   flags) -> None:
    dev = keys_g.device
    check_dim(plan.dim)
    nslots = plan.nsub << plan.cap_log2
    nrec = plan.nsrc * plan.nsub * plan.bucket_cap
    _check(recs, torch.int64, nrec * REC_WORDS if plan.rec_words == 3 else nrec * 2, "recs", dev)
    _check(counts, torch.int32, plan.nsrc * plan.nsub, "counts", dev)
    _check(vec, torch.float32, (nrec if plan.positional else 1) * plan.dim, "vec", dev)
    _check(keys_g, torch.int64, nslots, "keys_g", dev)
    _check(acc_g, torch.float32, plan.ring * nslots * plan.dim, "acc_g", dev)
    _check(cnt_g, torch.int32, plan.ring * nslots, "cnt_g", dev)
    _check(dirty_g, torch.uint8, plan.ring * nslots, "dirty_g", dev)
    _check(occ, torch.int32, plan.nsub, "occupancy", dev)
    _check(flags, torch.int32, 1, "flags", dev)
    if plan.np_step > plan.ring:
        raise ValueError("step touches more panes than the ring holds")
    m = load()
    if _is_gpu(keys_g) and m.vec_window_agg_lds(plan.cap_log2) > 160 * 1024:
        raise ValueError("vec_window_agg: LDS image exceeds 160 KiB")
    args = (_p(recs), _p(counts), plan.as_dict(), _p(vec), _p(keys_g), _p(acc_g), _p(cnt_g),
            _p(dirty_g), _p(occ), _p(flags))
    if _is_gpu(keys_g):
        m.gpu_vec_window_agg(*args, _stream(keys_g))
    else:
        m.cpu_vec_window_agg(*args)


def vec_window_fire(keys_g, acc_g, cnt_g, dirty_g, *, dim: int, npanes: int, ring: int, p0: int,
                    only_dirty: bool, avg: bool, threshold: float | None, out_keys, out_vec,
                    out_cnt, out_n) -> None:
    dev = keys_g.device
    check_dim(dim)
    nslots = keys_g.numel()
    cap = out_keys.numel()
    _check(acc_g, torch.float32, ring * nslots * dim, "acc_g", dev)
    _check(cnt_g, torch.int32, ring * nslots, "cnt_g", dev)
    _check(dirty_g, torch.uint8, ring * nslots, "dirty_g", dev)
    _check(out_vec, torch.float32, cap * dim, "out_vec", dev)
    _check(out_cnt, torch.int32, cap, "out_cnt", dev)
    _check(out_n, torch.int32, 1, "out_n", dev)
    if npanes > ring:
        raise ValueError("window spans more panes than the ring")
    plan = dict(dim=dim, npanes=npanes, ring=ring, only_dirty=int(only_dirty), avg=int(avg),
                use_thr=int(threshold is not None),
                thr=float(threshold) if threshold is not None else 0.0, nslots=nslots, p0=p0,
                out_cap=cap)
    m = load()
    args = (_p(keys_g), _p(acc_g), _p(cnt_g), _p(dirty_g), plan, _p(out_keys), _p(out_vec),
            _p(out_cnt), _p(out_n))
    if _is_gpu(keys_g):
        m.gpu_vec_window_fire(*args, _stream(keys_g))
    else:
        m.cpu_vec_window_fire(*args)


def vec_gather(recs, rec_words: int, counts, nb: int, bcap: int, vec, out) -> None:
    """G > 1: out[j] = vec[row of record j] for every record of the send buckets."""
    dev = recs.device
    dim = vec.shape[1]
    check_dim(dim)
    _check(recs, torch.int64, nb * bcap * (REC_WORDS if rec_words == 3 else 2), "recs", dev)
    _check(counts, torch.int32, nb, "counts", dev)
    _check(vec, torch.float32, dim, "vec", dev)
    _check(out, torch.float32, nb * bcap * dim, "out", dev)
    m = load()
    args = (_p(recs), int(rec_words), _p(counts), nb, int(bcap), _p(vec), dim, _p(out))
    if _is_gpu(recs):
        m.gpu_vec_gather(*args, _stream(recs))
    else:
        m.cpu_vec_gather(*args)
