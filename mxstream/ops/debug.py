"""Debug-mode helpers: the keyed-state invariant checker.

``check_table`` runs csrc/check_hip.hip (GPU) or its C++ twin over an operator's slot table and
returns ``{"live", "misplaced", "broken_chain", "duplicate"}``; anything but ``live`` non-zero
means a corrupted table. With ``MXS_DEBUG=1`` the keyed window operators run it after every step
and raise :class:`StateCorruption` on a violation.
"""
from __future__ import annotations

import os

import torch

from .kernels import _check, _is_gpu, _p, _stream
from .native import load

FIELDS = ("live", "misplaced", "broken_chain", "duplicate")


class StateCorruption(RuntimeError):
    pass


def debug_enabled() -> bool:
    v = os.environ.get("MXS_DEBUG", "")
    return bool(v) and v != "0"


def check_table(keys_g: torch.Tensor, *, nsub: int, nsub_log2: int, cap_log2: int) -> dict:
    dev = keys_g.device
    _check(keys_g, torch.int64, nsub << cap_log2, "keys_g", dev)
    stats = torch.zeros(len(FIELDS), dtype=torch.int64, device=dev)
    m = load()
    if _is_gpu(keys_g):
        m.gpu_check_table(_p(keys_g), nsub, nsub_log2, cap_log2, _p(stats), _stream(keys_g))
    else:
        m.cpu_check_table(_p(keys_g), nsub, nsub_log2, cap_log2, _p(stats))
    return dict(zip(FIELDS, stats.cpu().tolist()))


def assert_table_ok(keys_g: torch.Tensor, *, nsub: int, nsub_log2: int, cap_log2: int,
                    where: str = "") -> dict:
    r = check_table(keys_g, nsub=nsub, nsub_log2=nsub_log2, cap_log2=cap_log2)
    if r["misplaced"] or r["broken_chain"] or r["duplicate"]:
        raise StateCorruption(f"keyed state invariant violated {where}: {r}")
    return r
