"""Communication layer: one process per GPU over torch.distributed (RCCL on ROCm, gloo on CPU).

The engine's exchange pattern is:
  * keyBy shuffle  = ONE equal-split all-to-all of fixed-capacity bucket ranges (the partition
    kernel makes every destination range the same size, so no host-side count exchange precedes
    the payload) plus a tiny all-to-all of the per-bucket counts;
  * watermark valve = MIN all-reduce of a few int64 (per-rank watermark, pane range, flags);
  * barriers / checkpoint agreement = all-reduce on the step id.
On a fully connected xGMI node (7 links/GPU) an all-to-all moves B*W/G bytes per link
concurrently, so it is per-link bound and never the bottleneck at micro-batch sizes.
"""
from __future__ import annotations

import datetime
import os

import torch
import torch.distributed as dist


class Comm:
    """Interface; LocalComm is the G=1 case, TorchComm the multi-process one."""

    rank: int = 0
    world: int = 1

    def all_to_all(self, out: torch.Tensor, inp: torch.Tensor) -> None:
        raise NotImplementedError

    def allreduce_min_(self, t: torch.Tensor) -> None:
        raise NotImplementedError

    def allreduce_max_(self, t: torch.Tensor) -> None:
        raise NotImplementedError

    def allreduce_sum_(self, t: torch.Tensor) -> None:
        raise NotImplementedError

    def barrier(self) -> None:
        pass

    def broadcast_object(self, obj, src: int = 0):
        return obj

    def all_gather_object(self, obj) -> list:
        return [obj]


class LocalComm(Comm):
    """Single rank: every collective is the identity."""

    def all_to_all(self, out, inp):
        if out.data_ptr() != inp.data_ptr():
            out.copy_(inp)

    def allreduce_min_(self, t):
        return None

    def allreduce_max_(self, t):
        return None

    def allreduce_sum_(self, t):
        return None


class TorchComm(Comm):
    """torch.distributed process group: backend 'nccl' (= RCCL over xGMI) or 'gloo' (CPU)."""

    def __init__(self, group=None):
        if not dist.is_initialized():
            raise RuntimeError("torch.distributed is not initialised (use init_distributed())")
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.backend = dist.get_backend(group)

    def all_to_all(self, out, inp):
        if self.world == 1:
            LocalComm.all_to_all(self, out, inp)
            return
        dist.all_to_all_single(out, inp, group=self.group)

    def allreduce_min_(self, t):
        if self.world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MIN, group=self.group)

    def allreduce_max_(self, t):
        if self.world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)

    def allreduce_sum_(self, t):
        if self.world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)

    def barrier(self):
        if self.world > 1:
            if self.backend == "nccl":
                dist.barrier(group=self.group, device_ids=[torch.cuda.current_device()])
            else:
                dist.barrier(group=self.group)

    def broadcast_object(self, obj, src: int = 0):
        lst = [obj]
        dist.broadcast_object_list(lst, src=src, group=self.group)
        return lst[0]

    def all_gather_object(self, obj):
        out = [None] * self.world
        dist.all_gather_object(out, obj, group=self.group)
        return out


def init_distributed(device: str = "auto", timeout_s: int = 600) -> Comm:
    """Initialise one-process-per-GPU from torchrun env vars; returns a Comm.

    device='cuda' -> backend nccl (RCCL), 'cpu' -> gloo. Without WORLD_SIZE>1 returns LocalComm.
    """
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world <= 1:
        return LocalComm()
    if device == "auto":
        device = "cuda" if torch.cuda.is_available() else "cpu"
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    backend = "nccl" if device == "cuda" else "gloo"
    if backend == "nccl":
        from ..runtime.health import configure_collective_errors

        configure_collective_errors()
    if not dist.is_initialized():
        kw = dict(backend=backend, timeout=datetime.timedelta(seconds=timeout_s))
        if backend == "nccl":
            local = int(os.environ.get("LOCAL_RANK", "0"))
            torch.cuda.set_device(local)
            kw["device_id"] = torch.device("cuda", local)
        dist.init_process_group(**kw)
    return TorchComm()
