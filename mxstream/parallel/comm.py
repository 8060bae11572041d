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

import collections
import datetime
import os
import sys

import torch
import torch.distributed as dist

from ..utils.log import get_logger

log = get_logger(__name__)


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

    def broadcast_(self, t: torch.Tensor, src: int = 0) -> None:
        """In place: every rank's `t` (same shape and dtype everywhere) becomes rank src's."""
        return None

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


class LoopbackGroup:
    """G virtual ranks inside ONE process (SURVEY.md §2.5 "testing": LoopbackComm).

    Every virtual rank is a thread that owns its operator instances and calls the collectives in
    the same order a real rank would. The exchange has exactly ``all_to_all_single``'s layout
    (equal split, chunk j of rank i lands in chunk i of rank j); on a GPU the chunks move with
    device-to-device copies on the reading rank's current stream, ordered against the producing
    rank's stream with HIP events (deposit event -> reader waits; reader-done events -> the
    producer waits before it may overwrite its buffer). So the whole G>1 GPU path -- key-group
    partition, combiner, combined-record aggregation, overflow regrow, watermark valve -- runs on
    one MI355X (or on the CPU twins) with RCCL's data layout, without RCCL.
    """

    def __init__(self, world: int, timeout_s: float = 600.0):
        import threading

        if world < 1:
            raise ValueError("world must be >= 1")
        self.world = world
        self.timeout_s = timeout_s
        self._barrier = threading.Barrier(world, timeout=timeout_s)
        self._slots: list = [None] * world
        self._events: list = [None] * world
        # every collective's kind per rank, checked at its first barrier (a rank that enters a
        # different collective than its peers fails loudly instead of mixing buffers), and the
        # last few kinds with their callers, for that error message
        self._kinds: list = [None] * world
        self._hist: list = [collections.deque(maxlen=12) for _ in range(world)]
        self._done: list = [[None] * world for _ in range(world)]
        self.a2a_bytes = 0

    def comm(self, rank: int) -> "LoopbackComm":
        return LoopbackComm(self, rank)

    def abort(self) -> None:
        self._barrier.abort()

    def wait(self) -> None:
        self._barrier.wait()


def _record_event(t: torch.Tensor):
    if t.device.type != "cuda":
        return None
    ev = torch.cuda.Event()
    ev.record(torch.cuda.current_stream(t.device))
    return ev


def _wait_event(t: torch.Tensor, ev) -> None:
    if ev is not None:
        torch.cuda.current_stream(t.device).wait_event(ev)


class LoopbackComm(Comm):
    """One virtual rank of a LoopbackGroup (same interface as TorchComm)."""

    def __init__(self, group: LoopbackGroup, rank: int):
        self.group_obj = group
        self.group = None
        self.rank = rank
        self.world = group.world
        self.backend = "loopback"

    # Collective skeleton: deposit -> barrier -> read peers -> barrier (peers done reading) ->
    # the owner's stream waits for the readers' events before it reuses its buffer.
    def _enter(self, kind: str, slot) -> None:
        """Deposit this rank's slot, wait for the peers, check they entered the same collective."""
        g = self.group_obj
        if isinstance(slot, torch.Tensor):
            kind = f"{kind}[{slot.device.type},{str(slot.dtype)[6:]}]"
        f = sys._getframe(2)
        g._hist[self.rank].append(f"{kind} <- {f.f_code.co_name}:{f.f_lineno} "
                                  f"<- {f.f_back.f_code.co_name if f.f_back else '?'}")
        g._kinds[self.rank] = kind
        g._slots[self.rank] = slot
        g._events[self.rank] = _record_event(slot) if isinstance(slot, torch.Tensor) else None
        g.wait()
        if any(k != kind for k in g._kinds):
            hist = "\n".join(f"  rank {r}: " + " | ".join(list(h)[-4:]) for r, h in enumerate(g._hist))
            raise RuntimeError(f"loopback collective mismatch: ranks entered {g._kinds}\n{hist}")

    def _deposit(self, t, kind: str = "collective") -> None:
        self._enter(kind, t)

    def _finish(self, t) -> None:
        g = self.group_obj
        g.wait()
        if isinstance(t, torch.Tensor) and t.device.type == "cuda":
            for src in range(self.world):
                _wait_event(t, g._done[src][self.rank])
        g.wait()  # every rank consumed its done events before the next collective reuses them

    def _read(self, src: int, like: torch.Tensor) -> torch.Tensor:
        g = self.group_obj
        _wait_event(like, g._events[src])
        return g._slots[src]

    def _mark_read(self, src: int, like: torch.Tensor) -> None:
        self.group_obj._done[self.rank][src] = _record_event(like)

    def all_to_all(self, out, inp):
        if out.numel() != inp.numel() or inp.numel() % self.world:
            raise ValueError("all_to_all: equal split needs numel divisible by world")
        if self.world == 1:
            LocalComm.all_to_all(self, out, inp)
            return
        self._deposit(inp, f"all_to_all_{inp.numel()}")
        c = inp.numel() // self.world
        for src in range(self.world):
            peer = self._read(src, out)
            out[src * c:(src + 1) * c].copy_(peer[self.rank * c:(self.rank + 1) * c],
                                             non_blocking=True)
            self._mark_read(src, out)
        if self.rank == 0:
            self.group_obj.a2a_bytes += inp.numel() * inp.element_size() * self.world
        self._finish(inp)

    def _allreduce(self, t, op) -> None:
        if self.world == 1:
            return
        self._deposit(t, f"allreduce_{op.__name__}")
        acc = t.clone()
        for src in range(self.world):
            if src == self.rank:
                self._mark_read(src, t)
                continue
            peer = self._read(src, t)
            acc = op(acc, peer)
            self._mark_read(src, t)
        # Nobody may overwrite its own input before every peer has read it.
        g = self.group_obj
        g.wait()
        if t.device.type == "cuda":
            for src in range(self.world):
                _wait_event(t, g._done[src][self.rank])
        t.copy_(acc)
        g.wait()

    def allreduce_min_(self, t):
        self._allreduce(t, torch.minimum)

    def allreduce_max_(self, t):
        self._allreduce(t, torch.maximum)

    def allreduce_sum_(self, t):
        self._allreduce(t, torch.add)

    def barrier(self):
        if self.world > 1:
            self._enter("barrier", None)
            self.group_obj.wait()  # (every rank checked the kinds before any enters the next)

    def broadcast_(self, t, src: int = 0):
        if self.world == 1:
            return
        self._deposit(t, f"broadcast_{src}")
        if self.rank != src:
            peer = self._read(src, t)
            t.copy_(peer)
        self._mark_read(src, t)
        self._finish(t)

    def broadcast_object(self, obj, src: int = 0):
        if self.world == 1:
            return obj
        g = self.group_obj
        self._enter(f"broadcast_object_{src}", obj)
        v = g._slots[src]
        g.wait()
        return v

    def all_gather_object(self, obj):
        if self.world == 1:
            return [obj]
        g = self.group_obj
        self._enter("all_gather_object", obj)
        v = list(g._slots)
        g.wait()
        return v


I64_MIN, I64_MAX = -(1 << 63), (1 << 63) - 1


def control_reduce(comm: Comm, mins: list[int] = (), maxs: list[int] = ()) -> tuple[list, list]:
    """The host control plane's one collective: a packed int64 MIN all-reduce of small integers
    (flags, clocks, watermarks). MAX words travel negated (I64_MIN clamps to I64_MIN + 1, so its
    negation fits). One CPU tensor over the control group (gloo) or the loopback ranks -- no
    pickling, a fixed 8 bytes per word."""
    mins, maxs = [int(x) for x in mins], [int(x) for x in maxs]
    if comm is None or comm.world == 1:
        return mins, maxs
    t = torch.tensor(mins + [-max(x, I64_MIN + 1) for x in maxs], dtype=torch.int64)
    comm.allreduce_min_(t)
    v = t.tolist()
    return v[:len(mins)], [-x for x in v[len(mins):]]


def run_loopback(world: int, fn, *args, device: torch.device | None = None,
                 timeout_s: float = 600.0) -> list:
    """Run ``fn(comm, *args)`` on `world` virtual ranks (threads) of one LoopbackGroup and return
    the per-rank results in rank order. An exception on any rank aborts the group (the others
    leave their barrier with BrokenBarrierError) and is re-raised here."""
    import threading

    if device is not None and device.type == "cuda" and device.index is None:
        device = torch.device("cuda", torch.cuda.current_device())
    group = LoopbackGroup(world, timeout_s=timeout_s)
    res: list = [None] * world
    errs: list = [None] * world

    def body(r):
        try:
            if device is not None and device.type == "cuda":
                torch.cuda.set_device(device)
            res[r] = fn(group.comm(r), *args)
        except BaseException as e:  # noqa: BLE001 - re-raised on the caller's thread
            errs[r] = e
            group.abort()

    ths = [threading.Thread(target=body, args=(r,), name=f"mxs-loopback-{r}") for r in range(world)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    first = next((e for e in errs if e is not None and not isinstance(e, threading.BrokenBarrierError)
                  and not isinstance(e.__cause__, threading.BrokenBarrierError)),
                 next((e for e in errs if e is not None), None))
    if first is not None:
        for r, e in enumerate(errs):  # the other ranks' errors, for the log
            if e is not None and e is not first:
                log.warning("loopback rank %d also failed: %s: %s", r, type(e).__name__, e)
        raise first
    return res


class TorchComm(Comm):
    """torch.distributed process group: backend 'nccl' (= RCCL over xGMI) or 'gloo' (CPU)."""

    def __init__(self, group=None):
        if not dist.is_initialized():
            raise RuntimeError("torch.distributed is not initialised (use init_distributed())")
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.backend = dist.get_backend(group)
        if self.world > 1:
            # Create (and, on RCCL, connect) the payload communicator now: every rank constructs
            # its TorchComm at the same point, while a lazy creation would sit inside the first
            # all-to-all -- a window firing in the middle of a timed run.
            g = self._data_group()
            dev = (torch.device("cuda", torch.cuda.current_device()) if self.backend == "nccl"
                   else torch.device("cpu"))
            t = torch.zeros(self.world, dtype=torch.int32, device=dev)
            dist.all_to_all_single(torch.empty_like(t), t, group=g)

    def _data_group(self):
        """The keyBy payload travels on its own communicator: RCCL runs each communicator's
        collectives on its own internal stream, so the all-to-all of step i (issued on the
        operator's state stream) does not queue behind the watermark all-reduce of step i+1,
        which waits for that step's partition kernel. Created in __init__."""
        g = getattr(self, "_dgroup", None)
        if g is None:
            ranks = dist.get_process_group_ranks(self.group) if self.group is not None else None
            g = self._dgroup = dist.new_group(ranks=ranks, backend=self.backend)
        return g

    def all_to_all(self, out, inp):
        if self.world == 1:
            LocalComm.all_to_all(self, out, inp)
            return
        dist.all_to_all_single(out, inp, group=self._data_group())

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

    def broadcast_(self, t, src: int = 0):
        if self.world > 1:
            dist.broadcast(t, src=src, group=self.group)

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


def shutdown_distributed(comm: Comm | None = None) -> None:
    """Orderly end of a multi-process run: a barrier on every rank, then the process groups are
    destroyed. Without it the first rank to exit closes its gloo sockets while a slower peer may
    still be completing the last collective; gloo's transport thread then sees the reset
    connection and aborts that peer (SIGABRT: the round-4 2-rank records bench under load)."""
    if not dist.is_initialized():
        return
    if comm is not None and comm.world > 1:
        comm.barrier()
    dist.barrier()
    dist.destroy_process_group()
