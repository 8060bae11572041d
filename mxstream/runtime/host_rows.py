"""Host-side row transport of the GPU operators: pinned slab pools (reused page-locked buffers),
the device-counted D2H of a step's rows into one slab without a host round trip
(CountedHostRows, csrc gpu_d2h_counted), the synchronous column copy (to_host_arrays), and the
GIL-free event waits (gpu_event_spin). Used by the window, session and rolling operators.
"""
from __future__ import annotations

import os as _os

import numpy as np
import torch


class PinnedSlabPool:
    """Pinned host slabs for fired rows, reused once every array handed out of a slab is gone.

    `torch.empty(..., pin_memory=True)` per fire cost ~1.5 ms of host time per firing in the
    rocprofv3 timeline of the headline bench (profiles/r1_fire_pinned_pool.md): the GPU idled
    between the fire kernel and the D2H copies. A slab is one pinned byte tensor plus its numpy
    view; every column handed out is a numpy view of that array, so the array's refcount says
    whether any caller still holds rows of the slab."""

    def __init__(self, pin: bool = True, max_slabs: int = 8):
        self.pin = pin
        self.max_slabs = max_slabs
        self.slabs: list[tuple[torch.Tensor, np.ndarray]] = []
        self.allocs = 0

    def _free(self, i: int) -> bool:
        # References to a free slab's array: the pool's tuple + getrefcount's own argument.
        import sys

        return sys.getrefcount(self.slabs[i][1]) <= 2

    def reserve_async(self, nbytes: int) -> None:
        """Allocate a slab of `nbytes` (rounded up) on a background thread, for a later take():
        a growing caller (the host tier's firing export) asks ahead of need, so the page-locking
        of a large slab (~25 ms at 512 MB on the box; torch releases the GIL inside it) runs
        beside the step instead of inside it."""
        if not self.pin or getattr(self, "_reserving", None) is not None:
            return
        size = _next_pow2(max(nbytes, 1 << 16))
        if any(s[0].numel() >= size for s in self.slabs):
            return
        import threading

        box = {}

        def work():
            try:
                box["t"] = torch.empty(size, dtype=torch.uint8, pin_memory=True)
            except BaseException as e:  # surfaced by the next take()
                box["err"] = e

        th = threading.Thread(target=work, name="mxs-pin-reserve", daemon=True)
        th.start()
        self._reserving = (th, box)

    def _land_reserve(self, block: bool) -> None:
        r = getattr(self, "_reserving", None)
        if r is None or (not block and r[0].is_alive()):
            return
        r[0].join()
        self._reserving = None
        if "err" in r[1]:
            raise r[1]["err"]
        t = r[1]["t"]
        if len(self.slabs) >= self.max_slabs:
            free = [i for i in range(len(self.slabs)) if self._free(i)]
            if not free:
                return  # every slab is in use: the reserve is dropped
            self.slabs.pop(min(free, key=lambda i: self.slabs[i][0].numel()))
        self.allocs += 1
        self.slabs.append((t, t.numpy()))

    def take(self, nbytes: int, twins: bool = False) -> tuple[torch.Tensor, np.ndarray]:
        """A free slab of at least nbytes. twins: when a new slab must be allocated, allocate a
        second one of the same size with it -- a caller that holds one slab while it fills the
        next (the tier export) would otherwise page-lock the second at a later, busier call."""
        if getattr(self, "_reserving", None) is not None:
            # a reserve in flight that this take needs is waited for (not allocated twice)
            self._land_reserve(block=not any(s[0].numel() >= nbytes and self._free(i)
                                             for i, s in enumerate(self.slabs)))
        for i in range(len(self.slabs)):
            if self.slabs[i][0].numel() >= nbytes and self._free(i):
                return self.slabs[i]
        if len(self.slabs) >= self.max_slabs:
            # Drop the smallest free slab so a long-lived caller cannot grow the pool unbounded.
            free = [i for i in range(len(self.slabs)) if self._free(i)]
            if free:
                self.slabs.pop(min(free, key=lambda i: self.slabs[i][0].numel()))
        size = _next_pow2(max(nbytes, 1 << 16))
        t = torch.empty(size, dtype=torch.uint8, pin_memory=self.pin)
        self.allocs += 1
        slab = (t, t.numpy())
        self.slabs.append(slab)
        if twins and len(self.slabs) < self.max_slabs + 1:
            if len(self.slabs) > self.max_slabs:  # make room: the smallest free other slab
                free = [i for i in range(len(self.slabs) - 1) if self._free(i)]
                if free:
                    self.slabs.pop(min(free, key=lambda i: self.slabs[i][0].numel()))
            if len(self.slabs) < self.max_slabs:
                t2 = torch.empty(size, dtype=torch.uint8, pin_memory=self.pin)
                self.allocs += 1
                self.slabs.append((t2, t2.numpy()))
        return slab


_TLS = __import__("threading").local()


def _thread_pool() -> PinnedSlabPool:
    """One pool per host thread: virtual ranks of a LoopbackGroup (threads) must never be handed
    the same free slab at once."""
    pool = getattr(_TLS, "pool", None)
    if pool is None:
        pool = _TLS.pool = PinnedSlabPool()
    return pool


def to_host_arrays(cols: list[torch.Tensor], n: int, pool: PinnedSlabPool | None = None) -> list[np.ndarray]:
    """The first n rows of each output column as host arrays. On a GPU: non-blocking copies into
    one pinned slab (reused from `pool` once the caller dropped the previous arrays) and one
    stream sync — a pageable .cpu() stages every column through a bounce buffer at a fraction of
    the PCIe rate. On the CPU: copies (the device buffers are reused by the next fire)."""
    if not cols or cols[0].device.type != "cuda":
        return [c[:n].numpy().copy() for c in cols]
    pool = _thread_pool() if pool is None else pool
    offs, nbytes = [], 0
    for c in cols:
        offs.append(nbytes)
        nbytes += (n * c.element_size() + 255) & ~255
    t, arr = pool.take(nbytes)
    out, copies = [], []
    kernel_ok = _D2H != "dma"
    for o, c in zip(offs, cols):
        nb = n * c.element_size()
        if not c.is_contiguous() or n > c.numel():
            raise ValueError("to_host_arrays: columns must be contiguous with at least n rows")
        nb16 = (nb + 15) & ~15
        kernel_ok = kernel_ok and nb16 <= c.numel() * c.element_size() and c.data_ptr() % 16 == 0
        copies.append((c.data_ptr(), nb16, o))
        out.append(arr[o:o + nb].view(_NP_DTYPE[c.dtype]))
    # The DMA path (hipMemcpyAsync, and torch's copy_ before it) stalled the host for 7-9 ms at
    # one firing in some runs (profiles/r2_fire_d2h.md): a copy kernel storing into the mapped
    # pinned slab by default, one native call either way.
    from ..ops.native import load

    stream = torch.cuda.current_stream(cols[0].device)
    m = load()
    if not kernel_ok or m.gpu_d2h_kernel(t.data_ptr(), copies, stream.cuda_stream) != 0:
        m.gpu_d2h_many(t.data_ptr(), [(p, min(b, n * c.element_size()), o)
                                      for (p, b, o), c in zip(copies, cols)], stream.cuda_stream)
    stream.synchronize()
    return out


_D2H = _os.environ.get("MXS_D2H", "kernel")  # "dma": hipMemcpyAsync (A/B)
class CountedHostRows:
    """Columns whose row count is still on the device, copied to one pinned slab WITHOUT a host
    round trip: the copy kernel reads the uint32 count (`n_dev`) itself and moves only that many
    rows (gpu_d2h_counted); small `fixed` device tensors (flags, per-window bounds) ride along
    whole. The host reads the slab once `ready()` -- nothing blocks at launch, so a firing no
    longer drains the stream twice (once for its count, once for its rows).

    Layout: fixed tensors first (16-byte granules), then each column at its capacity."""

    def __init__(self, pool: PinnedSlabPool, cols: list[torch.Tensor], n_dev: torch.Tensor,
                 fixed: list[torch.Tensor] = (), copy_stream=None):
        """copy_stream: run the copy there, after the producer's work on the current stream
        (it overlaps the compute that follows; ``done`` is the event the producer must wait for
        before it overwrites the columns)."""
        from ..ops.native import load

        self.cols_meta, self.fixed_meta, copies, off = [], [], [], 0
        for t in fixed:
            nb = t.numel() * t.element_size()
            if nb % 16 or not t.is_contiguous() or t.data_ptr() % 16:
                raise ValueError("CountedHostRows: fixed tensors must be 16-byte granules")
            copies.append((t.data_ptr(), nb, off, 0))
            self.fixed_meta.append((off, nb, t.dtype))
            off += (nb + 255) & ~255
        self.cap = min(c.numel() for c in cols)
        for c in cols:
            nb = self.cap * c.element_size()
            if not c.is_contiguous() or c.data_ptr() % 16 or nb % 16:
                raise ValueError("CountedHostRows: columns must be contiguous, 16-byte aligned "
                                 "and a 16-byte multiple long")
            copies.append((c.data_ptr(), nb, off, c.element_size()))
            self.cols_meta.append((off, c.dtype))
            off += (nb + 255) & ~255
        t0 = __import__("time").perf_counter()
        self.t, self.arr = pool.take(off)
        t1 = __import__("time").perf_counter()
        dev = cols[0].device
        cur = torch.cuda.current_stream(dev)
        st = cur
        if copy_stream is not None:
            ready = torch.cuda.Event()
            ready.record(cur)
            copy_stream.wait_event(ready)
            st = copy_stream
        e = load().gpu_d2h_counted(self.t.data_ptr(), copies, n_dev.data_ptr(), st.cuda_stream,
                                   64 if copy_stream is not None else 1024)
        if e != 0:
            raise RuntimeError(f"gpu_d2h_counted failed (hipError {e})")
        self.ev = torch.cuda.Event()
        self.ev.record(st)
        self.done = self.ev
        # host seconds: slab take, the rest of the launch (phase timers of the callers)
        self.t_take, self.t_launch = t1 - t0, __import__("time").perf_counter() - t1

    def ready(self) -> bool:
        return self.ev.query()

    def wait(self) -> None:
        _event_spin(self.ev)

    def fixed(self, i: int) -> np.ndarray:
        off, nb, dt = self.fixed_meta[i]
        return self.arr[off:off + nb].view(_NP_DTYPE[dt])

    def columns(self, n: int) -> list[np.ndarray]:
        """The first n rows of every column (views of the slab); n is capped at the capacity."""
        n = min(n, self.cap)
        out = []
        for off, dt in self.cols_meta:
            es = torch.empty((), dtype=dt).element_size()
            out.append(self.arr[off:off + n * es].view(_NP_DTYPE[dt]))
        return out


_NP_DTYPE = {torch.int64: np.int64, torch.int32: np.int32, torch.float64: np.float64,
             torch.float32: np.float32, torch.uint8: np.uint8, torch.int16: np.int16,
             torch.bfloat16: np.uint16, torch.float16: np.float16}


# How the step's host sync waits for the GPU (MXS_SYNC, measured in profiles/r2_host_sync.md):
#   "query" (default): poll hipEventQuery on the step's event -- the host resumes within a
#     microsecond of the partition finishing, where a blocking wait (hipEventSynchronize /
#     hipStreamSynchronize) sleeps in the driver and wakes tens of microseconds late, time
#     the pipelined step cannot hide; "event": hipEventSynchronize; "stream":
#     hipStreamSynchronize (unpipelined only).
_SYNC = __import__("os").environ.get("MXS_SYNC", "query")


def _event_spin(ev) -> None:
    """Poll the event in C++ with the GIL released (csrc/bindings.cpp gpu_event_spin)."""
    from ..ops.native import load

    e = load().gpu_event_spin(ev.cuda_event)
    if e != 0:
        raise RuntimeError(f"hipEventQuery failed (hipError {e})")


def _host_wait(ev, device, pipelined: bool) -> None:
    if _SYNC == "query":
        _event_spin(ev)
    elif _SYNC == "event" or pipelined:
        ev.synchronize()
    else:
        torch.cuda.current_stream(device).synchronize()


def _next_pow2(x: int) -> int:
    return 1 << max(0, int(x - 1).bit_length())
