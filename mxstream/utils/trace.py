"""Tracing: roctx stage ranges for rocprofv3 and Chrome-trace JSON export.

The recorder is native (csrc/trace.cpp); this module is the Python face:

* ``span(name)``: a host range (context manager). With roctx enabled (``MXS_ROCTX=1`` or
  ``enable(roctx=True)``) it is also a roctx range, so ``rocprofv3 --marker-trace`` groups the
  kernels of each engine stage (partition, all_to_all, window_agg, fire, spill, checkpoint).
* ``gpu_span(name, start_event, end_event)``: a device-time span from two HIP events, placed on
  the host timeline via a reference event recorded when tracing was enabled.
  ``utils.metrics.StageTimer`` feeds every stage it times through here.
* ``dump(path)``: Chrome trace JSON (open in chrome://tracing or Perfetto); one process id per
  rank, one track per host thread plus a ``gpu-<device>`` track.

Enable from the environment (``MXS_TRACE=1``), the engine config (``trace_path``), the bench
(``bench.py --trace out.json``) or code (``trace.enable()``).
"""
from __future__ import annotations

import contextlib
import os

from ..ops.native import load

_ref = {}  # device index -> (reference hip event, host ns when it was recorded)


def enable(on: bool = True, *, roctx: bool | None = None, capacity: int | None = None) -> None:
    m = load()
    m.trace_enable(bool(on))
    if roctx is not None:
        m.trace_enable_roctx(bool(roctx))
    if capacity:
        m.trace_set_capacity(int(capacity))


def enabled() -> bool:
    return load().trace_enabled()


def roctx_enabled() -> bool:
    return load().trace_roctx_enabled()


def active() -> bool:
    m = load()
    return m.trace_enabled() or m.trace_roctx_enabled()


@contextlib.contextmanager
def span(name: str, cat: str = "stage"):
    m = load()
    if not (m.trace_enabled() or m.trace_roctx_enabled()):
        yield
        return
    m.trace_push(name, cat)
    try:
        yield
    finally:
        m.trace_pop()


def mark(name: str) -> None:
    load().trace_mark(name)


def _reference(device):
    import torch

    idx = device.index if device.index is not None else torch.cuda.current_device()
    ref = _ref.get(idx)
    if ref is None:
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        ev.synchronize()
        ref = (ev, load().trace_now_ns())
        _ref[idx] = ref
    return idx, ref


def gpu_span(name: str, start, end, device=None, cat: str = "gpu") -> None:
    """Record a device span from two completed HIP events (torch.cuda.Event)."""
    m = load()
    if not m.trace_enabled():
        return
    import torch

    idx, (ref, ref_ns) = _reference(device or torch.device("cuda"))
    t0 = ref_ns + int(ref.elapsed_time(start) * 1e6)
    dur = int(start.elapsed_time(end) * 1e6)
    m.trace_complete(name, cat, f"gpu-{idx}", t0, dur)


def complete(name: str, ts_ns: int, dur_ns: int, track: str = "host", cat: str = "stage") -> None:
    load().trace_complete(name, cat, track, int(ts_ns), int(dur_ns))


def now_ns() -> int:
    return load().trace_now_ns()


def count() -> int:
    return load().trace_count()


def clear() -> None:
    load().trace_clear()
    _ref.clear()


def dump(path: str | os.PathLike, rank: int = 0) -> int:
    """Write the Chrome trace JSON; returns the number of spans written."""
    return load().trace_dump_chrome(str(path), int(rank))
