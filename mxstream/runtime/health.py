"""Failure detection: step watchdog, peer heartbeats, collective error handling.

The reference runs with checkpointing off, so any failure ends the job; Flink
detects dead TaskManagers by heartbeat timeouts (JobMaster <-> TaskExecutor) and stuck tasks by
the task cancellation watchdog. mxstream's equivalents, one process per GPU:

* :class:`Watchdog` — a step-time watchdog. The executor (or a bench loop) calls ``beat()`` once
  per micro-batch; if no beat arrives within ``timeout_ms`` the watchdog thread dumps every thread's
  stack, counts the event and either interrupts the main thread (``action="interrupt"``: the job
  fails with :class:`StepTimeout` and the restart strategy decides) or terminates the process
  (``action="abort"``, exit code 75) — the right action when the GPU or a collective is hung and
  the main thread can never return to Python. The supervisor (torchrun's elastic agent, or the
  job's restart strategy) then restarts from the latest completed checkpoint.
* :class:`PeerHeartbeat` — every rank publishes ``(step, wall ms)`` to the rendezvous key-value
  store every ``interval_ms`` and watches its peers; a rank whose heartbeat is older than
  ``timeout_ms`` is reported dead (``check()`` raises :class:`RankFailure`) so the survivors stop
  waiting inside a collective that will never complete.
* :func:`configure_collective_errors` — RCCL asynchronous error handling for the process group
  (``TORCH_NCCL_ASYNC_ERROR_HANDLING``): a failed or timed-out collective aborts the communicator
  instead of hanging every rank.

All three work with the gloo backend, so they are tested with multi-process CPU runs.
"""
from __future__ import annotations

import faulthandler
import os
import sys
import threading
import time
import _thread

from ..utils.log import get_logger

log = get_logger("runtime.health")

ABORT_EXIT_CODE = 75  # EX_TEMPFAIL: "retry me" for a supervisor


class StepTimeout(RuntimeError):
    """A micro-batch step exceeded the watchdog timeout."""


class RankFailure(RuntimeError):
    """A peer rank stopped heart-beating (crashed or hung)."""


def configure_collective_errors(blocking_wait: bool = False) -> None:
    """Make RCCL surface collective failures instead of hanging: asynchronous error handling
    tears the communicator down when a collective fails or exceeds the process group's timeout.
    Must run before the process group is created (init_distributed calls it)."""
    os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
    if blocking_wait:
        os.environ.setdefault("TORCH_NCCL_BLOCKING_WAIT", "1")


class Watchdog:
    def __init__(self, timeout_ms: int, *, name: str = "job", action: str = "interrupt",
                 on_expire=None, poll_ms: int | None = None):
        if timeout_ms <= 0:
            raise ValueError("watchdog timeout must be positive")
        if action not in ("interrupt", "abort", "none"):
            raise ValueError("action must be interrupt | abort | none")
        self.timeout = timeout_ms / 1000.0
        self.name = name
        self.action = action
        self.on_expire = on_expire
        self.poll = (poll_ms / 1000.0) if poll_ms else min(0.05, self.timeout / 4)
        self.step = -1
        self.expired = False
        self.expirations = 0
        self._deadline = time.monotonic() + self.timeout
        self._stop = threading.Event()
        self._lock = threading.Lock()
        self._thread: threading.Thread | None = None

    def start(self) -> "Watchdog":
        self._deadline = time.monotonic() + self.timeout
        self._thread = threading.Thread(target=self._run, name=f"mxs-watchdog-{self.name}",
                                        daemon=True)
        self._thread.start()
        return self

    def stop(self) -> None:
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=1.0)
            self._thread = None

    def __enter__(self):
        return self.start()

    def __exit__(self, *exc):
        self.stop()
        return False

    def beat(self, step: int | None = None) -> None:
        with self._lock:
            self.step = self.step + 1 if step is None else step
            self._deadline = time.monotonic() + self.timeout

    def check(self) -> None:
        """Raise StepTimeout in the caller if the watchdog fired (used by loops that catch the
        interrupt themselves)."""
        if self.expired:
            raise StepTimeout(f"{self.name}: step {self.step + 1} exceeded {self.timeout * 1e3:.0f} ms")

    def _run(self) -> None:
        while not self._stop.wait(self.poll):
            with self._lock:
                late = time.monotonic() > self._deadline
            if not late or self.expired:
                continue
            self.expired = True
            self.expirations += 1
            log.error("watchdog %s: step %d made no progress for %.0f ms; thread stacks follow",
                      self.name, self.step + 1, self.timeout * 1e3)
            try:
                faulthandler.dump_traceback(file=sys.stderr, all_threads=True)
            except Exception:  # pragma: no cover - stderr closed
                pass
            if self.on_expire is not None:
                try:
                    self.on_expire(self)
                except Exception:  # pragma: no cover
                    log.exception("watchdog callback failed")
            if self.action == "interrupt":
                _thread.interrupt_main()
            elif self.action == "abort":
                os._exit(ABORT_EXIT_CODE)


def default_store():
    """The rendezvous store of the default process group (torchrun / init_process_group)."""
    import torch.distributed as dist

    if not dist.is_initialized():
        raise RuntimeError("torch.distributed is not initialised")
    return dist.distributed_c10d._get_default_store()


class PeerHeartbeat:
    """Heartbeats through a torch.distributed Store (TCPStore / FileStore)."""

    PREFIX = "mxs/hb/"

    def __init__(self, store, rank: int, world: int, *, interval_ms: int = 500,
                 timeout_ms: int = 10_000):
        self.store, self.rank, self.world = store, rank, world
        self.interval = interval_ms / 1000.0
        self.timeout_ms = timeout_ms
        self.step = 0
        self.dead: set[int] = set()
        self.last_seen: dict[int, int] = {}
        self._stop = threading.Event()
        self._paused = False
        self._thread: threading.Thread | None = None
        self._started_ms = int(time.time() * 1000)

    def _publish(self) -> None:
        self.store.set(f"{self.PREFIX}{self.rank}", f"{self.step}:{int(time.time() * 1000)}")

    def start(self) -> "PeerHeartbeat":
        self._publish()
        self._thread = threading.Thread(target=self._run, name=f"mxs-heartbeat-{self.rank}",
                                        daemon=True)
        self._thread.start()
        return self

    def stop(self) -> None:
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=2.0)
            self._thread = None

    def pause(self, paused: bool = True) -> None:
        """Stop publishing (tests: simulate a hung rank without killing the process)."""
        self._paused = paused

    def beat(self, step: int) -> None:
        self.step = int(step)

    def _poll_peers(self) -> None:
        now = int(time.time() * 1000)
        for r in range(self.world):
            if r == self.rank or r in self.dead:
                continue
            key = f"{self.PREFIX}{r}"
            try:
                present = self.store.check([key])
            except Exception:
                present = False
            if present:
                try:
                    ts = int(self.store.get(key).decode().split(":")[1])
                    self.last_seen[r] = ts
                except Exception:
                    pass
            last = self.last_seen.get(r, self._started_ms)
            if now - last > self.timeout_ms:
                self.dead.add(r)
                log.error("rank %d: peer rank %d missed heartbeats for %d ms", self.rank, r,
                          now - last)

    def _run(self) -> None:
        while not self._stop.wait(self.interval):
            if not self._paused:
                try:
                    self._publish()
                except Exception:  # store gone: the job is shutting down
                    return
            self._poll_peers()

    def check(self) -> None:
        if self.dead:
            raise RankFailure(f"rank {self.rank}: peer rank(s) {sorted(self.dead)} stopped "
                              f"heart-beating")
