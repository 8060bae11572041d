"""Sources for the DataStream executor.

* ``SocketTextSource`` — ``env.socketTextStream(host, port)`` (every reference job, e.g.
  Main.java:17): the C++ ``SocketSource`` reader thread ('\n' delimiter, trailing '\r'
  stripped, remainder flushed at EOF, ``maxRetry = 0``); parallelism 1, rank 0 only.
* ``CollectionSource`` / ``TimedCollectionSource`` — finite, deterministic sources for tests;
  the timed variant replays ``(processing_time, value)`` pairs against a manual clock so the
  README's "wait one minute" processing-time runs are instantaneous.
* ``TextFileSource``, ``SequenceSource``, ``FunctionSource`` (user SourceFunction).

A source's ``poll(now)`` returns ``(items, finished)``; each poll is one micro-batch, after which
periodic watermark assigners emit (the engine's auto-watermark interval).
"""
from __future__ import annotations

import queue
import threading
from typing import Any, Iterable

from .operators import LONG_MIN, Rec, WM


class Source:
    parallelism = 1
    name = "Source"
    # Set by the planner when the consumer chain parses text columnar (runtime/columnar.py):
    # text sources then emit one TextBatch of raw lines per poll instead of a Rec per line.
    columnar = False

    def open(self, rank: int, world: int, clock) -> None:
        self.rank, self.world, self.clock = rank, world, clock

    def poll(self, now: int) -> tuple[list, bool]:
        raise NotImplementedError

    def next_event_time(self) -> int | None:
        """For timed sources: the processing time at which the next item arrives."""
        return None

    def close(self) -> None:
        pass

    # Replayable sources report their read position in checkpoints and seek back to it on
    # restore (Flink's source offsets). Non-replayable ones (socket) return {}.
    #
    # Rank-strided sources (global item i on rank i % G) keep, after a restore at another world
    # size, the old layout's positions they were re-split from (`_prior`): a later checkpoint
    # stores them next to its own positions, so the set of items emitted before it is exact
    # after any number of rescales -- a same-size restore re-applies the filter, a further
    # rescale chains it.
    _prior: list | None = None

    def snapshot(self) -> dict:
        pos = getattr(self, "pos", None)
        return {} if pos is None else {"pos": pos, "rescale": self._rescale_info()}

    def restore(self, snap: dict) -> None:
        if "rescaled" in snap:
            self.restore_rescaled(snap["rescaled"])
        elif "pos" in snap:
            prior = snap.get("rescale", {}).get("prior")
            if prior is not None:
                self.restore_rescaled(prior)  # the re-split layout the positions index into
            self.pos = snap["pos"]

    def _rescale_info(self) -> dict:
        return {"rank": self.rank, "world": self.world, "pos": getattr(self, "pos", None),
                "prior": self._prior}

    def restore_rescaled(self, old: list[dict]) -> None:
        """Resume from a checkpoint written at another world size: `old` = every old rank's
        _rescale_info(). Sources whose partitions can be re-split override this."""
        raise ValueError(f"{self.name}: no restore at a different world size")

    @staticmethod
    def _consumed(old: list[dict], n_items: int):
        """Predicate over global item indices: emitted before the checkpoint whose ranks'
        positions are `old`. Old rank r's items were the indices i = r (mod G) that its own
        prior layout had not emitted, in order; it emitted the first `pos` of them."""
        g = len(old)
        old = sorted(old, key=lambda o: o["rank"])
        prior = [o.get("prior") for o in old]
        before = Source._consumed(prior[0], n_items) if prior[0] is not None else None
        bound = []
        for r, o in enumerate(old):
            idx = [i for i in range(r, n_items, g) if before is None or not before(i)]
            bound.append(idx[o["pos"]] if o["pos"] < len(idx) else n_items)
        return lambda i: (before is not None and before(i)) or i < bound[i % g]

class CollectionSource(Source):
    name = "Collection Source"

    def __init__(self, values: Iterable, batch_size: int | None = None,
                 timestamps: list[int] | None = None):
        self.values = list(values)
        self.batch = batch_size or max(1, len(self.values))
        self.timestamps = timestamps
        self.pos = 0

    def open(self, rank, world, clock):
        super().open(rank, world, clock)
        # Distributed runs: each rank is one source partition (global index i on rank i % G).
        self._all = (self.values, self.timestamps)
        idx = list(range(len(self.values)))[rank::world]
        self.values = [self.values[i] for i in idx]
        if self.timestamps is not None:
            self.timestamps = [self.timestamps[i] for i in idx]

    def restore_rescaled(self, old):
        values, ts = self._all
        done = self._consumed(old, len(values))
        idx = [i for i in range(self.rank, len(values), self.world) if not done(i)]
        self.values = [values[i] for i in idx]
        if ts is not None:
            self.timestamps = [ts[i] for i in idx]
        self.pos = 0
        self._prior = old

    def poll(self, now):
        if self.pos >= len(self.values):
            return [], True
        end = min(len(self.values), self.pos + self.batch)
        if self.columnar and self.timestamps is None:
            from .columnar import TextBatch

            lines = self.values[self.pos:end]
            self.pos = end
            return [TextBatch("\n".join(lines).encode(), len(lines))], self.pos >= len(self.values)
        out = [Rec(v, self.timestamps[i] if self.timestamps else LONG_MIN)
               for i, v in zip(range(self.pos, end), self.values[self.pos:end])]
        self.pos = end
        return out, self.pos >= len(self.values)


class TimedCollectionSource(Source):
    """Items arrive at given processing times: [(t_ms, value), ...]; `end_time` is when the
    source closes (e.g. a minute after the last line, like waiting before closing nc)."""

    name = "Timed Source"

    def __init__(self, timed: list[tuple[int, Any]], end_time: int | None = None):
        self.timed = sorted(timed, key=lambda tv: tv[0])
        self.end_time = end_time if end_time is not None else (self.timed[-1][0] if self.timed else 0)
        self.pos = 0

    def open(self, rank, world, clock):
        super().open(rank, world, clock)
        if rank != 0:
            self.timed = []
            self.end_time = 0

    def restore_rescaled(self, old):
        # every item lives on rank 0 (a non-parallel source): its position carries over
        self.pos = next(o["pos"] for o in old if o["rank"] == 0) if self.rank == 0 else 0

    def next_event_time(self):
        if self.pos < len(self.timed):
            return self.timed[self.pos][0]
        return self.end_time

    def poll(self, now):
        out = []
        while self.pos < len(self.timed) and self.timed[self.pos][0] <= now:
            v = self.timed[self.pos][1]
            if self.columnar:
                from .columnar import TextBatch

                out.append(TextBatch(v.encode(), 1))
            else:
                out.append(Rec(v))
            self.pos += 1
            break  # one line per micro-batch: a human typing into `nc`
        done = self.pos >= len(self.timed) and now >= self.end_time
        return out, done


class SlotToken:
    """A pinned ring slot lent to one TextBatch: returned to the reader once the consumer's H2D
    copy has completed (event) or the consumer copied the bytes out (consumed)."""

    __slots__ = ("slot", "event", "done")

    def __init__(self, slot: int):
        self.slot, self.event, self.done = slot, None, False

    def uploaded(self, event) -> None:
        self.event = event
        if event is None:
            self.done = True

    def consumed(self) -> None:
        self.done = True

    def ready(self, wait: bool = False) -> bool:
        if self.done:
            return True
        if self.event is None:
            return False
        if wait:
            self.event.synchronize()
            return True
        return bool(self.event.query())


def _aligned_range(path: str, rank: int, world: int) -> tuple[int, int]:
    """K18: this rank's newline-aligned byte range of the file."""
    import os as _os

    size = _os.path.getsize(path)
    lo, hi = (size * rank) // world, (size * (rank + 1)) // world

    def next_line(pos):
        if pos <= 0:
            return 0
        with open(path, "rb") as f:
            f.seek(pos - 1)
            while True:
                blk = f.read(1 << 16)
                if not blk:
                    return size
                j = blk.find(b"\n")
                if j >= 0:
                    return pos - 1 + j + 1
                pos += len(blk)

    return next_line(lo) if rank else 0, next_line(hi) if rank + 1 < world else size


_PINNED_SLOTS: dict = {}  # (bytes, pinned) -> free page-locked slot tensors, reused across jobs

# Text batch upload: "1" = the copy kernel reading the pinned slot (csrc gpu::h2d_kernel, at
# most MXS_H2D_BLOCKS workgroups so the parse of the previous batch keeps the other CUs),
# "0" = the SDMA engine (hipMemcpyAsync).
_H2D_KERNEL = __import__("os").environ.get("MXS_H2D_KERNEL", "0") == "1"
_H2D_BLOCKS = int(__import__("os").environ.get("MXS_H2D_BLOCKS", "512"))
# Pinned slots of the file reader's ring (>= 3): the reader stays up to slots - 1 chunks ahead.
_RING_SLOTS = max(3, int(__import__("os").environ.get("MXS_RING_SLOTS", "8")))
# Slots are page-locked pageable buffers (hipHostRegister) instead of pinned allocations.
_SLOT_REGISTER = __import__("os").environ.get("MXS_SLOT_REGISTER", "0") == "1"
# "1": device ingest reads the file through its mapping (csrc/text_ring.h mapped mode): the
# mapping is page-locked read-only segment by segment and every chunk goes page cache -> HBM in
# one DMA, no host memcpy. Off by default: page-locking page-cache pages the first time costs
# more than copying them (7.5 GB/s on the box, against 26 GB/s for the parallel pread into pinned
# slots; 39-56 GB/s once the pages were locked before), so it only pays for a file read again
# and again (profiles/r5_text_reader.md).
_TEXT_MMAP = __import__("os").environ.get("MXS_TEXT_MMAP", "0") == "1"
_HIP_REGISTER_READONLY = 0x08
_TEXT_SEG = 64 << 20  # page-locked segment of the mapped reader (bytes; raised to the chunk size)


def _native():
    from ..ops.native import load

    return load()


_LOCKABLE: list = []


def _mapping_lockable() -> bool:
    """Once per process: can a read-only file mapping be page-locked (hipHostRegister ReadOnly)?
    Otherwise the device ingest keeps the pread reader."""
    if not _LOCKABLE:
        import mmap
        import tempfile

        ok = False
        with tempfile.TemporaryFile() as f:
            f.write(b"\n" * 4096)
            f.flush()
            mm = mmap.mmap(f.fileno(), 4096, prot=mmap.PROT_READ, flags=mmap.MAP_SHARED)
            try:
                import numpy as np

                p = np.frombuffer(mm, dtype=np.uint8).ctypes.data  # (the view is released here)
                if _native().gpu_host_register_flags(p, 4096, _HIP_REGISTER_READONLY) == 0:
                    _native().gpu_host_unregister(p)
                    ok = True
            finally:
                mm.close()
        _LOCKABLE.append(ok)
    return _LOCKABLE[0]


_REGISTERED: list = []  # page-locked pageable buffers (kept for the process' lifetime)


def _registered_slot(nbytes: int):
    """A page-aligned ordinary host buffer, page-locked with hipHostRegister: DMA-able like a
    pinned allocation, but with the cacheable mapping of pageable memory -- the reader's copies
    from the page cache into it ran at 32 GB/s on the box against 23 GB/s into torch's pinned
    allocations (profiles/r4_reader_box.md)."""
    import torch

    raw = torch.empty(nbytes + 4096, dtype=torch.uint8)
    off = (-raw.data_ptr()) % 4096
    t = raw[off:off + nbytes]
    rc = _native().gpu_host_register(t.data_ptr(), nbytes)
    if rc:
        raise RuntimeError(f"hipHostRegister failed ({rc})")
    _REGISTERED.append(raw)
    t._mxs_registered = True
    return t


def _take_slots(nbytes: int, count: int, pin: bool) -> list:
    import torch

    reg = pin and _SLOT_REGISTER
    free = _PINNED_SLOTS.setdefault((nbytes, pin, reg), [])
    out = [free.pop() for _ in range(min(count, len(free)))]
    while len(out) < count:
        out.append(_registered_slot(nbytes) if reg else
                   torch.empty(nbytes, dtype=torch.uint8, pin_memory=pin))
    return out


def _give_slots(slots: list, pin: bool) -> None:
    if slots:
        reg = bool(getattr(slots[0], "_mxs_registered", False))
        _PINNED_SLOTS.setdefault((slots[0].numel(), pin, reg), []).extend(slots)


class TextFileSource(Source):
    name = "Text File Source"
    # Set by the planner with the device ingest: batches are read by the C++ reader
    # (csrc/reader.cpp) into pinned ring slots and handed over without a host copy;
    # ring_device: the GPU of the ingest -- the next ready slot's H2D copy is started on a copy
    # stream while the current batch is processed (copy engine || compute).
    ring = False
    ring_device = None

    def __init__(self, path: str, batch_size: int = 65536):
        self.path = path
        self.batch = batch_size
        self.lines: list[str] | None = None
        self.pos = 0
        self._ring = None

    def _open_ring(self, start: int) -> None:
        import torch

        from ..ops.native import load

        chunk = max(1 << 20, self.batch * 48)
        self._dcap = (chunk + (2 << 20) - 1) & ~((2 << 20) - 1)  # device chunk buffers
        self._pin = torch.cuda.is_available()
        threads = min(16, max(1, __import__("os").cpu_count() or 1))
        threads = int(__import__("os").environ.get("MXS_READ_THREADS", threads))  # (A/B)
        self._cstream = None
        if self.ring_device is not None and str(self.ring_device).startswith("cuda") \
                and torch.cuda.is_available():
            self._dev = torch.device(self.ring_device)
            if self._dev.index is None:
                self._dev = torch.device("cuda", torch.cuda.current_device())
            self._cstream = torch.cuda.Stream(self._dev)
        self._mapped = False
        self._slots = []
        self._nslots = _RING_SLOTS
        if _TEXT_MMAP and self._cstream is not None and _mapping_lockable():
            ring = load().TextFileRing.mapped(self.path, self.lo + start, self.hi, _RING_SLOTS,
                                              chunk, threads)
            # page-locked by the reader thread a segment at a time (whole pages, >= a chunk:
            # a chunk's copy splits at most once, at a segment boundary)
            self._seg = max(_TEXT_SEG, (chunk + 4095) & ~4095)
            ring.register_segments(self._seg, _HIP_REGISTER_READONLY)
            self._ring, self._mapped = ring, True
        if not self._mapped:
            self._slots = _take_slots(chunk, _RING_SLOTS, self._pin)
            self._ring = load().TextFileRing(self.path, self.lo + start, self.hi,
                                             [(t.data_ptr(), t.numel()) for t in self._slots],
                                             chunk, threads)
        self._ring.start()
        self._held: list = []
        self._pre = None  # prefetched (TextBatch, end offset)
        self.bpos = start
        self._ring_done = self.lo + start >= self.hi

    def open(self, rank, world, clock):
        super().open(rank, world, clock)
        if self.columnar and self.ring:
            self.lo, self.hi = _aligned_range(self.path, rank, world)
            self._open_ring(0)
            return
        if self.columnar:
            # K18: the file is split into one contiguous newline-aligned byte range per rank,
            # read in batches of ~batch lines without building Python strings.
            with open(self.path, "rb") as f:
                data = f.read()
            lo, hi = (len(data) * rank) // world, (len(data) * (rank + 1)) // world
            if rank:
                j = data.find(b"\n", lo - 1) if lo else 0
                lo = len(data) if j < 0 else j + 1
            if rank + 1 < world:
                j = data.find(b"\n", hi - 1)
                hi = len(data) if j < 0 else j + 1
            self.data = memoryview(data)[lo:max(lo, hi)]
            self.bpos = 0
            return
        with open(self.path, "r", encoding="utf-8") as f:
            lines = f.read().split("\n")
        if lines and lines[-1] == "":
            lines.pop()
        self.lines = [l[:-1] if l.endswith("\r") else l for l in lines][rank::world]

    def snapshot(self) -> dict:
        return {"bpos": self.bpos} if self.columnar else super().snapshot()

    def restore_rescaled(self, old):
        if self.columnar or self.lines is None:
            raise ValueError("text file source: the columnar reader's byte ranges cannot be "
                             "re-split at another world size")
        with open(self.path, "r", encoding="utf-8") as f:
            lines = f.read().split("\n")
        if lines and lines[-1] == "":
            lines.pop()
        lines = [l[:-1] if l.endswith("\r") else l for l in lines]
        done = self._consumed(old, len(lines))
        self.lines = [lines[i] for i in range(self.rank, len(lines), self.world) if not done(i)]
        self.pos = 0
        self._prior = old

    def restore(self, snap: dict) -> None:
        if self.columnar and "bpos" in snap:
            if self._ring is not None:
                self._ring.close()
                self._open_ring(int(snap["bpos"]))
            else:
                self.bpos = snap["bpos"]
        else:
            super().restore(snap)

    def close(self):
        if self._ring is not None:
            for t in self._held:
                t.ready(wait=True)
            if self._pre is not None:
                self._pre[0].token.ready(wait=True)
            if self._mapped:
                # every copy out of the mapping has completed: its segments are unlocked and
                # unmapped on a helper thread (~6 ms for 768 MB, no GIL held) after the job
                import threading

                threading.Thread(target=self._ring.close, name="mxs-ring-close",
                                 daemon=True).start()
            else:
                self._ring.close()
            self._ring = None
            _give_slots(self._slots, self._pin)
            self._slots = []

    def _take(self, timeout_ms: int):
        """The next filled slot as a TextBatch (+ its end offset), or None."""
        from .columnar import TextBatch

        slot, nbytes, nlines, end, eof, ptr = self._ring.next(timeout_ms)
        if slot < 0:
            if eof:
                self._ring_eof = True
            return None
        tok = SlotToken(slot)
        if self._mapped:
            # the chunk's bytes in the page-locked file mapping: one DMA on the copy stream
            import torch

            with torch.cuda.stream(self._cstream):
                # one allocation size for every chunk: the caching allocator hands the freed
                # buffers back instead of going to the driver per chunk size
                dev = torch.empty(self._dcap, dtype=torch.uint8, device=self._dev)
                off = int(ptr) - self._ring.map_base
                cut = min(int(nbytes), (off // self._seg + 1) * self._seg - off)
                for a, b in ((0, cut), (cut, int(nbytes))):  # one copy per page-locked segment
                    if b > a:
                        rc = _native().gpu_h2d_async(dev.data_ptr() + a, int(ptr) + a, b - a,
                                                     self._cstream.cuda_stream)
                        if rc:
                            raise RuntimeError(f"text upload: hip error {rc}")
                ev = torch.cuda.Event()
                ev.record(self._cstream)
            tok.uploaded(ev)
            return TextBatch(dev[:nbytes], int(nlines), token=tok, ready=ev), end
        tb = TextBatch(self._slots[slot][:nbytes], int(nlines), token=tok)
        if self._cstream is not None:
            # H2D on the copy stream now: the consumer waits for `ready` (an event) instead of
            # copying; the pinned slot is released once that copy has completed.
            import torch

            with torch.cuda.stream(self._cstream):
                r16 = (int(nbytes) + 15) & ~15
                if _H2D_KERNEL and r16 <= self._slots[slot].numel():
                    # the copy kernel reads the pinned slot over PCIe (16-byte granules: the
                    # slot's bytes past nbytes ride along and are never parsed)
                    buf = torch.empty(max(r16, 16), dtype=torch.uint8, device=self._dev)
                    rc = _native().gpu_h2d_kernel(buf.data_ptr(), self._slots[slot].data_ptr(),
                                                  r16, self._cstream.cuda_stream, _H2D_BLOCKS)
                    if rc:
                        raise RuntimeError(f"text upload: hip error {rc}")
                    dev = buf[:nbytes]
                elif getattr(self._slots[slot], "_mxs_registered", False):
                    # registered (page-locked) pageable slot: an async DMA copy; torch would
                    # take it for pageable memory and copy synchronously
                    dev = torch.empty(max(int(nbytes), 1), dtype=torch.uint8, device=self._dev)
                    rc = _native().gpu_h2d_async(dev.data_ptr(), self._slots[slot].data_ptr(),
                                                 int(nbytes), self._cstream.cuda_stream)
                    if rc:
                        raise RuntimeError(f"text upload: hip error {rc}")
                    dev = dev[:nbytes]
                else:
                    dev = torch.empty(self._dcap, dtype=torch.uint8, device=self._dev)[:nbytes]
                    dev.copy_(tb.data, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(self._cstream)
            tok.uploaded(ev)
            tb.data, tb.ready = dev, ev
        return tb, end

    def _poll_ring(self):
        # Slots whose upload completed go back to the reader.
        keep = []
        for t in self._held:
            if t.ready(wait=len(self._held) >= self._nslots - 1 and t is self._held[0]):
                self._ring.release(t.slot)
            else:
                keep.append(t)
        self._held = keep
        if self._pre is not None:
            got, self._pre = self._pre, None
        elif self._ring_done:
            return [], True
        else:
            self._ring_eof = False
            got = self._take(1000)
            if got is None:
                self._ring_done = self._ring_eof
                return [], self._ring_done
        tb, end = got
        self._held.append(tb.token)
        self.bpos = end
        self._ring_done = self.lo + end >= self.hi
        if self._cstream is not None and not self._ring_done \
                and len(self._held) < self._nslots - 1:
            self._ring_eof = False
            self._pre = self._take(0)  # prefetch: its H2D overlaps this batch's processing
        return [tb], self._ring_done and self._pre is None

    def poll(self, now):
        if self.columnar and self._ring is not None:
            return self._poll_ring()
        if self.columnar and self.ring:
            return [], True
        if self.columnar:
            from .columnar import TextBatch

            d = self.data
            if self.bpos >= len(d):
                return [], True
            end = min(len(d), self.bpos + self.batch * 48)  # ~batch lines of a metric log
            if end < len(d):
                j = bytes(d[end - 1:end]) == b"\n"
                if not j:
                    k = bytes(d[end:min(len(d), end + 4096)]).find(b"\n")
                    while k < 0 and end < len(d):
                        end = min(len(d), end + 4096)
                        k = bytes(d[end:min(len(d), end + 4096)]).find(b"\n")
                    end = len(d) if k < 0 else end + k + 1
            chunk = bytes(d[self.bpos:end])
            self.bpos = end
            n = chunk.count(b"\n") + (0 if chunk.endswith(b"\n") else 1)
            return [TextBatch(chunk, n)], self.bpos >= len(d)
        end = min(len(self.lines), self.pos + self.batch)
        out = [Rec(l) for l in self.lines[self.pos:end]]
        self.pos = end
        return out, self.pos >= len(self.lines)


class SequenceSource(Source):
    name = "Sequence Source"

    def __init__(self, start: int, end: int, batch_size: int = 65536):
        self.start, self.end, self.batch = start, end, batch_size

    def open(self, rank, world, clock):
        super().open(rank, world, clock)
        self.cur = self.start + rank
        self.step = world

    def snapshot(self) -> dict:
        return {"cur": self.cur, "rescale": {"rank": self.rank, "world": self.world,
                                             "cur": self.cur, "prior": self._prior}}

    def restore(self, snap: dict) -> None:
        if "rescaled" in snap:
            self.restore_rescaled(snap["rescaled"])
        else:
            prior = snap.get("rescale", {}).get("prior")
            if prior is not None:
                self.restore_rescaled(prior)  # keep skipping what the older layout emitted
            self.cur = snap.get("cur", self.cur)

    def _emitted(self, old: list[dict]):
        """Predicate: value x was emitted under the layout `old` (old rank r emitted its values
        start + r, start + r + G, ... below its cursor, except those its prior layout had)."""
        g = len(old)
        old = sorted(old, key=lambda o: o["rank"])
        cur = [o["cur"] for o in old]
        before = self._emitted(old[0]["prior"]) if old[0].get("prior") is not None else None
        return lambda x: (before is not None and before(x)) or x < cur[(x - self.start) % g]

    def restore_rescaled(self, old):
        self._skip = self._emitted(old)
        self._prior = old
        self.cur = self.start + self.rank

    def poll(self, now):
        out = []
        skip = getattr(self, "_skip", None)
        while self.cur <= self.end and len(out) < self.batch:
            if skip is None or not skip(self.cur):
                out.append(Rec(self.cur))
            self.cur += self.step
        return out, self.cur > self.end


class SocketTextSource(Source):
    name = "Socket Stream"

    def __init__(self, host: str, port: int, delimiter: str = "\n", max_retry: int = 0,
                 poll_timeout_ms: int = 100, max_lines: int = 1 << 16):
        self.host, self.port, self.delim, self.max_retry = host, port, delimiter, max_retry
        self.poll_timeout_ms = poll_timeout_ms
        self.max_lines = max_lines
        self.reader = None

    # Set by the executor on multi-rank jobs (host-object collectives): a columnar socket source
    # then spreads rank 0's text batches over every rank (K18, Main.java:17 -> 18 rebalance).
    comm = None
    max_queue_lines = 1 << 22  # lines buffered between the socket and the job

    def open(self, rank, world, clock):
        super().open(rank, world, clock)
        if rank != 0:
            return
        from ..ops.native import load

        # Bounded reader queue: a slow job back-pressures the sender through TCP flow control.
        self.reader = load().SocketSource(self.host, self.port, self.delim, self.max_retry,
                                          max_queue=self.max_queue_lines)
        self.reader.start()

    def _poll_spread(self):
        """Multi-rank columnar: rank 0 reads, cuts the batch into newline-aligned chunks of
        about equal size, one per rank, and every rank takes its chunk (a collective on every
        pass, so all ranks also learn end-of-stream on the same pass)."""
        from .columnar import TextBatch

        import torch

        world, rank = self.comm.world, self.comm.rank
        # Header (int64): eof, error flag, then each rank's chunk length; then the chunks as one
        # uint8 tensor. Two tensor broadcasts, no pickling (the error text alone is an object).
        head = torch.zeros(2 + world, dtype=torch.int64)
        payload = b""
        err = None
        if rank == 0:
            data, n, eof, err = self.reader.poll(self.max_lines, self.poll_timeout_ms)
            cuts = [0] * (world + 1)
            if n:
                data = bytes(data)
                cuts = [0]
                for r in range(1, world):
                    c = max(cuts[-1], len(data) * r // world)
                    j = data.find(b"\n", c - 1) if c > 0 else -1
                    cuts.append(len(data) if j < 0 else j + 1)
                cuts.append(len(data))
                payload = data
            head[0], head[1] = int(bool(eof)), int(bool(err))
            head[2:] = torch.tensor([cuts[r + 1] - cuts[r] for r in range(world)])
        self.comm.broadcast_(head, src=0)
        eof, has_err = bool(head[0]), bool(head[1])
        if has_err:
            raise ConnectionError(self.comm.broadcast_object(err, src=0))
        lens = head[2:].tolist()
        total = sum(lens)
        chunks = [b""] * world
        if total:
            buf = (torch.frombuffer(bytearray(payload), dtype=torch.uint8) if rank == 0
                   else torch.empty(total, dtype=torch.uint8))
            self.comm.broadcast_(buf, src=0)
            off = sum(lens[:rank])
            chunks[rank] = buf[off:off + lens[rank]].numpy().tobytes()
        mine = chunks[rank]
        if not mine:
            return [], eof
        return [TextBatch(mine, mine.count(b"\n") + (0 if mine.endswith(b"\n") else 1))], eof

    def poll(self, now):
        if self.columnar and self.comm is not None and self.comm.world > 1:
            return self._poll_spread()
        if self.reader is None:
            return [], True
        data, n, eof, err = self.reader.poll(self.max_lines, self.poll_timeout_ms)
        if err:
            raise ConnectionError(err)
        out = []
        if n and self.columnar:
            from .columnar import TextBatch

            return [TextBatch(bytes(data), int(n))], bool(eof)
        if n:
            text = data.decode("utf-8", errors="replace")
            parts = text.split("\n")[:n]
            out = [Rec(p) for p in parts]
        return out, bool(eof)

    def close(self):
        if self.reader is not None:
            self.reader.close()


class _SourceCtx:
    def __init__(self, q: "queue.Queue"):
        self.q = q

    def collect(self, v):
        self.q.put(Rec(v))

    def collect_with_timestamp(self, v, ts):
        self.q.put(Rec(v, int(ts)))

    def emit_watermark(self, wm):
        self.q.put(WM(int(wm.timestamp if hasattr(wm, "timestamp") else wm)))

    def get_checkpoint_lock(self):
        return threading.Lock()

    collectWithTimestamp = collect_with_timestamp
    emitWatermark = emit_watermark


class FunctionSource(Source):
    """Runs a user SourceFunction in a thread (Flink's SourceStreamTask)."""

    name = "Custom Source"

    def __init__(self, fn, batch_size: int = 65536):
        self.fn = fn
        self.batch = batch_size

    def open(self, rank, world, clock):
        super().open(rank, world, clock)
        self.q: queue.Queue = queue.Queue()
        self.done = threading.Event()
        self.err: list = []

        def run():
            try:
                if rank == 0 or getattr(self.fn, "parallel", False):
                    self.fn.run(_SourceCtx(self.q))
            except Exception as e:  # propagate to the executor
                self.err.append(e)
            finally:
                self.done.set()

        self.th = threading.Thread(target=run, daemon=True)
        self.th.start()

    def poll(self, now):
        out = []
        try:
            out.append(self.q.get(timeout=0.05))
            while len(out) < self.batch:
                out.append(self.q.get_nowait())
        except queue.Empty:
            pass
        if self.err:
            raise self.err[0]
        return out, self.done.is_set() and self.q.empty()

    def close(self):
        try:
            self.fn.cancel()
        except Exception:
            pass
