"""Device text ingest: text batch -> typed device columns + a device string dictionary.

This is the GPU path behind ``socketTextStream(..).map(split + parse)`` of every reference job
(``Main.java:17-24``, ``ComputeCpuMax.java:16-23``, ``BandwidthMonitorWithEventTime.java:28-45``;
SURVEY.md K1/K2). A batch goes H2D once (from a pinned staging slot) and is parsed by five
stream-ordered launches (csrc/ingest.h): line starts, the parse with dictionary probes, the
new-string compaction + id assignment, and the id resolve. String fields become **dense
dictionary ids** that the keyed operators' dense state addresses directly; the ids equal the host
``StringDict``'s (first appearance order), so a job gets the same ids on the CPU and the GPU.

``DeviceDict`` keeps the strings in HBM (hash table, id -> (offset, length, Java hash), byte
arena); the host mirrors the names lazily, only when an operator needs a key's name (a fired row
reaching a host sink, a checkpoint). One host synchronisation per batch reads back a handful of
counters (flagged lines, max timestamp, filter total, dictionary counters).

On the CPU the same pipeline runs the C++ twins (csrc/ingest_cpu.cpp): identical outputs, so the
device ingest path of the DataStream API is covered by the CPU test suite.
"""
from __future__ import annotations

import numpy as np
import torch

from .native import load
from .text import FK_DOUBLE, FK_STR

I64_MIN = -(1 << 63)
I64_MAX = (1 << 63) - 1
FK_ISO_SEC = 7


def _spin(ev) -> None:
    """hipEventQuery polled in C++ with the GIL released (runtime/host_rows._event_spin)."""
    from ..runtime.host_rows import _event_spin

    _event_spin(ev)

def _pow2(x: int) -> int:
    return 1 << max(1, int(x - 1).bit_length())


def count_lines(data) -> int:
    """Lines of a text batch ('\\n'-separated; a trailing newline starts no line)."""
    if isinstance(data, (bytes, bytearray, memoryview)):
        b = bytes(data) if isinstance(data, memoryview) else data
        if not b:
            return 0
        return b.count(b"\n") + (0 if b.endswith(b"\n") else 1)
    arr = data.numpy() if isinstance(data, torch.Tensor) else np.asarray(data)
    if not arr.size:
        return 0
    return int(np.count_nonzero(arr == 10)) + (0 if arr[-1] == 10 else 1)


class DictionaryError(RuntimeError):
    pass


class DeviceDict:
    """String <-> dense id dictionary resident on `device` (HBM on a GPU)."""

    def __init__(self, device="cpu", cap: int = 4096, id_cap: int = 1024, arena_cap: int = 1 << 16):
        self.device = torch.device(device)
        self.cuda = self.device.type == "cuda"
        self._m = load()
        dev = self.device
        self._alloc_table(_pow2(cap))
        self.id_off = torch.zeros(id_cap, dtype=torch.int64, device=dev)
        self.id_len = torch.zeros(id_cap, dtype=torch.int32, device=dev)
        self.id_jh = torch.zeros(id_cap, dtype=torch.int32, device=dev)
        self.arena = torch.zeros(arena_cap, dtype=torch.uint8, device=dev)
        self.ctr = torch.zeros(4, dtype=torch.int64, device=dev)
        self.n_ids = 0           # ids that exist (exact after every batch's readback)
        self.arena_used = 0
        self._names: list[str] = []
        self._arena_synced = 0   # arena bytes mirrored on the host

    # ---- storage ------------------------------------------------------------------------------
    def _alloc_table(self, cap: int) -> None:
        dev = self.device
        self.cap = cap
        self.tab_h = torch.zeros(cap, dtype=torch.int64, device=dev)
        self.tab_id = torch.full((cap,), -1, dtype=torch.int32, device=dev)
        self.tab_first = torch.full((cap,), I64_MAX, dtype=torch.int64, device=dev)

    def state(self) -> dict:
        return {"tab_h": self.tab_h.data_ptr(), "tab_id": self.tab_id.data_ptr(),
                "tab_first": self.tab_first.data_ptr(), "cap": self.cap,
                "id_off": self.id_off.data_ptr(), "id_len": self.id_len.data_ptr(),
                "id_jh": self.id_jh.data_ptr(), "arena": self.arena.data_ptr(),
                "arena_cap": self.arena.numel(), "id_cap": self.id_off.numel(),
                "ctr": self.ctr.data_ptr()}

    def _stream(self) -> int:
        return torch.cuda.current_stream(self.device).cuda_stream if self.cuda else 0

    @staticmethod
    def _grow(t: torch.Tensor, n: int, fill=0) -> torch.Tensor:
        if t.numel() >= n:
            return t
        out = torch.full((_pow2(n),), fill, dtype=t.dtype, device=t.device)
        out[:t.numel()].copy_(t)
        return out

    def reserve(self, new_strings: int, new_bytes: int) -> bool:
        """Capacity for up to `new_strings` more ids / `new_bytes` more arena bytes: the table stays
        at most half full, so probes are short and an insert always finds a slot. Growth is
        stream-ordered (no host sync). Returns True when the table was rehashed (slots moved)."""
        need = self.n_ids + int(new_strings)
        moved = False
        if 2 * need > self.cap:
            old_h, old_id, old_cap = self.tab_h, self.tab_id, self.cap
            self._alloc_table(_pow2(2 * need))
            self._m.dict_rehash(self.cuda, old_h.data_ptr(), old_id.data_ptr(), old_cap,
                                self.state(), self._stream())
            moved = True
        self.id_off = self._grow(self.id_off, need)
        self.id_len = self._grow(self.id_len, need)
        self.id_jh = self._grow(self.id_jh, need)
        self.arena = self._grow(self.arena, self.arena_used + int(new_bytes))
        return moved

    def add_agreed(self, strings: list[bytes]) -> None:
        """Append an agreed list of new strings (several ranks: every rank adds the same list
        in the same order, so ids agree): string i gets id n_ids + i."""
        if not strings:
            return
        self.reserve(len(strings), sum(len(b) for b in strings))
        buf = b"".join(strings)
        lens = np.fromiter((len(b) for b in strings), dtype=np.int32, count=len(strings))
        offs = np.zeros(len(strings), dtype=np.int64)
        offs[1:] = np.cumsum(lens[:-1], dtype=np.int64)
        dev = self.device
        tb = torch.from_numpy(np.frombuffer(buf, dtype=np.uint8).copy() if buf else
                              np.zeros(1, np.uint8)).to(dev)
        to = torch.from_numpy(offs).to(dev)
        tl = torch.from_numpy(lens).to(dev)
        self._m.dict_insert_ids(self.cuda, tb.data_ptr(), to.data_ptr(), tl.data_ptr(),
                                len(strings), self.n_ids, self.state(), self._stream())
        self.n_ids += len(strings)
        self.arena_used += len(buf)

    def note_counters(self, ctr: list[int]) -> None:
        """Host view of the device counters after a batch (read back with the batch's other
        counters); raises on a dictionary error."""
        n_ids, used, err = int(ctr[0]), int(ctr[1]), int(ctr[2])
        if err:
            what = []
            if err & 1:
                what.append("table full")
            if err & 2:
                what.append("two different strings with the same 64-bit hash")
            if err & 4:
                what.append("id / arena capacity exceeded")
            raise DictionaryError("device string dictionary: " + ", ".join(what))
        self.n_ids, self.arena_used = n_ids, used

    # ---- host mirror --------------------------------------------------------------------------
    def _sync_names(self) -> None:
        k0, k1 = len(self._names), self.n_ids
        if k1 <= k0:
            return
        offs = self.id_off[k0:k1].cpu().numpy()
        lens = self.id_len[k0:k1].cpu().numpy()
        lo = int(offs.min())
        hi = int((offs + lens).max())
        raw = self.arena[lo:hi].cpu().numpy().tobytes()
        self._names.extend(raw[o - lo:o - lo + n].decode("utf-8", errors="replace")
                           for o, n in zip(offs.tolist(), lens.tolist()))
        self._arena_synced = max(self._arena_synced, hi)

    def get(self, i: int) -> str:
        i = int(i)
        if i >= len(self._names):
            self._sync_names()
        if not 0 <= i < len(self._names):
            raise IndexError(f"dictionary id {i} out of range")
        return self._names[i]

    def strings(self) -> list[str]:
        self._sync_names()
        return list(self._names)

    def jhash_table(self) -> np.ndarray:
        return self.id_jh[:self.n_ids].cpu().numpy().copy()

    def __len__(self) -> int:
        return self.n_ids

    def intern_many(self, strings: list[str]) -> np.ndarray:
        """Ids of `strings` (new ones appended in order) -- restore / host-side keys."""
        if not strings:
            return np.zeros(0, dtype=np.int64)
        if any("\n" in s or "\r" in s for s in strings):
            raise ValueError("dictionary strings cannot contain line breaks")
        text = ("\n".join(strings) + "\n").encode("utf-8")
        ing = TextIngest([(0, FK_STR)], sep="\n", device=self.device, dictionary=self)
        res = ing.parse(text)
        return res.cols[0].to(torch.int64).cpu().numpy()

    def intern(self, s: str) -> int:
        return int(self.intern_many([s])[0])


class IngestResult:
    """One parsed batch: `cols[j]` is the device column of output field j (int32 dictionary ids
    for strings, float64 or int64 otherwise); `ts` the timestamp column (the spec's ts field)."""

    def __init__(self, n, cols, ts, max_ts, line_idx, n_lines):
        self.n, self.cols, self.ts, self.max_ts = n, cols, ts, max_ts
        self.line_idx = line_idx      # input line of every kept row (None: all lines, in order)
        self.n_lines = n_lines


class _PendingParse:
    """A batch whose parse is enqueued (TextIngest.begin) and whose control words are on their
    way to pinned memory; TextIngest.finish completes it."""

    __slots__ = ("data", "keep_alive", "buf", "starts", "status", "cols", "ids", "n", "fidx",
                 "fscr", "ocols", "oids", "hb", "ev")

    def __init__(self, **kw):
        for k, v in kw.items():
            setattr(self, k, v)


class TextIngest:
    """Parser of one text layout (separator + fields) onto `device`; see the module docstring.

    fields: (split index, FK_* kind) per output column; ts_field: the column whose values are the
    event timestamps (its batch maximum drives the watermark); filter_prog: a traced predicate
    over the output columns (var j = column j), compacted on the device in input order."""

    def __init__(self, fields, sep: str = " ", offset_s: int = 0, ts_field: int = -1,
                 device="cpu", dictionary: DeviceDict | None = None, filter_prog=None):
        if not 1 <= len(fields) <= 8:
            raise ValueError("1..8 fields")
        if len(sep.encode()) != 1:
            raise ValueError("separator must be one byte")
        self.fields = [(int(f), int(k)) for f, k in fields]
        self.kinds = tuple(k for _, k in self.fields)
        self.nf = len(self.fields)
        self.str_cols = [j for j, k in enumerate(self.kinds) if k == FK_STR]
        self.nstr = len(self.str_cols)
        self.sep, self.offset_s, self.ts_field = sep, int(offset_s), int(ts_field)
        self.device = torch.device(device)
        self.cuda = self.device.type == "cuda"
        self.dict = dictionary if dictionary is not None else DeviceDict(self.device)
        if self.dict.device != self.device:
            raise ValueError("dictionary and parser on different devices")
        self.filter_prog = filter_prog if (filter_prog is not None and filter_prog.code) else None
        self._m = load()
        self._spec = {"fields": [f for f, _ in self.fields], "kinds": list(self.kinds),
                      "ts_col": self.ts_field, "offset_s": self.offset_s, "sep": sep}
        self._ws: dict = {}
        self._pins: list = []
        self._pin_i = 0
        self._hbuf = None
        self.dbl_mask = sum(1 << j for j, k in enumerate(self.kinds) if k == FK_DOUBLE)
        self.stats = {"batches": 0, "lines": 0, "flagged_lines": 0, "bytes": 0}

    # ---- buffers ------------------------------------------------------------------------------
    def _buf(self, name: str, n: int, dtype) -> torch.Tensor:
        t = self._ws.get(name)
        if t is None or t.numel() < n or t.dtype != dtype:
            t = torch.empty(_pow2(max(n, 1)), dtype=dtype, device=self.device)
            self._ws[name] = t
        return t

    def _stream(self) -> int:
        return torch.cuda.current_stream(self.device).cuda_stream if self.cuda else 0

    def _upload(self, data) -> tuple[torch.Tensor, object]:
        """The text on the device (+ the host object that keeps host memory alive)."""
        if isinstance(data, torch.Tensor):
            if data.dtype != torch.uint8 or data.dim() != 1:
                raise ValueError("text batch tensor must be 1-D uint8")
            if data.device == self.device:
                return data, data
            return data.to(self.device, non_blocking=data.is_pinned()), data
        raw = np.frombuffer(bytes(data) if isinstance(data, memoryview) else data, dtype=np.uint8)
        if not self.cuda:
            return torch.from_numpy(raw.copy()), raw
        # A pinned staging slot (two, reused once the H2D that last read them has completed).
        n = raw.size
        if len(self._pins) < 2:
            self._pins.append([None, None])
        slot = self._pins[self._pin_i]
        self._pin_i ^= 1
        if slot[1] is not None:
            slot[1].synchronize()
        if slot[0] is None or slot[0].numel() < n:
            slot[0] = torch.empty(_pow2(max(n, 1 << 16)), dtype=torch.uint8, pin_memory=True)
        slot[0][:n].numpy()[:] = raw
        dev = slot[0][:n].to(self.device, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.device))
        slot[1] = ev
        return dev, slot[0]

    # ---- parse ----------------------------------------------------------------------------------
    def parse(self, data, nlines: int | None = None, on_upload=None, agree=None,
              ready=None) -> IngestResult:
        """on_upload(event): called with a device event recorded after the H2D copy of a host
        tensor input (its pinned slot may be reused once the event completed).

        agree(list[bytes]) -> list[bytes]: several ranks share one id space (keyBy across GPUs
        needs the same id for the same string everywhere): the batch's new strings go to `agree`
        (a collective: every rank's new strings, in rank order, deduplicated), every rank appends
        the agreed list to its dictionary, and the batch is resolved against it."""
        p = self.begin(data, nlines, on_upload, agree, ready)
        return p if isinstance(p, IngestResult) else self.finish(p)

    def begin(self, data, nlines: int | None = None, on_upload=None, agree=None, ready=None):
        """Enqueue a batch's whole parse -- upload, line starts, parse + dictionary probes, id
        assignment, filter compaction, gather -- and the copy of its control words to pinned
        memory, with NO host wait: finish() reads them (one batch later in the deferred ingest of
        TextParseOp, so the host's work on batch i overlaps the GPU's parse of batch i + 1).
        Returns a pending handle (or the IngestResult of an empty batch)."""
        m = self._m
        n = count_lines(data) if nlines is None else int(nlines)
        nbytes = len(data) if not isinstance(data, torch.Tensor) else data.numel()
        self.stats["batches"] += 1
        self.stats["lines"] += n
        self.stats["bytes"] += nbytes
        if n == 0:
            if agree is not None:
                self.dict.add_agreed(agree([]))
            empty = [torch.empty(0, dtype=torch.int32 if k == FK_STR else
                                 (torch.float64 if k == FK_DOUBLE else torch.int64), device=self.device)
                     for k in self.kinds]
            return IngestResult(0, empty, None if self.ts_field < 0 else empty[self.ts_field],
                                None, None, 0)
        if ready is not None and self.cuda:
            # Device text copied by the source on its copy stream: order after that copy, and
            # let the allocator know this stream uses the buffer.
            torch.cuda.current_stream(self.device).wait_event(ready)
            data.record_stream(torch.cuda.current_stream(self.device))
        buf, keep_alive = self._upload(data)
        if on_upload is not None:
            ev = None
            if self.cuda:
                ev = torch.cuda.Event()
                ev.record(torch.cuda.current_stream(self.device))
            on_upload(ev)
        dev, st = self.device, self._stream()
        nf, S = self.nf, self.nstr
        # Two sets of per-batch workspace (a deferred batch's status / line starts are read by
        # its host patch after the next batch was enqueued).
        par = self._par = getattr(self, "_par", 0) ^ 1
        ctl = self._buf("ctl", 8, torch.int64)[:8]
        ctl.zero_()
        ctl[1] = I64_MIN
        starts = self._buf(f"starts{par}", n + 64, torch.int64)
        if self.cuda:
            scratch = self._buf("scratch", max(m.gpu_filter_compact_scratch_bytes(max(nbytes, n * max(S, 1))), 1),
                                torch.uint8)
            m.gpu_line_starts(buf.data_ptr(), nbytes, scratch.data_ptr(), starts.data_ptr(),
                              ctl[3:4].data_ptr(), st)
        else:
            scratch = self._buf("scratch", 1, torch.uint8)
            m.cpu_line_starts(buf.data_ptr(), nbytes, starts.data_ptr(), ctl[3:4].data_ptr())
        # A batch still in flight may add up to its own bound of new strings / bytes (the host's
        # id count learns them at its finish()).
        infl = getattr(self, "_inflight", None)
        if infl is None:
            infl = self._inflight = {}
        self.dict.reserve(n * S + sum(a for a, _ in infl.values()),
                          nbytes + sum(b for _, b in infl.values()))
        # Output columns are fresh per batch (consumers may hold a batch across ticks); the
        # per-string work arrays are workspace.
        cols = torch.empty(nf * n, dtype=torch.int64, device=dev)
        ids = torch.empty(max(S, 1) * n, dtype=torch.int32, device=dev)
        status = self._buf(f"status{par}", n, torch.uint8)
        np_ = max(n * S, 1)
        out = {"cols": cols.data_ptr(), "ids": ids.data_ptr(), "status": status.data_ptr(),
               "spos": self._buf("spos", np_, torch.int64).data_ptr(),
               "slen": self._buf("slen", np_, torch.int32).data_ptr(),
               "sjh": self._buf("sjh", np_, torch.int32).data_ptr(),
               "sslot": self._buf("sslot", np_, torch.int32).data_ptr(),
               "shash": self._buf("shash", np_, torch.int64).data_ptr(),
               "nflag": ctl[0:1].data_ptr(), "maxts": ctl[1:2].data_ptr(),
               "tile_max": self._buf("tilemax", (n + 255) // 256, torch.int64).data_ptr()}
        ds = self.dict.state()
        m.ingest_parse(self.cuda, buf.data_ptr(), nbytes, starts.data_ptr(), n, self._spec, out,
                       ds, st)
        if S and agree is None:
            newpos = self._buf("newpos", np_, torch.int64)
            m.dict_assign_new(self.cuda, buf.data_ptr(), n, S, out, ds, scratch.data_ptr(),
                              newpos.data_ptr(), st)
        elif agree is not None:
            self._agree_ids(agree, data, keep_alive, buf, nbytes, starts, n, out, scratch)
        fidx = fscr = ocols = oids = None
        if self.filter_prog is not None:
            # fresh per batch: the kept rows' line indices leave with the batch (line_idx)
            fidx = torch.empty(n, dtype=torch.int64, device=dev)
            fscr = (self._buf("fscratch", m.gpu_filter_compact_scratch_bytes(n), torch.uint8)
                    if self.cuda else scratch)
            m.ingest_filter_compact(self.cuda, cols.data_ptr(), n, nf, self.dbl_mask,
                                    self.filter_prog.code, self.filter_prog.consts,
                                    fscr.data_ptr(), fidx.data_ptr(), ctl[2:3].data_ptr(), st)
            # the kept rows, gathered with the device count (sized for every line)
            ocols = torch.empty(nf * n, dtype=torch.int64, device=dev)
            oids = torch.empty(max(S, 1) * n, dtype=torch.int32, device=dev)
            m.ingest_gather(self.cuda, cols.data_ptr(), n, nf, ids.data_ptr(), S,
                            fidx.data_ptr(), ctl[2:3].data_ptr(), ocols.data_ptr(),
                            oids.data_ptr(), n, st)
        # ---- the batch's control words + dictionary counters -> pinned memory (no wait) ----
        hb = self._hbuf_for(par)
        ev = None
        if self.cuda:
            hb[:8].copy_(ctl, non_blocking=True)
            hb[8:12].copy_(self.dict.ctr, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(self.device))
        else:
            hb[:8].copy_(ctl)
            hb[8:12].copy_(self.dict.ctr)
        p = _PendingParse(data=data, keep_alive=keep_alive, buf=buf, starts=starts,
                          status=status, cols=cols, ids=ids, n=n, fidx=fidx, fscr=fscr,
                          ocols=ocols, oids=oids, hb=hb, ev=ev)
        infl[id(p)] = (n * S, nbytes)  # new strings / bytes it may add, until its finish()
        return p

    def _hbuf_for(self, par: int) -> torch.Tensor:
        hb = getattr(self, "_hbufs", None)
        if hb is None:
            pin = self.cuda
            hb = self._hbufs = [torch.zeros(12, dtype=torch.int64, pin_memory=pin)
                                for _ in range(2)]
        return hb[par]

    def finish(self, p: "_PendingParse") -> IngestResult:
        """The batch's one host synchronisation (usually long complete when deferred): counters,
        dictionary errors, host patch of flagged lines, then the (kept) columns."""
        m, nf, S, n = self._m, self.nf, self.nstr, p.n
        if p.ev is not None:
            _spin(p.ev)  # poll: a blocking wait wakes tens of microseconds late
        h = p.hb.tolist()
        self._inflight.pop(id(p), None)
        nflag, max_ts, ftotal, ltotal = h[0] & 0xFFFFFFFF, h[1], h[2], h[3]
        if ltotal != n:
            raise RuntimeError(f"ingest: {ltotal} line starts on the device, {n} counted")
        self.dict.note_counters(h[8:12])
        max_ts = None if max_ts == I64_MIN else max_ts
        if nflag:
            self.stats["flagged_lines"] += nflag
            max_ts = self._host_patch(p.data, p.keep_alive, p.buf, p.starts, p.status, p.cols, n,
                                      max_ts)
            if self.filter_prog is not None:
                st = self._stream()
                ctl = self._buf("ctl", 8, torch.int64)[:8]
                m.ingest_filter_compact(self.cuda, p.cols.data_ptr(), n, nf, self.dbl_mask,
                                        self.filter_prog.code, self.filter_prog.consts,
                                        p.fscr.data_ptr(), p.fidx.data_ptr(),
                                        ctl[2:3].data_ptr(), st)
                m.ingest_gather(self.cuda, p.cols.data_ptr(), n, nf, p.ids.data_ptr(), S,
                                p.fidx.data_ptr(), ctl[2:3].data_ptr(), p.ocols.data_ptr(),
                                p.oids.data_ptr(), n, st)
                ftotal = int(ctl[2].item())
        if self.filter_prog is not None:
            k = int(ftotal)
            return self._result(p.ocols, p.oids, n, k, max_ts, p.fidx[:k], n)
        return self._result(p.cols, p.ids, n, n, max_ts, None, n)

    def _agree_ids(self, agree, data, keep_alive, buf, nbytes, starts, n, out, scratch) -> None:
        """Several ranks: this batch's new strings -> agree() -> the agreed list appended on every
        rank -> resolve. One extra host round trip per batch (the new strings' positions)."""
        m, S, st = self._m, self.nstr, self._stream()
        local: list[bytes] = []
        if S:
            np_ = n * S
            newpos = self._buf("newpos", np_, torch.int64)
            m.dict_find_new(self.cuda, n, S, out, self.dict.state(), scratch.data_ptr(),
                            newpos.data_ptr(), st)
            k = int(self.dict.ctr[3].item())
            if k:
                pos = newpos[:k]
                spos = self._ws["spos"][pos].cpu().numpy()
                slen = self._ws["slen"].index_select(0, pos).cpu().numpy()
                if isinstance(data, torch.Tensor):
                    raw = (data if data.device.type == "cpu" else data.cpu()).numpy()
                    local = [raw[a:a + b].tobytes() for a, b in zip(spos.tolist(), slen.tolist())]
                else:
                    mv = bytes(data)
                    local = [mv[a:a + b] for a, b in zip(spos.tolist(), slen.tolist())]
        agreed = agree(local)
        if agreed:
            moved = self.dict.reserve(len(agreed), sum(len(b) for b in agreed))
            if moved:
                # The rehash dropped this batch's claimed-but-unassigned slots: insert the agreed
                # list into the new table, then probe the batch again (every string now has an id).
                self.dict.add_agreed(agreed)
                ctl = self._ws["ctl"][:8]
                m.ingest_parse(self.cuda, buf.data_ptr(), nbytes, starts.data_ptr(), n,
                               self._spec, dict(out, nflag=ctl[6:7].data_ptr(),
                                                maxts=ctl[7:8].data_ptr()),
                               self.dict.state(), st)
            else:
                self.dict.add_agreed(agreed)
        if S:
            m.dict_resolve(self.cuda, buf.data_ptr(), n, S, out, self.dict.state(), st)

    def _result(self, cols, ids, stride, k, max_ts, line_idx, n_lines) -> IngestResult:
        out = []
        for j, kind in enumerate(self.kinds):
            if kind == FK_STR:
                s = self.str_cols.index(j)
                out.append(ids[s * stride:s * stride + k])
            else:
                c = cols[j * stride:j * stride + k]
                out.append(c.view(torch.float64) if kind == FK_DOUBLE else c)
        ts = None if self.ts_field < 0 else out[self.ts_field]
        return IngestResult(k, out, ts, max_ts, line_idx, n_lines)

    def _readback(self, ctl: torch.Tensor, dctr: torch.Tensor) -> list[int]:
        if not self.cuda:
            return ctl.tolist() + dctr.tolist()
        if self._hbuf is None:
            self._hbuf = torch.zeros(12, dtype=torch.int64, pin_memory=True)
        self._hbuf[:8].copy_(ctl, non_blocking=True)
        self._hbuf[8:12].copy_(dctr, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.device))
        _spin(ev)  # poll: a blocking wait wakes tens of microseconds late
        return self._hbuf.tolist()

    def _host_patch(self, data, keep_alive, buf, starts, status, cols, n, max_ts):
        """Lines the kernel flagged: the C++ runtime parses them (exact Java semantics and
        exception text) and their numeric fields are patched into the device columns."""
        from .text import ParseError

        m = self._m
        bad = torch.nonzero(status[:n]).flatten().cpu().numpy()
        if isinstance(data, torch.Tensor):
            raw = (data if data.device.type == "cpu" else data.cpu()).numpy().tobytes()
        else:
            raw = bytes(data)
        st_h = starts[:n].cpu().numpy()
        ends = np.append(st_h[1:] - 1, len(raw))
        lines = []
        for i in bad.tolist():
            line = raw[st_h[i]:ends[i]]
            if line.endswith(b"\n"):
                line = line[:-1]
            if line.endswith(b"\r"):
                line = line[:-1]
            lines.append(line)
        d = m.StringDict()
        res_cols, _, err_idx, err = m.parse_lines(b"\n".join(lines) + b"\n", self.fields,
                                                  self.sep, d, self.offset_s)
        if err:
            kind = err.split(":", 1)[0]
            msg = err.split(": ", 1)[1] if ": " in err else err
            from ..api import java as J

            exc = {"NumberFormatException": J.NumberFormatException,
                   "ArrayIndexOutOfBoundsException": J.ArrayIndexOutOfBoundsException}.get(kind)
            if exc is not None:
                raise exc(msg)
            raise ParseError(f"line {int(bad[err_idx]) + 1}: {err}")
        idx = torch.from_numpy(bad.astype(np.int64)).to(self.device)
        for j, kind in enumerate(self.kinds):
            if kind == FK_STR:
                continue  # string fields of flagged lines were interned by the device
            vals = res_cols[j]
            if kind == FK_DOUBLE:
                vals = np.asarray(vals, dtype=np.float64).view(np.int64)
            v = np.ascontiguousarray(vals, dtype=np.int64)
            cols[j * n + idx] = torch.from_numpy(v).to(self.device)
            if j == self.ts_field and v.size:
                mx = int(v.max())
                max_ts = mx if max_ts is None else max(max_ts, mx)
        return max_ts
