"""Row exchange between ranks for keyed operators without a partition kernel of their own.

``exchange_rows(comm, dest, cols)`` routes row i of every column to rank ``dest[i]`` (the
keyBy shuffle of operators whose records are not the 24-byte (key, ts, value) triple of the
window/rolling/session partition kernels: the median pane arena's (key id, ts, f64) rows, the
rolling operator's template rows). ``gather_rows(comm, cols)`` gives every rank every rank's
rows (a replicated table's new entries).

Shape of the exchange: the columns travel as ONE packed row (their 32-bit
words back to back) in ONE equal-split all-to-all of fixed-capacity per-destination slices,
built by the hand-written stable scatter of csrc/exchange_hip.hip (C++ twin on the CPU): no
library sort, no per-column collective. The slice capacity is the largest per-destination count
over all ranks (one MAX all-reduce), read on the host together with the received counts (one
all-to-all of int32 counts) in the exchange's ONE host read, which sizes the outputs. Received
rows come back compacted in (source rank, source row) order, which keeps every key's rows in
arrival order when each source sends its rows in order. On RCCL the slices move over xGMI peer
links; LoopbackComm and gloo move the same layout.
"""
from __future__ import annotations

import torch


def _words(c: torch.Tensor) -> int:
    per = c.element_size()
    for d in c.shape[1:]:
        per *= d
    if per % 4:
        raise ValueError("exchange_rows: a row of every column must be whole 32-bit words")
    return per // 4


class NotExchangeable(RuntimeError):
    """Some rank flagged its rows as not encodable: every rank raises it, before any payload
    moved (the caller switches every rank to its fallback together)."""


def exchange_rows(comm, dest: torch.Tensor, cols: list[torch.Tensor],
                  abort: bool = False) -> list[torch.Tensor]:
    """Rows to their destination ranks; returns the received columns (same dtypes and trailing
    shapes). Collective: every rank calls it, with or without rows. abort=True on any rank: every
    rank raises NotExchangeable after the first (small) collective."""
    from ..ops.native import load

    world = comm.world
    dev = dest.device
    n = dest.numel()
    if world == 1:
        return [c[:n] for c in cols]
    m = load()
    gpu = dev.type == "cuda"
    st = torch.cuda.current_stream(dev).cuda_stream if gpu else 0
    dest = dest.to(torch.int64).contiguous()
    cols = [c[:n].contiguous() for c in cols]
    words = [_words(c) for c in cols]
    rw = sum(words)
    counts = torch.empty(world, dtype=torch.int32, device=dev)
    flags = torch.zeros(1, dtype=torch.int32, device=dev)  # a destination outside [0, world)
    if gpu:
        blk = torch.empty(max(1, m.xrows_blocks(n) * world), dtype=torch.int32, device=dev)
        m.gpu_xrows_count(dest.data_ptr(), n, world, blk.data_ptr(), counts.data_ptr(),
                          flags.data_ptr(), st)
    else:
        m.cpu_xrows_count(dest.data_ptr(), n, world, counts.data_ptr(), flags.data_ptr())
    # [largest per-destination count, bad-destination flag]: one MAX all-reduce, so a bad
    # destination on any rank is seen by every rank before the payload exchange (all raise
    # together instead of the others blocking in the all-to-all).
    mx = torch.stack([counts.max().to(torch.int64), flags[0].to(torch.int64),
                      torch.tensor(int(abort), dtype=torch.int64, device=dev)])
    comm.allreduce_max_(mx)
    rc = torch.empty_like(counts)
    comm.all_to_all(rc, counts)
    h = torch.cat([mx, rc.to(torch.int64)]).cpu().tolist()  # one read
    if h[1]:
        raise ValueError("exchange_rows: a destination rank outside [0, world)")
    if h[2]:
        raise NotExchangeable("exchange_rows: a rank's rows are not encodable")
    h = h[:2] + h[3:]
    cap = int(h[0])
    if cap == 0:
        return [c[:0] for c in cols]
    total = sum(min(x, cap) for x in h[2:])
    send = torch.empty(world * cap * rw, dtype=torch.int32, device=dev)
    ovf = torch.zeros(1, dtype=torch.int32, device=dev)
    spec_send = [(c.data_ptr(), 0, w) for c, w in zip(cols, words)]
    if gpu:
        m.gpu_xrows_scatter(dest.data_ptr(), n, world, blk.data_ptr(), cap, spec_send,
                            send.data_ptr(), ovf.data_ptr(), st)
    else:
        m.cpu_xrows_scatter(dest.data_ptr(), n, world, cap, spec_send, send.data_ptr(),
                            ovf.data_ptr())
    recv = torch.empty_like(send)
    comm.all_to_all(recv, send)
    outs = [torch.empty((total,) + tuple(c.shape[1:]), dtype=c.dtype, device=dev) for c in cols]
    spec_recv = [(0, o.data_ptr(), w) for o, w in zip(outs, words)]
    if gpu:
        m.gpu_xrows_unpack(recv.data_ptr(), rc.data_ptr(), world, cap, spec_recv, st)
    else:
        m.cpu_xrows_unpack(recv.data_ptr(), rc.data_ptr(), world, cap, spec_recv)
    return outs


def exchange_records(comm, outs: list[list], last_wm: int | None):
    """The keyBy edge of host (Python) operators: ``outs[r]`` = this rank's records (``Rec``)
    for rank r. Records travel code-free and typed (runtime/statecodec.py JSON of each
    destination's (value, timestamp) list, no pickle) as 32-bit words through ONE exchange_rows
    call -- a destination receives only its own records, O(N) bytes per pass instead of every
    rank's records on every rank. Returns (received records in source-rank order, every rank's
    last watermark). Raises NotExchangeable on every rank when a value has no typed encoding on
    some rank (the caller falls back to the object collective on every rank together)."""
    import numpy as np

    from ..runtime.operators import LONG_MIN, Rec
    from ..runtime.statecodec import _Enc, decode

    world = comm.world
    blobs, abort = [], False
    for r in range(world):
        try:
            enc = _Enc()
            tree = [[enc.enc(it.value), it.ts] for it in outs[r]]
            if enc.arrays:
                raise TypeError("numpy arrays inside records")
            import json

            blobs.append(json.dumps(tree, allow_nan=False, separators=(",", ":")).encode()
                         if outs[r] else b"")
        except TypeError:
            abort, blobs = True, [b""] * world
            break
    # one blob per destination: [nbytes u32][bytes padded to 4]; every word tagged with its rank
    words, dest = [], []
    for r, b in enumerate(blobs):
        if not b:
            continue
        pad = (-len(b)) % 4
        w = np.frombuffer(len(b).to_bytes(4, "little") + b + b"\0" * pad, dtype=np.int32)
        words.append(w)
        dest.append(np.full(len(w), r, dtype=np.int64))
    # (RCCL moves device tensors: the words go through the GPU exchange kernels there)
    dev = (torch.device("cuda", torch.cuda.current_device())
           if getattr(comm, "backend", "") == "nccl" else torch.device("cpu"))
    wv = torch.from_numpy(np.concatenate(words)) if words else torch.empty(0, dtype=torch.int32)
    dv = torch.from_numpy(np.concatenate(dest)) if dest else torch.empty(0, dtype=torch.int64)
    # every rank's last watermark: one all-to-all of world int64 (rank r sends its value to all)
    wm = torch.full((world,), LONG_MIN if last_wm is None else int(last_wm), dtype=torch.int64,
                    device=dev)
    all_wm = torch.empty_like(wm)
    comm.all_to_all(all_wm, wm)
    got = exchange_rows(comm, dv.to(dev), [wv.to(dev)], abort=abort)[0].cpu().numpy()
    got = got.view(np.uint8).tobytes()
    recv, o = [], 0
    while o < len(got):
        nb = int.from_bytes(got[o:o + 4], "little")
        for v, ts in decode(got[o + 4:o + 4 + nb].decode()):
            recv.append(Rec(v, ts))
        o += 4 + nb + ((-nb) % 4)
    return recv, [None if w == LONG_MIN else w for w in all_wm.tolist()]


def gather_rows(comm, cols: list[torch.Tensor]) -> list[torch.Tensor]:
    """Every rank's rows on every rank, in rank order. Collective."""
    world = comm.world
    if world == 1:
        return list(cols)
    n = cols[0].shape[0]
    dev = cols[0].device
    dest = torch.arange(world, device=dev, dtype=torch.int64).repeat_interleave(n)
    rep = [c.repeat((world,) + (1,) * (c.dim() - 1)) for c in cols]
    return exchange_rows(comm, dest, rep)


def _flat(t: torch.Tensor) -> torch.Tensor:
    """A 1-D view the equal-split all-to-all can cut (byte view of narrow or 2-D dtypes)."""
    if t.dtype == torch.bool:
        t = t.view(torch.uint8)
    return t.reshape(-1)
