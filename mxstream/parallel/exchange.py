"""Row exchange between ranks for keyed operators without a partition kernel of their own.

``exchange_rows(comm, dest, cols)`` routes row i of every column to rank ``dest[i]`` (the
keyBy shuffle of operators whose records are not the 24-byte (key, ts, value) triple of the
window/rolling/session partition kernels: the median pane arena's (key id, ts, f64) rows, the
rolling operator's template rows). ``gather_rows(comm, cols)`` gives every rank every rank's
rows (a replicated table's new entries).

Shape of the exchange: ONE equal-split all-to-all per column of fixed-capacity
per-destination slices -- the capacity is the largest slice over all ranks, one MAX all-reduce
of an int64, so no count round trip precedes the payload -- plus an all-to-all of the
per-destination counts. Received rows come back compacted in (source rank, source row) order,
which keeps every key's rows in arrival order when each source sends its rows in order.
On RCCL the slices move over xGMI peer links; LoopbackComm and gloo move the same layout.
"""
from __future__ import annotations

import torch


def _cap(comm, counts: torch.Tensor) -> int:
    m = counts.max().reshape(1).to(torch.int64) if counts.numel() else \
        torch.zeros(1, dtype=torch.int64, device=counts.device)
    comm.allreduce_max_(m)
    return int(m.item())


def exchange_rows(comm, dest: torch.Tensor, cols: list[torch.Tensor]) -> list[torch.Tensor]:
    """Rows to their destination ranks; returns the received columns (same dtypes and trailing
    shapes). Collective: every rank calls it, with or without rows."""
    world = comm.world
    dev = dest.device
    n = dest.numel()
    if world == 1:
        return [c[:n] for c in cols]
    dest = dest.to(torch.int64)
    counts = torch.bincount(dest, minlength=world)[:world] if n else \
        torch.zeros(world, dtype=torch.int64, device=dev)
    cap = _cap(comm, counts)
    rc = torch.empty_like(counts)
    comm.all_to_all(rc, counts)
    if cap == 0:
        return [c[:0] for c in cols]
    # Stable order by destination: slot of row i = dest * cap + (rank among its destination).
    order = torch.sort(dest, stable=True).indices if n else dest
    starts = torch.cumsum(counts, 0) - counts
    ds = dest[order]
    pos = ds * cap + (torch.arange(n, device=dev, dtype=torch.int64) - starts[ds])
    # Valid received rows: source slice s holds rc[s] rows at the front.
    valid = (torch.arange(cap, device=dev).unsqueeze(0) < rc.unsqueeze(1)).reshape(-1)
    out = []
    for c in cols:
        c = c[:n]
        send = torch.zeros((world * cap,) + tuple(c.shape[1:]), dtype=c.dtype, device=dev)
        send[pos] = c[order]
        recv = torch.empty_like(send)
        comm.all_to_all(_flat(recv), _flat(send))
        out.append(recv[valid])
    return out


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
