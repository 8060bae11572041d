"""Checkpoint half of the keyed window operator (runtime/window_operator.py): state sizes,
synchronous and asynchronous snapshots (device tables cloned on the stream, the host tier and the
firing bookkeeping frozen), restore with key-group filtering (rescaling), and the merge-ring
rebuild. The tables are the native step's memory (csrc/window_step.h), seen as tensors.

Reference: chapter3/README.md:454-456 (checkpointed state survives failures).
"""
from __future__ import annotations

import numpy as np
import torch

from ..ops import kernels as K
from .host_rows import _next_pow2
from .window_types import combine_partials

I64_MIN = K.I64_MIN
I64_MAX = K.I64_MAX


def _to_host(ts: list[torch.Tensor]) -> list[np.ndarray]:
    """Device columns -> numpy: page-locked destinations (torch's caching host allocator reuses
    them from one snapshot to the next), every copy queued on the current stream, one wait."""
    if not ts or not ts[0].is_cuda:
        return [t.cpu().numpy() for t in ts]
    out = []
    for t in ts:
        h = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
        h.copy_(t, non_blocking=True)
        out.append(h)
    torch.cuda.current_stream(ts[0].device).synchronize()
    return [h.numpy() for h in out]


class _StateMixin:
    """Methods of KeyedWindowOperator (mixed in; state lives in the native step)."""

    # ---- introspection ---------------------------------------------------------------------
    def state_bytes(self) -> int:
        return sum(t.numel() * t.element_size() for t in (self.keys_g, self.acc_g, self.cnt_g,
                                                          self.dirty_g))

    def host_state_bytes(self) -> int:
        """Bytes of keyed state in the host-DRAM tier (0 without spill)."""
        if self.host_tier is None:
            return 0
        self._sync_state()
        return self.host_tier.nbytes

    def num_keys(self) -> int:
        self._sync_state()
        if self.dense_bits:  # no insertion: keys with data in a live pane
            return int((self.cnt_g.view(self.ring, self.nslots) > 0).any(0).sum().item())
        return int(self.occ.sum().item())

    def _book(self) -> dict:
        """Firing bookkeeping as of now (or as of the freeze, for a frozen copy)."""
        b = self.__dict__.get("_frozen_book")
        if b is not None:
            return b
        m = self.metrics
        return {"wm": self.wm, "next_fire_start": self.next_fire_start,
                "min_live_pane": self.min_live_pane, "max_seen_pane": self.max_seen_pane,
                "ring": self.ring,
                "metrics": {k: getattr(m, k) for k in ("num_records_in", "num_late_records_dropped",
                                                       "num_records_out", "num_fires", "steps")}}

    # ---- checkpoint / restore (runtime/checkpoint.py) --------------------------------------
    def owned_key_groups(self) -> tuple[int, int]:
        from .checkpoint import owned_key_groups

        return owned_key_groups(self.rank, self.world, self.parallelism, self.max_parallelism)

    def _check_ckpt_meta(self, meta: dict) -> None:
        for k in ("size", "slide", "offset", "agg", "time_mode"):
            if meta[k] != getattr(self, k):
                raise ValueError(f"checkpoint {k}={meta[k]!r} does not match operator "
                                 f"{getattr(self, k)!r}")

    def snapshot_state_async(self):
        """Freeze the state now (D2D clones, bookkeeping and host tier copied), export it later:
        see checkpoint.freeze_operator."""
        from .checkpoint import freeze_operator

        self._sync_state()
        book = self._book()

        def private(frozen):
            # The export runs on a worker thread while the step loop keeps going: the frozen copy
            # gets its own bookkeeping and its own tier as of now.
            frozen._frozen_book = book
            if self.host_tier is not None:
                frozen._frozen_tier = self.host_tier.copy()

        return freeze_operator(self, self._state_tensors, post=private)

    def _snapshot_tier(self):
        t = self.__dict__.get("_frozen_tier")
        return t if t is not None else self.host_tier

    def snapshot_state(self):
        """Live (key, pane) accumulators grouped by key group, plus the firing bookkeeping."""
        from .checkpoint import OperatorSnapshot

        if "_frozen_book" not in self.__dict__:
            self._sync_state()
        book = self._book()
        keys_g, cnt_g, acc_g, dirty_g = self.keys_g, self.cnt_g, self.acc_g, self.dirty_g
        ring, nslots = book["ring"], self.nslots
        live = torch.nonzero(keys_g != -1).flatten()
        cols = {"key": np.zeros(0, np.int64), "pane": np.zeros(0, np.int64),
                "acc": np.zeros(0, np.int64), "cnt": np.zeros(0, np.int32),
                "dirty": np.zeros(0, np.uint8)}
        kg = np.zeros(0, np.int32)
        lo, hi = book["min_live_pane"], book["max_seen_pane"]
        if lo is not None and live.numel():
            panes = torch.arange(lo, hi + 1, device=keys_g.device)
            idx = ((panes & (ring - 1)) * nslots)[:, None] + live[None, :]
            cnt = cnt_g[idx]
            sel = cnt > 0
            keys = keys_g[live][None, :].expand_as(idx)[sel].contiguous()
            kgd = K.keygroups(keys, max_parallelism=self.max_parallelism, hash_mode=self.hash_mode,
                              jhash=self.jhash)
            # Rows in file order (key group, stable) before they leave the device: the state file
            # writer then writes the columns as they are (csrc/kg_file.h).
            kgd, order = torch.sort(kgd, stable=True)
            at = idx[sel][order]
            kg, *vals = _to_host([kgd, keys[order], panes[:, None].expand_as(idx)[sel][order],
                                  acc_g[at], cnt[sel][order], dirty_g[at]])
            cols = dict(zip(("key", "pane", "acc", "cnt", "dirty"), vals))
        tier = self._snapshot_tier()
        if tier is not None and tier.nrows:
            # Spilled state travels in the same rows (restore folds duplicate (key, pane) rows).
            h = tier.rows()
            hk = torch.from_numpy(h["key"].view(np.int64))
            kg = np.concatenate([kg, K.keygroups(hk, max_parallelism=self.max_parallelism,
                                                 hash_mode=self.hash_mode,
                                                 jhash=None if self.jhash is None else self.jhash.cpu()
                                                 ).numpy()]).astype(np.int32)
            cols = {"key": np.concatenate([cols["key"], h["key"].view(np.int64)]),
                    "pane": np.concatenate([cols["pane"], h["pane"]]),
                    "acc": np.concatenate([cols["acc"], h["acc"]]),
                    "cnt": np.concatenate([cols["cnt"], h["cnt"].astype(np.int32)]),
                    "dirty": np.concatenate([cols["dirty"], h["dirty"]])}
        meta = {"kind": "window", "size": self.size, "slide": self.slide, "offset": self.offset,
                "lateness": self.lateness, "agg": self.agg, "time_mode": self.time_mode,
                "wm": book["wm"], "next_fire_start": book["next_fire_start"],
                "min_live_pane": lo, "max_seen_pane": hi, "metrics": book["metrics"]}
        return OperatorSnapshot(kg, cols, meta)

    def _restore_book(self, meta: dict) -> None:
        """Bookkeeping of a restore; the ring is re-laid (zeroed) to hold the live panes."""
        lo, hi = meta["min_live_pane"], meta["max_seen_pane"]
        ring = self.ring
        if lo is not None and hi - lo + 1 > ring:
            ring = _next_pow2(hi - lo + 1)
        self._s.reset_state(ring)
        self.wm = meta["wm"]
        self.next_fire_start = meta["next_fire_start"]
        self._set_live(lo, hi)
        for k, v in meta.get("metrics", {}).items():
            setattr(self.metrics, k, v)

    def restore_state(self, rows: dict, meta: dict) -> None:
        """Rebuild the tables from checkpoint rows (this rank's key groups only)."""
        self._check_ckpt_meta(meta)
        self._restore_book(meta)
        dev = self.device
        if not len(rows["key"]):
            if self.local_global:
                self._s.rebuild_merge_ring(self._stream())
            return
        keys_g, acc_g, cnt_g, dirty_g = self.keys_g, self.acc_g, self.cnt_g, self.dirty_g
        keys = torch.from_numpy(np.ascontiguousarray(rows["key"])).to(dev)
        pane = torch.from_numpy(np.ascontiguousarray(rows["pane"])).to(dev)
        acc = torch.from_numpy(np.ascontiguousarray(rows["acc"])).to(dev)
        cnt = torch.from_numpy(np.ascontiguousarray(rows["cnt"])).to(dev)
        dirty = torch.from_numpy(np.ascontiguousarray(rows["dirty"])).to(dev)
        uniq, inv = torch.unique(keys, return_inverse=True)
        occ_slots = None
        if self.dense_bits:
            if bool((uniq >> self.dense_bits).any()):
                raise RuntimeError("restore: key id outside the dense key space (raise max_keys)")
            slots_u = (uniq * self.dense_mul) & ((1 << self.dense_bits) - 1)
        elif self.host_tier is not None:
            # With the spill tier the checkpoint may hold more keys than the table: keys without
            # data in the newest spill_keep_panes panes go back to the tier (as compact_state
            # would have put them), the others are inserted; any that find no slot join the tier.
            to_tier = torch.zeros(uniq.numel(), dtype=torch.bool, device=dev)
            if self.max_seen_pane is not None:
                newest = torch.full((uniq.numel(),), I64_MIN, dtype=torch.int64, device=dev)
                newest.scatter_reduce_(0, inv, pane, "amax")
                keep = self.spill_keep_panes or self.panes_per_window
                to_tier = newest <= self.max_seen_pane - keep
            slots_u = torch.full((uniq.numel(),), -1, dtype=torch.int64, device=dev)
            hot = torch.nonzero(~to_tier).flatten()
            if hot.numel():
                slots_u[hot] = K.table_insert(uniq[hot].contiguous(), keys_g,
                                              nsub_log2=self.nsub_log2, cap_log2=self.cap_log2)
            row_tier = (slots_u < 0)[inv]
            occ_slots = slots_u[slots_u >= 0]
            if bool(row_tier.any()):
                sel = torch.nonzero(row_tier).flatten()
                self.host_tier.absorb(keys[sel].cpu().numpy().view(np.uint64),
                                      pane[sel].cpu().numpy(), acc[sel].cpu().numpy(),
                                      cnt[sel].cpu().numpy(), dirty[sel].cpu().numpy())
                sel = torch.nonzero(~row_tier).flatten()
                keys, pane, acc, cnt, dirty = keys[sel], pane[sel], acc[sel], cnt[sel], dirty[sel]
                inv = inv[sel]
                slots_u = torch.where(slots_u < 0, torch.zeros_like(slots_u), slots_u)
        else:
            slots_u = K.table_insert(uniq.contiguous(), keys_g, nsub_log2=self.nsub_log2,
                                     cap_log2=self.cap_log2)
        if bool((slots_u < 0).any()):
            raise RuntimeError("restore: keyed state does not fit the table (raise max_keys)")
        slot = slots_u[inv]
        idx = (pane & (self.ring - 1)) * self.nslots + slot
        u, inv = torch.unique(idx, return_inverse=True)
        if u.numel() == idx.numel():
            acc_g[idx], cnt_g[idx], dirty_g[idx] = acc, cnt, dirty
        else:
            # Several rows per (key, pane): partial accumulators of a local-global checkpoint
            # (every rank held a partial of every key) -- fold them with the aggregate.
            acc_g[u] = combine_partials(self.agg, acc, inv, u.numel())
            cnt_g[u] = torch.zeros(u.numel(), dtype=torch.int32, device=dev).index_add_(0, inv, cnt)
            dirty_g[u] = torch.zeros(u.numel(), dtype=torch.int32, device=dev).scatter_reduce_(
                0, inv, dirty.to(torch.int32), "amax").to(torch.uint8)
        if self.dlist is not None:
            # Rebuild the touched-slot list from the restored dirty bytes.
            ds = torch.unique(slot[dirty != 0]).to(torch.int32)
            self.dlist[:ds.numel()] = ds
            self.dlist_n.fill_(ds.numel())
            self.slot_mark[ds.long()] = 1
        occ_slots = slots_u if occ_slots is None else occ_slots
        self.occ.copy_(torch.bincount(occ_slots >> self.cap_log2, minlength=self.nsub)
                       .to(torch.int32))
        if self.local_global:
            self._s.rebuild_merge_ring(self._stream())
