"""Checkpoint half of the keyed window operator (runtime/window_operator.py): state sizes,
synchronous and asynchronous snapshots (device tables copied on a side stream, the host tier
frozen), restore with key-group filtering (rescaling), and the merge-ring rebuild.

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


class _StateMixin:
    """Methods of KeyedWindowOperator (mixed in; state lives on the operator)."""

    # ---- introspection ---------------------------------------------------------------------
    def state_bytes(self) -> int:
        return sum(t.numel() * t.element_size() for t in (self.keys_g, self.acc_g, self.cnt_g,
                                                          self.dirty_g))

    def host_state_bytes(self) -> int:
        """Bytes of keyed state in the host-DRAM tier (0 without spill)."""
        if self.host_tier is None:
            return 0
        self._land_evictions()
        return self.host_tier.nbytes

    def num_keys(self) -> int:
        self._sync_state()
        if self.dense_bits:  # no insertion: keys with data in a live pane
            return int((self.cnt_g.view(self.ring, self.nslots) > 0).any(0).sum().item())
        return int(self.occ.sum().item())

    def _sync_state(self) -> None:
        """Make the state tables current for a host reader: the pending step must be applied
        (its fired rows are kept for the next process()/flush() caller) and S1 drained."""
        if self._pending is not None:
            self._carry.extend(self.flush())
        self._drain()
        self._land_evictions()  # evicted rows still in flight belong to the tier's state

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
        """Freeze the state now (D2D copies), export it later: see checkpoint.freeze_operator."""
        from .checkpoint import freeze_operator

        self._sync_state()

        def private_tier(frozen):
            # The export reads the spill tier from a worker thread while the step loop keeps
            # absorbing / purging the live one: the frozen copy gets its own tier as of now, so
            # keys evicted after the freeze are neither lost nor exported twice.
            if self.host_tier is not None:
                frozen.host_tier = self.host_tier.copy()

        return freeze_operator(self, self._state_tensors, post=private_tier)

    def snapshot_state(self):
        """Live (key, pane) accumulators grouped by key group, plus the firing bookkeeping."""
        from .checkpoint import OperatorSnapshot

        self._sync_state()
        live = torch.nonzero(self.keys_g != -1).flatten()
        cols = {"key": np.zeros(0, np.int64), "pane": np.zeros(0, np.int64),
                "acc": np.zeros(0, np.int64), "cnt": np.zeros(0, np.int32),
                "dirty": np.zeros(0, np.uint8)}
        kg = np.zeros(0, np.int32)
        if self.min_live_pane is not None and live.numel():
            panes = torch.arange(self.min_live_pane, self.max_seen_pane + 1, device=self.device)
            idx = ((panes & (self.ring - 1)) * self.nslots)[:, None] + live[None, :]
            cnt = self.cnt_g[idx]
            sel = cnt > 0
            keys = self.keys_g[live][None, :].expand_as(idx)[sel].contiguous()
            kg = K.keygroups(keys, max_parallelism=self.max_parallelism, hash_mode=self.hash_mode,
                             jhash=self.jhash).cpu().numpy()
            cols = {"key": keys.cpu().numpy(),
                    "pane": panes[:, None].expand_as(idx)[sel].cpu().numpy(),
                    "acc": self.acc_g[idx][sel].cpu().numpy(),
                    "cnt": cnt[sel].cpu().numpy(),
                    "dirty": self.dirty_g[idx][sel].cpu().numpy()}
        if self.host_tier is not None and self.host_tier.nrows:
            # Spilled state travels in the same rows (restore folds duplicate (key, pane) rows).
            h = self.host_tier.rows()
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
                "wm": self.wm, "next_fire_start": self.next_fire_start,
                "min_live_pane": self.min_live_pane, "max_seen_pane": self.max_seen_pane,
                "metrics": {"num_records_in": self.metrics.num_records_in,
                            "num_late_records_dropped": self.metrics.num_late_records_dropped,
                            "num_records_out": self.metrics.num_records_out,
                            "num_fires": self.metrics.num_fires, "steps": self.metrics.steps}}
        return OperatorSnapshot(kg, cols, meta)

    def restore_state(self, rows: dict, meta: dict) -> None:
        """Rebuild the tables from checkpoint rows (this rank's key groups only)."""
        self._check_ckpt_meta(meta)
        if self.host_tier is not None:
            self._evict_pending = None  # rows of the replaced state
            self.host_tier.clear()
        self._pending, self._carry = None, []
        self._drain()
        dev = self.device
        self.wm = meta["wm"]
        self.metrics.current_watermark = self.wm
        self.next_fire_start = meta["next_fire_start"]
        self.min_live_pane, self.max_seen_pane = meta["min_live_pane"], meta["max_seen_pane"]
        for k, v in meta.get("metrics", {}).items():
            setattr(self.metrics, k, v)
        if self.min_live_pane is not None and self.max_seen_pane - self.min_live_pane + 1 > self.ring:
            self.ring = _next_pow2(self.max_seen_pane - self.min_live_pane + 1)
            self.acc_g = torch.zeros(self.ring * self.nslots, dtype=torch.int64, device=dev)
            self.cnt_g = torch.zeros(self.ring * self.nslots, dtype=torch.int32, device=dev)
            self.dirty_g = torch.zeros(self.ring * self.nslots, dtype=torch.uint8, device=dev)
        if not self.dense_bits:
            self.keys_g.fill_(-1)
        if self.dlist is not None:
            self.dlist_n.zero_()
            self.slot_mark.zero_()
        self.acc_g.zero_()
        self.cnt_g.zero_()
        self.dirty_g.zero_()
        self.occ.zero_()
        if self.local_global and self.lateness > 0:
            self.dacc_g = torch.zeros(self.ring * self.nslots, dtype=torch.int64, device=dev)
            self.dcnt_g = torch.zeros(self.ring * self.nslots, dtype=torch.int32, device=dev)
        if not len(rows["key"]):
            if self.local_global:
                self._rebuild_merge_ring()
            return
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
                slots_u[hot] = K.table_insert(uniq[hot].contiguous(), self.keys_g,
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
            slots_u = K.table_insert(uniq.contiguous(), self.keys_g, nsub_log2=self.nsub_log2,
                                     cap_log2=self.cap_log2)
        if bool((slots_u < 0).any()):
            raise RuntimeError("restore: keyed state does not fit the table (raise max_keys)")
        slot = slots_u[inv]
        idx = (pane & (self.ring - 1)) * self.nslots + slot
        u, inv = torch.unique(idx, return_inverse=True)
        if u.numel() == idx.numel():
            self.acc_g[idx], self.cnt_g[idx], self.dirty_g[idx] = acc, cnt, dirty
        else:
            # Several rows per (key, pane): partial accumulators of a local-global checkpoint
            # (every rank held a partial of every key) -- fold them with the aggregate.
            self.acc_g[u] = combine_partials(self.agg, acc, inv, u.numel())
            self.cnt_g[u] = torch.zeros(u.numel(), dtype=torch.int32, device=dev).index_add_(
                0, inv, cnt)
            self.dirty_g[u] = torch.zeros(u.numel(), dtype=torch.int32, device=dev).scatter_reduce_(
                0, inv, dirty.to(torch.int32), "amax").to(torch.uint8)
        if self.dlist is not None:
            # Rebuild the touched-slot list from the restored dirty bytes.
            self.slot_mark.zero_()
            ds = torch.unique(slot[dirty != 0]).to(torch.int32)
            self.dlist[:ds.numel()] = ds
            self.dlist_n.fill_(ds.numel())
            self.slot_mark[ds.long()] = 1
        occ_slots = slots_u if occ_slots is None else occ_slots
        self.occ.copy_(torch.bincount(occ_slots >> self.cap_log2, minlength=self.nsub)
                       .to(torch.int32))
        if self.local_global:
            self._rebuild_merge_ring()

    def _rebuild_merge_ring(self) -> None:
        """Local-global with allowed lateness, after a restore: the owners' merged values of the
        windows that fired but are not cleaned (a late re-firing adds deltas to them) are
        recomputed from the restored state -- the same collective exchange as a fire, without
        the emit. Every rank runs the same window sequence (identical restored bookkeeping)."""
        self.keys_m.fill_(-1)
        self.acc_m.zero_()
        self.cnt_m.zero_()
        self.dirty_m.zero_()
        self.occ_m.zero_()
        if (self.lateness <= 0 or self.next_fire_start is None or self.min_live_pane is None
                or self.wm == I64_MIN):
            return
        s = max(self._align_up(self.wm - self.size - self.lateness + 2),
                self.first_start_containing(self.pane_start(self.min_live_pane)))
        while s < self.next_fire_start:
            p0 = max(self.pane_of(s), self.min_live_pane)
            p1 = min(self.pane_of(s) + self.panes_per_window - 1, self.max_seen_pane)
            if p1 >= p0:
                self._fire_window_partials(s, p0, p1, only_dirty=False, emit=False)
            s += self.slide
