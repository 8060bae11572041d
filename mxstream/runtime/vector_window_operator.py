"""Keyed windows over metric VECTORS: per (key, window) sum or average of D-float vectors.

The reference's ``ComputeCpuAvg`` (chapter2/src/main/java/me/zjy/ComputeCpuAvg.java:27-59:
``keyBy(host).timeWindow(1 min).aggregate(avg)``) averages one usage value per event; a real
host reports one value per core (the README's ``cpuN`` field, chapter1/README.md:15-19), so the
engine generalises the accumulator to a D-vector: ``aggregate(VectorAvgAggregate(field))`` keeps
one f32 vector per (key, pane) and fires the per-key average vector per window — BASELINE.json's
"batched metric-vector reduces" that belong on the matrix cores.

Everything except the accumulator is the scalar operator (``KeyedWindowOperator``): the same
keyBy partition (records carry the event's row as their value), watermark valve, pane ring,
firing schedule, lateness re-firing and purge. The aggregation kernel (csrc/vector_hip.hip)
counting-sorts each sub-table's records by (pane, slot) in LDS and reduces every 32-record tile
as one-hot x vectors on ``v_mfma_f32_32x32x16_bf16`` (3-term bf16 split = exact f32 inputs).
With G > 1 the vectors travel next to their records in the all-to-all (gather into the send
layout, then positional reads on the receiver).
"""
from __future__ import annotations

import numpy as np
import torch

from ..ops import kernels as K
from ..ops import vector as V
from .window_operator import FireResult, KeyedWindowOperator

I64_MIN = K.I64_MIN


class VectorWindowOperator(KeyedWindowOperator):
    """Per-rank keyed tumbling/sliding window over D-float metric vectors (GPU or C++ twin)."""

    def __init__(self, *, dim: int, avg: bool = True, threshold: float | None = None,
                 mfma: bool = True, cap_log2: int | None = None, **kw):
        V.check_dim(dim)
        for k in ("agg", "map_prog", "filter_prog", "combine", "dense_keys", "spill"):
            if k in kw:
                raise TypeError(f"VectorWindowOperator does not take {k!r}")
        self.dim = int(dim)
        self.avg = bool(avg)
        self.threshold = threshold
        self.mode = V.MODE_MFMA if mfma else V.MODE_VALU
        # Records carry the event's row index as an int32 value: compact 16-byte records on GPU.
        # Not pipelined: the vectors of a batch are gathered into the send layout during its own
        # call (the caller may reuse `vecs` right after process() returns).
        super().__init__(agg=K.AGG_SUM_I64, combine=False, cap_log2=cap_log2, pipeline=False,
                         _vector={"dim": self.dim, "avg": self.avg, "threshold": threshold,
                                  "mode": self.mode}, **kw)
        self._rows: torch.Tensor | None = None

    # ---- entry point -----------------------------------------------------------------------
    def process(self, keys: torch.Tensor, ts: torch.Tensor, vecs: torch.Tensor) -> list[FireResult]:
        n = keys.numel()
        if vecs.dim() != 2 or vecs.shape[0] != n or vecs.shape[1] != self.dim:
            raise ValueError(f"vecs must be [{n}, {self.dim}]")
        if (vecs.dtype != torch.float32 or not vecs.is_contiguous()
                or vecs.device.type != self.device.type):
            raise ValueError("vecs must be contiguous float32 on the operator's device")
        if n >= (1 << 31):
            raise ValueError("batch too large for 32-bit row indices")
        if self._rows is None or self._rows.numel() < n:
            self._rows = torch.arange(max(n, 1), dtype=torch.int64, device=self.device)
        return super().process(keys, ts, self._rows[:n], _vecs=vecs)

    def _collect(self, block: bool = True) -> list[FireResult]:
        # rows: (keys, per-key vectors [n, dim] as the values, no raw accumulator, counts)
        return [FireResult(s, e, k, v, np.zeros(len(k), dtype=np.int64), c, refire=rf, seq=sq)
                for s, e, k, v, _r, c, rf, sq in self._s.take(block)]

    # ---- introspection / checkpoint ---------------------------------------------------------
    def state_bytes(self) -> int:
        return sum(t.numel() * t.element_size() for t in (self.keys_g, self.vacc_g, self.cnt_g,
                                                          self.dirty_g))

    def _check_ckpt_meta(self, meta: dict) -> None:
        for k in ("size", "slide", "offset", "time_mode", "dim"):
            if meta[k] != getattr(self, k):
                raise ValueError(f"checkpoint {k}={meta[k]!r} does not match operator "
                                 f"{getattr(self, k)!r}")

    _state_tensors = ("keys_g", "vacc_g", "cnt_g", "dirty_g")

    def snapshot_state(self):
        """Live (key, pane) vectors grouped by key group; the vector column is stored as one
        fixed-width binary field per row (dtype V<4*dim>)."""
        from .checkpoint import OperatorSnapshot

        D = self.dim
        if "_frozen_book" not in self.__dict__:
            self._sync_state()
        live = torch.nonzero(self.keys_g != -1).flatten()
        vdt = np.dtype((np.void, 4 * D))
        cols = {"key": np.zeros(0, np.int64), "pane": np.zeros(0, np.int64),
                "vec": np.zeros(0, vdt), "cnt": np.zeros(0, np.int32),
                "dirty": np.zeros(0, np.uint8)}
        kg = np.zeros(0, np.int32)
        if self.min_live_pane is not None and live.numel():
            panes = torch.arange(self.min_live_pane, self.max_seen_pane + 1, device=self.device)
            idx = ((panes & (self.ring - 1)) * self.nslots)[:, None] + live[None, :]
            cnt = self.cnt_g[idx]
            sel = cnt > 0
            flat = idx[sel]
            keys = self.keys_g[live][None, :].expand_as(idx)[sel].contiguous()
            kg = K.keygroups(keys, max_parallelism=self.max_parallelism, hash_mode=self.hash_mode,
                             jhash=self.jhash).cpu().numpy()
            vec = self.vacc_g.view(-1, D)[flat].cpu().numpy()
            cols = {"key": keys.cpu().numpy(),
                    "pane": panes[:, None].expand_as(idx)[sel].cpu().numpy(),
                    "vec": np.ascontiguousarray(vec).view(vdt).reshape(-1),
                    "cnt": cnt[sel].cpu().numpy(),
                    "dirty": self.dirty_g[flat].cpu().numpy()}
        book = self._book()
        meta = {"kind": "vector_window", "size": self.size, "slide": self.slide,
                "offset": self.offset, "lateness": self.lateness, "dim": self.dim,
                "avg": self.avg, "time_mode": self.time_mode, "wm": book["wm"],
                "next_fire_start": book["next_fire_start"], "min_live_pane": book["min_live_pane"],
                "max_seen_pane": book["max_seen_pane"], "metrics": book["metrics"]}
        return OperatorSnapshot(kg, cols, meta)

    def restore_state(self, rows: dict, meta: dict) -> None:
        self._check_ckpt_meta(meta)
        self._restore_book(meta)
        dev, D = self.device, self.dim
        if not len(rows["key"]):
            return
        keys = torch.from_numpy(np.ascontiguousarray(rows["key"])).to(dev)
        uniq, inv = torch.unique(keys, return_inverse=True)
        slots_u = K.table_insert(uniq.contiguous(), self.keys_g, nsub_log2=self.nsub_log2,
                                 cap_log2=self.cap_log2)
        if bool((slots_u < 0).any()):
            raise RuntimeError("restore: keyed state does not fit the table (raise max_keys)")
        slot = slots_u[inv]
        pane = torch.from_numpy(np.ascontiguousarray(rows["pane"])).to(dev)
        idx = (pane & (self.ring - 1)) * self.nslots + slot
        vec = np.ascontiguousarray(rows["vec"]).view(np.float32).reshape(-1, D)
        self.vacc_g.view(-1, D)[idx] = torch.from_numpy(vec).to(dev)
        self.cnt_g[idx] = torch.from_numpy(np.ascontiguousarray(rows["cnt"])).to(dev)
        self.dirty_g[idx] = torch.from_numpy(np.ascontiguousarray(rows["dirty"])).to(dev)
        self.occ.copy_(torch.bincount(slots_u >> self.cap_log2, minlength=self.nsub)
                       .to(torch.int32))


_ = I64_MIN
