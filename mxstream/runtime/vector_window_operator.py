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
from .window_operator import FireResult, KeyedWindowOperator, _next_pow2, to_host_arrays

I64_MIN = K.I64_MIN


class VectorWindowOperator(KeyedWindowOperator):
    """Per-rank keyed tumbling/sliding window over D-float metric vectors (GPU or C++ twin)."""

    def __init__(self, *, dim: int, avg: bool = True, threshold: float | None = None,
                 mfma: bool = True, cap_log2: int | None = None, **kw):
        V.check_dim(dim)
        for k in ("agg", "map_prog", "filter_prog", "combine"):
            if k in kw:
                raise TypeError(f"VectorWindowOperator does not take {k!r}")
        self.dim = int(dim)
        # Records carry the event's row index as an int32 value: compact 16-byte records on GPU.
        # Not pipelined: the vectors of a batch are gathered into the send layout during its own
        # call (the caller may reuse `vecs` right after process() returns).
        super().__init__(agg=K.AGG_SUM_I64, combine=False, cap_log2=cap_log2, pipeline=False, **kw)
        self.avg = bool(avg)
        self.threshold = threshold
        self.mode = V.MODE_MFMA if mfma else V.MODE_VALU
        dev = self.device
        self.acc_g = torch.zeros(1, dtype=torch.int64, device=dev)  # scalar accumulator unused
        self.vacc_g = torch.zeros(self.ring * self.nslots * self.dim, dtype=torch.float32,
                                  device=dev)
        self.out_vec = torch.empty(self.nslots * self.dim, dtype=torch.float32, device=dev)
        self._rows: torch.Tensor | None = None
        self._vec: torch.Tensor | None = None
        self.send_vec = self.recv_vec = None

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
        self._vec = vecs
        return super().process(keys, ts, self._rows[:n])

    _local_global_ok = False
    _spill_ok = False  # vector panes are exchanged per step (records mode)
    _use_dlist = False        # its own fire kernel sweeps the table
    _narrow_ok = False        # records carry a row index into the vector batch
    _dense_ok = False         # its own aggregation kernel

    # ---- hooks -----------------------------------------------------------------------------
    def _rec_words(self) -> int:
        return 2 if self.compact else 3

    def _exchange(self, rw: int) -> None:
        nb, bcap = self.nbuckets, self.bucket_cap
        need = nb * bcap * self.dim
        if self.send_vec is None or self.send_vec.numel() < need:
            self.send_vec = torch.zeros(need, dtype=torch.float32, device=self.device)
            self.recv_vec = torch.zeros(need, dtype=torch.float32, device=self.device)
        V.vec_gather(self.send, rw, self.cursor, nb, bcap, self._vec, self.send_vec[:need])
        words = nb * bcap * rw  # records of rw words: each rank's chunk is a prefix share
        self.comm.all_to_all(self.recv[:words], self.send[:words])
        self.comm.all_to_all(self.recv_counts, self.cursor)
        self.comm.all_to_all(self.recv_vec[:need], self.send_vec[:need])
        self.metrics.extra["a2a_bytes"] = self.metrics.extra.get("a2a_bytes", 0) + \
            (words * 8 + need * 4)

    def _aggregate(self, recs, counts, aplan: K.AggPlan) -> None:
        positional = int(self.world > 1)
        plan = V.VecAggPlan(cap_log2=aplan.cap_log2, nsub=aplan.nsub, ring=self.ring, dim=self.dim,
                            nsrc=aplan.nsrc, bucket_cap=aplan.bucket_cap, np_step=aplan.np_step,
                            positional=positional, rec_words=aplan.rec_words, mode=self.mode,
                            pane_base=aplan.pane_base, p_lo=aplan.p_lo, fired_hi=aplan.fired_hi)
        vec = self.recv_vec if positional else self._vec
        V.vec_window_agg(recs, counts, plan, vec, self.keys_g, self.vacc_g, self.cnt_g,
                         self.dirty_g, self.occ, self.flags)

    def _zero_pane(self, so: int, k: int = 1) -> None:
        e = so + k * self.nslots
        self.vacc_g[so * self.dim:e * self.dim].zero_()
        self.cnt_g[so:e].zero_()
        self.dirty_g[so:e].zero_()

    def _grow_ring(self, need: int) -> None:
        new_ring = _next_pow2(need)
        old, D, ns = self.ring, self.dim, self.nslots
        vacc = torch.zeros(new_ring * ns * D, dtype=torch.float32, device=self.device)
        cnt = torch.zeros(new_ring * ns, dtype=torch.int32, device=self.device)
        dirty = torch.zeros(new_ring * ns, dtype=torch.uint8, device=self.device)
        if self.min_live_pane is not None and self.max_seen_pane is not None:
            for p in range(self.min_live_pane, self.max_seen_pane + 1):
                so, sn = (p & (old - 1)) * ns, (p & (new_ring - 1)) * ns
                vacc[sn * D:(sn + ns) * D].copy_(self.vacc_g[so * D:(so + ns) * D])
                cnt[sn:sn + ns].copy_(self.cnt_g[so:so + ns])
                dirty[sn:sn + ns].copy_(self.dirty_g[so:so + ns])
        self.vacc_g, self.cnt_g, self.dirty_g, self.ring = vacc, cnt, dirty, new_ring
        self.metrics.ring_regrows += 1

    def _fire_window(self, s: int, only_dirty: bool) -> FireResult | None:
        p0 = max(self.pane_of(s), self.min_live_pane)
        p1 = min(self.pane_of(s) + self.panes_per_window - 1, self.max_seen_pane)
        if p1 < p0:
            return None
        self.out_n.zero_()
        V.vec_window_fire(self.keys_g, self.vacc_g, self.cnt_g, self.dirty_g, dim=self.dim,
                          npanes=p1 - p0 + 1, ring=self.ring, p0=p0, only_dirty=only_dirty,
                          avg=self.avg, threshold=self.threshold, out_keys=self.out_keys,
                          out_vec=self.out_vec, out_cnt=self.out_cnt, out_n=self.out_n)
        n = self._fired_count()
        self.metrics.num_fires += 1
        if n == 0:
            return None
        n = min(n, self.out_keys.numel())
        self.metrics.num_records_out += n
        keys, cnts = to_host_arrays([self.out_keys, self.out_cnt], n)
        vecs = to_host_arrays([self.out_vec], n * self.dim)[0].reshape(n, self.dim)
        return FireResult(s, s + self.size, keys.view(np.uint64), vecs,
                          np.zeros(n, dtype=np.int64), cnts, refire=only_dirty)

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
        meta = {"kind": "vector_window", "size": self.size, "slide": self.slide,
                "offset": self.offset, "lateness": self.lateness, "dim": self.dim,
                "avg": self.avg, "time_mode": self.time_mode, "wm": self.wm,
                "next_fire_start": self.next_fire_start, "min_live_pane": self.min_live_pane,
                "max_seen_pane": self.max_seen_pane,
                "metrics": {"num_records_in": self.metrics.num_records_in,
                            "num_late_records_dropped": self.metrics.num_late_records_dropped,
                            "num_records_out": self.metrics.num_records_out,
                            "num_fires": self.metrics.num_fires, "steps": self.metrics.steps}}
        return OperatorSnapshot(kg, cols, meta)

    def restore_state(self, rows: dict, meta: dict) -> None:
        self._check_ckpt_meta(meta)
        dev, D = self.device, self.dim
        self.wm = meta["wm"]
        self.metrics.current_watermark = self.wm
        self.next_fire_start = meta["next_fire_start"]
        self.min_live_pane, self.max_seen_pane = meta["min_live_pane"], meta["max_seen_pane"]
        for k, v in meta.get("metrics", {}).items():
            setattr(self.metrics, k, v)
        if self.min_live_pane is not None and self.max_seen_pane - self.min_live_pane + 1 > self.ring:
            self.ring = _next_pow2(self.max_seen_pane - self.min_live_pane + 1)
            self.vacc_g = torch.zeros(self.ring * self.nslots * D, dtype=torch.float32, device=dev)
            self.cnt_g = torch.zeros(self.ring * self.nslots, dtype=torch.int32, device=dev)
            self.dirty_g = torch.zeros(self.ring * self.nslots, dtype=torch.uint8, device=dev)
        self.keys_g.fill_(-1)
        self.vacc_g.zero_()
        self.cnt_g.zero_()
        self.dirty_g.zero_()
        self.occ.zero_()
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
