"""BASELINE config 3: 1-min tumbling event-time window sum over 1M keys with a keyBy all-to-all.

The pipeline is the reference's ``BandwidthMonitorWithEventTime`` shape
(chapter3/src/main/java/me/zjy/BandwidthMonitorWithEventTime.java:30-55) at benchmark scale:

  synthetic source (device-side, per rank)  ->  BoundedOutOfOrderness watermark (2 s)
  -> keyBy(channel) [RCCL all-to-all over xGMI]  ->  timeWindow(1 min) reduce(sum bytes)
  -> map(bytes * 8.0 / 60 / 1024 / 1024)  ->  filter(Mbps < threshold)  ->  alert sink

Weak scaling: every GPU ingests `batch` events per step; the key space (1M) is global and
sharded by Flink key groups over the ranks.
"""
from __future__ import annotations

import statistics
import time
from dataclasses import dataclass

import torch

from ..ops import expr as E
from ..ops import kernels as K
from ..parallel.comm import Comm
from ..runtime.window_operator import KeyedWindowOperator


@dataclass
class TumblingBenchConfig:
    keys: int = 1_000_000
    batch: int = 1 << 24            # events per GPU per step
    window_ms: int = 60_000
    step_span_ms: int = 5_000        # event time covered by one micro-batch
    disorder_ms: int = 2_000         # bounded out-of-orderness of the source
    val_max: int = 20_000            # bytes per event ~ U[0, val_max)
    seed: int = 1234
    alert_fraction: float = 0.92     # alert when Mbps < fraction * expected Mbps
    # Step pipelining (KeyedWindowOperator): "stream" = partition of step i+1 enqueued ahead of
    # the state half of step i on one stream (hides the host's per-step sync); True = state
    # half on a second stream (hides a per-step exchange; measured slower at G = 1 with the
    # hashed tables, profiles/r2_pipeline_g1.md). None = "stream".
    pipeline: bool | str | None = None
    exchange: str = "auto"           # G > 1: "partials" (local-global) or "records"
    cap_log2: int | None = None      # sub-table size override (experiments)
    # Channel keys arrive as dictionary ids (the source interns strings, SURVEY.md F-ser), i.e.
    # dense ids < keys: directly addressed state. False: the hashed tables (arbitrary int64 keys).
    dense_keys: bool = True
    # Key ids as an int32 column (the columnar sources' dictionary ids) instead of int64: fewer
    # bytes, yet the partition measured slower on the same box (profiles/r2_partition_pairs.md).
    key32: bool = False
    # > 0: power-law skewed keys with this exponent (hot-key contention);
    # 0: uniform keys (the BASELINE config).
    zipf: float = 0.0


class TumblingWindowBench:
    def __init__(self, cfg: TumblingBenchConfig, comm: Comm, device: torch.device):
        self.cfg, self.comm, self.device = cfg, comm, device
        world = comm.world
        # Expected per-key window sum (all ranks feed every key) -> alert threshold in Mbps.
        events_per_window = cfg.batch * world * (cfg.window_ms / cfg.step_span_ms) / cfg.keys
        exp_sum = events_per_window * (cfg.val_max - 1) / 2.0
        self.threshold_mbps = cfg.alert_fraction * exp_sum * 8.0 / 60 / 1024 / 1024
        mbps = E.var(E.VAR_RESULT) * 8.0 / 60 / 1024 / 1024
        self.op = KeyedWindowOperator(
            size=cfg.window_ms, agg=K.AGG_SUM_I64, device=device, comm=comm,
            max_keys=cfg.keys, parallelism=world, batch_capacity=cfg.batch,
            ooo_bound=cfg.disorder_ms, map_prog=E.compile_expr(mbps),
            filter_prog=E.compile_expr(E.var(E.VAR_MAPPED) < self.threshold_mbps),
            pipeline="stream" if cfg.pipeline is None else cfg.pipeline,
            exchange=cfg.exchange, cap_log2=cfg.cap_log2, dense_keys=cfg.dense_keys)
        self.keys = torch.empty(cfg.batch, dtype=torch.int32 if cfg.dense_keys and cfg.key32
                                else torch.int64, device=device)
        self.ts = torch.empty(cfg.batch, dtype=torch.int64, device=device)
        self.vals = torch.empty(cfg.batch, dtype=torch.int64, device=device)
        self.step_idx = 0
        self.alerts = 0
        self.latencies_ms: list[tuple[float, int]] = []  # (latency, alerts) per firing step
        self.t0_event = 1_566_957_600_000  # 2019-08-28T10:00:00+08:00 (chapter3/README.md:286)
        self._ingest: dict[int, float] = {}  # batch seq (FireResult.seq) -> ingest wall time

    def _account(self, fired) -> int:
        """Alerts of the returned firings; each firing's latency runs from the ingest of the
        batch that triggered it (FireResult.seq) to now -- pipelined results come back one or
        more calls later, and that delay is part of the latency."""
        now = time.perf_counter()
        per_seq: dict[int, int] = {}
        for r in fired:
            per_seq[r.seq] = per_seq.get(r.seq, 0) + len(r.keys)
        for seq, n in per_seq.items():
            t = self._ingest.get(seq)
            if t is not None:
                self.latencies_ms.append(((now - t) * 1e3, n))
        n = sum(per_seq.values())
        self.alerts += n
        seq_now = self.op.metrics.steps
        for k in [k for k in self._ingest if k < seq_now - 64]:
            del self._ingest[k]
        return n

    def step(self) -> int:
        """One micro-batch. Pipelined, the windows a step fires come back from a LATER call;
        their alert latency is measured from the ingest time of the step that fired them."""
        cfg = self.cfg
        t_ingest = time.perf_counter()
        K.gen_events(self.keys, self.ts, self.vals, seed=cfg.seed, stream_id=self.comm.rank,
                     idx0=self.step_idx * cfg.batch, nkeys=cfg.keys,
                     ts_base=self.t0_event + self.step_idx * cfg.step_span_ms,
                     ts_span=cfg.step_span_ms, disorder=cfg.disorder_ms, val_lo=0,
                     val_span=cfg.val_max, zipf=cfg.zipf)
        self._ingest[self.op.metrics.steps + 1] = t_ingest
        fired = self.op.process(self.keys, self.ts, self.vals)
        self.step_idx += 1
        return self._account(fired)

    def device_warmup(self, ms: float) -> float:
        """Keep the GPU busy with the synthetic source's kernel (no operator state touched) for
        `ms` milliseconds of wall time, so clocks reach their sustained level before the
        warm-up steps; returns the time spent (ms)."""
        if self.device.type != "cuda":
            return 0.0
        cfg = self.cfg
        t0 = time.perf_counter()
        while (time.perf_counter() - t0) * 1e3 < ms:
            for _ in range(4):
                K.gen_events(self.keys, self.ts, self.vals, seed=cfg.seed + 1,
                             stream_id=self.comm.rank, idx0=0, nkeys=cfg.keys, ts_base=0,
                             ts_span=cfg.step_span_ms, disorder=cfg.disorder_ms, val_lo=0,
                             val_span=cfg.val_max, zipf=cfg.zipf)
            torch.cuda.synchronize(self.device)
        return (time.perf_counter() - t0) * 1e3

    def drain(self) -> int:
        """Run the pending state half (pipelined mode) and collect every queued firing."""
        return self._account(self.op.flush())

    def p50_latency_ms(self) -> float | None:
        return self.latency_quantile_ms(0.5)

    def latency_quantile_ms(self, q: float) -> float | None:
        """Quantile over alerts (each alert of a firing carries that firing's latency)."""
        if not self.latencies_ms:
            return None
        pts = sorted(self.latencies_ms)
        total = sum(c for _, c in pts)
        if total == 0:
            return statistics.median(l for l, _ in pts) if q == 0.5 else pts[-1][0]
        acc = 0
        for lat, c in pts:
            acc += c
            if acc >= q * total:
                return lat
        return pts[-1][0]
