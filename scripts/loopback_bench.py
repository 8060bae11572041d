#!/usr/bin/env python3
"""Per-rank cost of the G>1 headline step, measured with G virtual ranks on ONE MI355X.

Every virtual rank (a thread with its own LoopbackComm) runs the complete headline step of
bench.py at its own batch size -- source, Flink key-group partition into G x sub-table buckets,
sender-side combiner, the all-to-all (device-to-device copies in all_to_all_single's layout),
combined-record window aggregation, watermark valve, firing -- and the G ranks share the GPU.
The wall time of K steps divided by G is the GPU time one rank's step costs; what it leaves out
is the xGMI transfer itself (the copies here run at HBM speed) and RCCL's launch latency.

  python scripts/loopback_bench.py --world 8 --steps 10 --warmup 3 [--batch N] [--out f.json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from mxstream.models.bench_tumbling import TumblingBenchConfig, TumblingWindowBench  # noqa: E402
from mxstream.parallel.comm import run_loopback  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=1 << 24)
    ap.add_argument("--keys", type=int, default=1_000_000)
    ap.add_argument("--out", default=None)
    ap.add_argument("--no-pipeline", action="store_true")
    ap.add_argument("--exchange", default="auto", choices=["auto", "records", "partials"])
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)

    def rank_fn(comm):
        b = TumblingWindowBench(TumblingBenchConfig(keys=a.keys, batch=a.batch,
                                                    pipeline=False if a.no_pipeline else "stream",
                                                    exchange=a.exchange,
                                                    # the records exchange needs hashed keys
                                                    dense_keys=a.exchange != "records"),
                               comm, dev)
        for _ in range(a.warmup):
            b.step()
        torch.cuda.synchronize()
        comm.barrier()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            b.step()
        b.drain()
        torch.cuda.synchronize()
        comm.barrier()
        dt = time.perf_counter() - t0
        return dt, b.alerts, dict(b.op.metrics.extra), b.op.metrics.bucket_regrows

    res = run_loopback(a.world, rank_fn, device=dev)
    dt = max(r[0] for r in res)
    per_rank_ms = dt / a.steps / a.world * 1e3
    out = {
        "what": "G virtual ranks on one MI355X (LoopbackComm): per-rank step cost of the G>1 path",
        "world": a.world, "steps": a.steps, "warmup": a.warmup, "batch_per_rank": a.batch,
        "keys": a.keys, "pipeline": not a.no_pipeline, "exchange": a.exchange, "wall_s": dt, "per_rank_step_ms": per_rank_ms,
        "per_rank_events_per_s": a.batch / (per_rank_ms / 1e3),
        "alerts": sum(r[1] for r in res), "extra_rank0": res[0][2],
        "bucket_regrows": [r[3] for r in res],
    }
    line = json.dumps(out)
    print(line, flush=True)
    if a.out:
        with open(a.out, "w") as f:
            f.write(line + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
