"""Where a synchronous window checkpoint's time goes at BASELINE scale (10M keys): the operator's
snapshot (device gather + D2H) and the key-group file write, timed separately; then the restore
(file read, and the rebuild of a fresh operator's tables).

  python scripts/ckpt_breakdown.py --keys 10000000 --steps 4
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time
from pathlib import Path

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from mxstream.models.bench_tumbling import TumblingBenchConfig, TumblingWindowBench  # noqa: E402
from mxstream.parallel.comm import LocalComm  # noqa: E402
from mxstream.runtime.checkpoint import read_operator_rows, write_operator_file  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--batch", type=int, default=1 << 24)
    ap.add_argument("--keys", type=int, default=10_000_000)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    dev = torch.device("cuda:0" if torch.cuda.is_available() else "cpu")
    b = TumblingWindowBench(TumblingBenchConfig(batch=a.batch, keys=a.keys), LocalComm(), dev)
    for _ in range(a.steps):
        b.step()
    sync = torch.cuda.synchronize if dev.type == "cuda" else (lambda: None)
    out = {"keys": a.keys, "device": str(dev), "snapshot_ms": [], "write_ms": [], "rows": 0,
           "bytes": 0}
    with tempfile.TemporaryDirectory() as d:
        for _ in range(a.reps):
            sync()
            t0 = time.perf_counter()
            snap = b.op.snapshot_state()
            t1 = time.perf_counter()
            write_operator_file(Path(d), "window", 0, snap, b.op.max_parallelism)
            t2 = time.perf_counter()
            out["snapshot_ms"].append(round((t1 - t0) * 1e3, 2))
            out["write_ms"].append(round((t2 - t1) * 1e3, 2))
            out["rows"] = int(len(snap.kg))
            out["bytes"] = int(sum(v.nbytes for v in snap.columns.values()))
        fresh = TumblingWindowBench(TumblingBenchConfig(batch=a.batch, keys=a.keys), LocalComm(),
                                    dev)
        out["read_ms"], out["restore_ms"] = [], []
        for _ in range(a.reps):
            t0 = time.perf_counter()
            rows = read_operator_rows(Path(d), ["window-0.kg"], 0, b.op.max_parallelism - 1)
            t1 = time.perf_counter()
            fresh.op.restore_state(rows, snap.meta)
            sync()
            t2 = time.perf_counter()
            out["read_ms"].append(round((t1 - t0) * 1e3, 2))
            out["restore_ms"].append(round((t2 - t1) * 1e3, 2))
    print(json.dumps(out))
    return 0


if __name__ == "__main__":
    sys.exit(main())
