"""Checkpoint stall at headline scale (BASELINE config 3: 1M keys, 16M events/step, 1 GPU).

Runs the tumbling-window bench; at step `--at` takes a synchronous checkpoint, and at step
`--at + 4` an asynchronous one (completed at the last step). Prints one JSON line with the plain
step time, the step time of the step that took each checkpoint, the async freeze time and the
async checkpoint's end-to-end time.

  python scripts/ckpt_bench.py --steps 12 --at 3 --dir /tmp/mxs_ckpt
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from mxstream.models.bench_tumbling import TumblingBenchConfig, TumblingWindowBench  # noqa: E402
from mxstream.parallel.comm import LocalComm  # noqa: E402
from mxstream.runtime.checkpoint import CheckpointCoordinator, CheckpointStorage  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=12)
    ap.add_argument("--at", type=int, default=3)
    ap.add_argument("--dir", default="/tmp/mxs_ckpt")
    ap.add_argument("--batch", type=int, default=1 << 24)
    ap.add_argument("--keys", type=int, default=1_000_000, help="key space (10M: BASELINE scale)")
    a = ap.parse_args()
    dev = torch.device("cuda:0" if torch.cuda.is_available() else "cpu")
    shutil.rmtree(a.dir, ignore_errors=True)
    b = TumblingWindowBench(TumblingBenchConfig(batch=a.batch, keys=a.keys), LocalComm(), dev)
    coord = CheckpointCoordinator(CheckpointStorage(a.dir, job_id="e" * 32), {"window": b.op})
    times, marks = [], {}
    for s in range(a.steps):
        torch.cuda.synchronize() if dev.type == "cuda" else None
        t0 = time.perf_counter()
        b.step()
        if s == a.at:
            coord.trigger(s)
            marks["sync"] = s
        if s == a.at + 4:
            coord.trigger_async(s)
            marks["async"] = s
        if s == a.steps - 1:
            coord.complete_pending()
            marks["complete"] = s
        torch.cuda.synchronize() if dev.type == "cuda" else None
        times.append((time.perf_counter() - t0) * 1e3)
    special = set(marks.values())
    plain = [t for i, t in enumerate(times) if i >= 1 and i not in special]
    sync_st = next(x for x in coord.stats if x["type"] == "checkpoint")
    async_st = next(x for x in coord.stats if x["type"] == "checkpoint-async")
    print(json.dumps({
        "plain_step_ms": round(statistics.median(plain), 3),
        "sync_ckpt_step_ms": round(times[marks["sync"]], 3),
        "async_trigger_step_ms": round(times[marks["async"]], 3),
        "async_complete_step_ms": round(times[marks["complete"]], 3),
        "steps_between_ms": [round(t, 3) for t in times[marks["async"] + 1:marks["complete"]]],
        "sync_ckpt_ms": round(sync_st["ms"], 3), "async_freeze_ms": round(async_st["sync_ms"], 3),
        "async_end_to_end_ms": round(async_st["ms"], 3),
        "async_export_ms": round(async_st["export_ms"], 3), "bytes": sync_st["bytes"],
        "keys": a.keys, "device": str(dev)}))
    shutil.rmtree(a.dir, ignore_errors=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
