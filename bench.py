#!/usr/bin/env python3
"""Headline benchmark (BASELINE.json): events/sec (node) + p50 alert latency, 1M-key tumbling
event-time window, keyBy all-to-all, at 1/2/4/8 MI355X.

  python bench.py --gpus N --steps K --warmup W
  python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
      --master-port P bench.py --gpus N --steps K --warmup W

Each rank = one GPU = one source partition + one shard of the keyed window state. W untimed
steps, then exactly K timed steps bracketed by barrier + device sync; the slowest rank's time is
reported. Synthetic, device-generated events (no dataset/network); the full pipeline runs inside
the timed region: source -> partition -> RCCL all-to-all -> window aggregation -> watermark
-> firing + map/filter epilogue -> alert D2H.
"""
from __future__ import annotations

import argparse
import faulthandler
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from mxstream.models.bench_tumbling import TumblingBenchConfig, TumblingWindowBench  # noqa: E402
from mxstream.parallel.comm import init_distributed  # noqa: E402

METRIC = "events/sec (node) + p50 alert latency, 1M-key tumbling window at 1/2/4/8 MI355X"


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=48)
    ap.add_argument("--warmup", type=int, default=12)
    ap.add_argument("--batch", type=int, default=1 << 24, help="events per GPU per step")
    ap.add_argument("--keys", type=int, default=1_000_000)
    ap.add_argument("--device", default="cuda")
    ap.add_argument("--cap-log2", type=int, default=None, help="sub-table size (experiments)")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="unpipelined step (host sync between the partition and the aggregation)")
    ap.add_argument("--hashed-keys", action="store_true",
                    help="hash-table state for arbitrary int64 keys instead of dense dictionary ids")
    ap.add_argument("--zipf", type=float, default=0.0,
                    help="power-law key skew exponent (0 = uniform keys, the BASELINE config)")
    ap.add_argument("--int32-keys", action="store_true",
                    help="dense key ids as an int32 column instead of int64 (experiments)")
    ap.add_argument("--trace", default=None,
                    help="write a Chrome trace of the timed steps (stage spans; roctx with MXS_ROCTX=1)")
    ap.add_argument("--step-timeout-ms", type=int, default=0,
                    help="watchdog: abort the run if one step makes no progress for this long")
    ap.add_argument("--latency-firings", type=int, default=12,
                    help="after the timed steps: run untimed steps until this many firings "
                         "for the p50/p99 alert latency (0: timed firings only)")
    ap.add_argument("--no-hashed-figure", action="store_true",
                    help="skip the untimed-in-headline hashed-key run reported next to it")
    ap.add_argument("--exchange", choices=["auto", "partials", "records"], default="auto",
                    help="G > 1 keyBy strategy of the headline: partials = local-global "
                         "aggregation (partial accumulators cross one all-to-all per fired "
                         "window), records = every step's (key, pane)-combined records cross the "
                         "all-to-all to the key's owner (hashed state); auto = partials")
    ap.add_argument("--device-warmup-ms", type=float, default=0.0,
                    help="before the warm-up steps: keep the GPU busy with the synthetic source "
                         "for this long, so its clocks are at their sustained level when the "
                         "warm-up steps start (reported in the JSON)")
    ap.add_argument("--no-records-figure", action="store_true",
                    help="G > 1: skip the per-event-exchange (records) run reported next to it")
    a = ap.parse_args()
    faulthandler.enable()  # an abort or fault prints every thread's Python stack to stderr

    if os.environ.get("MXS_SPIN") == "1" and a.device == "cuda":
        # Spin-wait host syncs (hipDeviceScheduleSpin) before torch creates the HIP context.
        from mxstream.ops.native import load as _load

        print(f"hipSetDeviceFlags(spin) -> {_load().gpu_set_spin_schedule()}", file=sys.stderr)
    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    if a.gpus > 1 and world_env != a.gpus:
        print(f"--gpus {a.gpus} needs torch.distributed.run with {a.gpus} processes", file=sys.stderr)
        return 2
    dev_kind = a.device if (a.device == "cpu" or torch.cuda.is_available()) else "cpu"
    comm = init_distributed(dev_kind)
    if dev_kind == "cuda":
        local = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(local)
        device = torch.device("cuda", local)
    else:
        device = torch.device("cpu")

    # records exchange: every event reaches its key's owner, whose table holds a key share
    # (hashed state: dense dictionary-id slots need one destination per event)
    records = a.exchange == "records" and comm.world > 1
    cfg = TumblingBenchConfig(keys=a.keys, batch=a.batch, cap_log2=a.cap_log2,
                              dense_keys=not a.hashed_keys and not records, key32=a.int32_keys,
                              zipf=a.zipf, pipeline=False if a.no_pipeline else None,
                              exchange=a.exchange)
    bench = TumblingWindowBench(cfg, comm, device)
    if a.trace:
        from mxstream.utils import trace
        from mxstream.utils.metrics import StageTimer

        trace.enable(True)
        bench.op.timer = StageTimer(f"rank{comm.rank}", device)
    wd = None
    if a.step_timeout_ms > 0:
        from mxstream.runtime.health import Watchdog

        wd = Watchdog(a.step_timeout_ms, name=f"bench-rank{comm.rank}", action="abort").start()

    def sync():
        if device.type == "cuda":
            torch.cuda.synchronize(device)

    dev_warm = bench.device_warmup(a.device_warmup_ms) if a.device_warmup_ms > 0 else 0.0
    for _ in range(a.warmup):
        bench.step()
    # The warm-up steps complete before the clock starts: the pipelined operator's pending state
    # half of the last warm-up step is applied here, so the timed region holds exactly K
    # partitions and K state halves (the last one drained below).
    bench.drain()
    sync()
    comm.barrier()
    sync()
    bench.latencies_ms.clear()
    alerts0 = bench.alerts
    step_t = [] if os.environ.get("MXS_STEP_TIMES") == "1" else None
    t0 = time.perf_counter()
    prof_steps = os.environ.get("MXS_STEP_PROFILE") == "1"
    worst = (0.0, None)
    for _ in range(a.steps):
        if prof_steps:
            import cProfile

            pr = cProfile.Profile()
            ts_ = time.perf_counter()
            pr.enable()
        bench.step()
        if prof_steps:
            pr.disable()
            if time.perf_counter() - ts_ > worst[0]:
                worst = (time.perf_counter() - ts_, pr)
        if step_t is not None:
            step_t.append(time.perf_counter())
        if wd is not None:
            wd.beat()
    # Pipelined: the last step's state half (aggregation, firing) runs inside the timed region
    # too, so K timed steps = K partitions + K state halves.
    bench.drain()
    if step_t is not None:
        step_t.append(time.perf_counter())
    sync()
    if step_t is not None:
        step_t.append(time.perf_counter())
        d = [round((b - a_) * 1e3, 3) for a_, b in zip([t0] + step_t[:-1], step_t)]
        print(f"step host ms (last two: drain, final sync): {d}", file=sys.stderr)
        if worst[1] is not None:
            import pstats

            pstats.Stats(worst[1], stream=sys.stderr).sort_stats("tottime").print_stats(25)
        m = bench.op.metrics
        print(f"ring_regrows={m.ring_regrows} bucket_regrows={m.bucket_regrows} "
              f"extra={m.extra} ring={bench.op.ring}", file=sys.stderr)
    comm.barrier()
    sync()
    dt = time.perf_counter() - t0

    # Slowest rank defines the step time; latency stats gathered from every rank.
    t = torch.tensor([dt], dtype=torch.float64, device=device)
    comm.allreduce_max_(t)
    dt = float(t.item())
    al = torch.tensor([bench.alerts - alerts0], dtype=torch.int64, device=device)
    comm.allreduce_sum_(al)
    op_metrics = bench.op.metrics
    op_info = {"local_global": bench.op.local_global, "dense": bool(bench.op.dense_bits),
               "rec_w": bench.op.rec_w}

    # ---- after the timed region (not part of `value`) ----
    # Latency phase: the timed steps cover few firings (5 s of event time per step, 1-min
    # windows: one firing per 12 steps), so the alert-latency quantiles come from further,
    # untimed steps until `--latency-firings` firings were observed.
    timed_firings = len(bench.latencies_ms)
    lat_steps = 0
    # Every rank runs the same number of extra steps (they are collective): the stop decision
    # takes the smallest firing count over the ranks.
    have = torch.zeros(1, dtype=torch.int64, device=device)
    while a.latency_firings > 0 and lat_steps < 40 * a.latency_firings:
        have.fill_(len(bench.latencies_ms))
        comm.allreduce_min_(have)
        if int(have.item()) >= a.latency_firings:
            break
        bench.step()
        lat_steps += 1
    bench.drain()
    sync()
    lat = bench.p50_latency_ms()
    lat99 = bench.latency_quantile_ms(0.99)
    lt = torch.tensor([lat if lat is not None else -1.0, lat99 if lat99 is not None else -1.0,
                       float(len(bench.latencies_ms))], dtype=torch.float64, device=device)
    comm.allreduce_max_(lt)
    # The same step on hashed keyed state (arbitrary int64 keys: open-addressing sub-tables
    # instead of the dense dictionary-id bijection), timed the same way, reported next to it.
    def side_run(xcfg) -> tuple[float, float]:
        """The same timed loop on another configuration: (node events/s, ms per step)."""
        xb = TumblingWindowBench(xcfg, comm, device)
        for _ in range(a.warmup):
            xb.step()
        xb.drain()
        sync()
        comm.barrier()
        sync()
        th = time.perf_counter()
        for _ in range(a.steps):
            xb.step()
        xb.drain()
        sync()
        comm.barrier()
        sync()
        tt = torch.tensor([time.perf_counter() - th], dtype=torch.float64, device=device)
        comm.allreduce_max_(tt)
        return a.batch * a.steps * comm.world / float(tt.item()), float(tt.item()) / a.steps * 1e3

    hashed = None
    if not a.no_hashed_figure and not a.hashed_keys and not records:
        del bench
        ev_s, ms = side_run(TumblingBenchConfig(keys=a.keys, batch=a.batch, cap_log2=a.cap_log2,
                                                dense_keys=False, zipf=a.zipf,
                                                pipeline=False if a.no_pipeline else None,
                                                exchange=a.exchange))
        hashed = {"hashed_events_per_s": ev_s, "hashed_ms_per_step": ms}
    # G > 1 and a partials headline: the per-event keyBy shuffle (BASELINE config 3's
    # "all-to-all") measured the same way, reported next to it (not the headline value).
    recfig = None
    if comm.world > 1 and not records and not a.no_records_figure:
        ev_s, ms = side_run(TumblingBenchConfig(keys=a.keys, batch=a.batch, cap_log2=a.cap_log2,
                                                dense_keys=False, zipf=a.zipf,
                                                pipeline=False if a.no_pipeline else None,
                                                exchange="records"))
        recfig = {"records_events_per_s": ev_s, "records_ms_per_step": ms}

    n = comm.world
    events = a.batch * a.steps * n
    value = events / dt
    if comm.rank == 0:
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "events/s",
            "n_gpus": n,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": dt / a.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int64",
            "data": "synthetic (device-generated metric events, "
                    + (f"zipf({a.zipf:g})" if a.zipf > 0 else "uniform")
                    + f" keys = dictionary ids of {a.keys} channels, 2 s bounded disorder)",
            # over the timed firings plus the untimed latency phase (>= --latency-firings)
            "p50_alert_latency_ms": (lt[0].item() if lt[0].item() >= 0 else None),
            "p99_alert_latency_ms": (lt[1].item() if lt[1].item() >= 0 else None),
            "firings_timed": timed_firings,
            "firings_for_latency": int(lt[2].item()),
            "alerts": int(al.item()),
            "late_dropped": op_metrics.num_late_records_dropped,
            "device_warmup_ms": round(dev_warm, 1),
            # untimed extra runs, NOT the headline: the same job on hashed keyed state, and
            # (G > 1) with the per-event records exchange instead of local-global partials
            **(hashed or {}),
            **(recfig or {}),
            "config": {
                "model": "chapter3 1-min tumbling event-time window sum (BandwidthMonitorWithEventTime shape), 1M keys",
                "global_batch": a.batch * n,
                "seq_len": cfg.window_ms,
                "parallelism": f"keyBy-a2a{n}",
                # partials: local-global aggregation (per-rank pre-aggregation over the whole key
                # space, partial accumulators cross the all-to-all when a window fires);
                # records: per-step exchange of combined (key, pane) records.
                "exchange": ("partials" if op_info["local_global"]
                             else "records" if n > 1 else "none"),
                "keyed_state": "dense" if op_info["dense"] else "hashed",
                "record_bytes": {1: 8, 2: 16, 3: 24}[op_info["rec_w"]],
                "keys": a.keys,
                "key_distribution": f"zipf({a.zipf:g})" if a.zipf > 0 else "uniform",
                "events_per_gpu_per_step": a.batch,
                "event_time_per_step_ms": cfg.step_span_ms,
                "device": str(device),
            },
        }
        print(json.dumps(out), flush=True)
    if wd is not None:
        wd.stop()
    if a.trace and "bench" in locals():
        from mxstream.utils import trace

        if bench.op.timer is not None:
            bench.op.timer.flush()
        path = a.trace if comm.world == 1 else f"{a.trace}.rank{comm.rank}"
        trace.dump(path, comm.rank)
    from mxstream.parallel.comm import shutdown_distributed

    shutdown_distributed(comm)
    return 0


if __name__ == "__main__":
    sys.exit(main())
