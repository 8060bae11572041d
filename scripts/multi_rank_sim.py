#!/usr/bin/env python3
"""Per-rank kernel cost of the G-GPU window path, measured on ONE GPU (the 8-GPU node is the
driver's): rank 0's partition into G x nsub buckets (Flink key groups -> ranks), the sender-side
combiner and the resulting all-to-all volume, for G in {1, 2, 4, 8}, at the headline shape
(16.7M events per GPU per step, 1M keys, 1-min tumbling window). Prints one JSON line per G.
"""
import json
import math
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mxstream.ops import kernels as K  # noqa: E402
from mxstream.runtime.geometry import state_geometry  # noqa: E402


def timeit(fn, rounds=8):
    ts = []
    for _ in range(rounds):
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    return statistics.median(ts)


def main():
    dev = torch.device("cuda", 0)
    n, nkeys = 1 << 24, 1_000_000
    keys = torch.empty(n, dtype=torch.int64, device=dev)
    ts = torch.empty_like(keys)
    vals = torch.empty_like(keys)
    K.gen_events(keys, ts, vals, seed=1, stream_id=0, idx0=0, nkeys=nkeys, ts_base=60_000,
                 ts_span=5000, disorder=2000, val_lo=0, val_span=20000)
    for world in (1, 2, 4, 8):
        nsub, cap_log2 = state_geometry(nkeys, world)
        nsub_log2 = nsub.bit_length() - 1
        nb = world << nsub_log2
        per = n / nb
        bcap = (int(per * 1.5 + 6 * math.sqrt(per) + 64) + 8 * 256 + 7) & ~7
        kg = torch.tensor([(k * world) // 128 for k in range(128)], dtype=torch.int32, device=dev)
        cursor = torch.zeros(nb, dtype=torch.int32, device=dev)
        send = torch.empty(nb * bcap * 3, dtype=torch.int64, device=dev)
        stats = K.new_stats(dev)
        plan = K.PartitionPlan(max_parallelism=128, nsub_log2=nsub_log2, nranks=world,
                               window_mode=1, drop_late=1, hash_mode=0, bucket_cap=bcap,
                               late_ts=-(1 << 62), tbase=0, pane=60_000, rec_words=2)

        def part():
            K.step_begin(cursor, stats)
            K.partition(keys, ts, vals, plan, kg, cursor, send, stats)

        t_part = timeit(part)
        res = {"world": world, "nsub": nsub, "cap_log2": cap_log2, "buckets": nb,
               "partition_us": round(t_part, 1)}
        if world > 1:
            cap = 1 << cap_log2
            ccap = cap * 2
            out = torch.empty(nb * ccap * 3, dtype=torch.int64, device=dev)
            oc = torch.zeros(nb, dtype=torch.int32, device=dev)
            flags = torch.zeros(4, dtype=torch.int32, device=dev)
            cplan = K.AggPlan(cap_log2=cap_log2, nsub=nb, ring=4, agg=K.AGG_SUM_I64, nsrc=1,
                              bucket_cap=bcap, np_step=2, pg=2, pane_base=0, p_lo=0, fired_hi=0,
                              rec_words=2)

            def comb():
                K.window_combine(send, cursor, cplan, out, ccap, oc, flags)

            res["combine_us"] = round(timeit(comb), 1)
            res["combined_records"] = int(oc.sum())
            res["a2a_bytes_per_rank"] = int(oc.sum()) * 24 * (world - 1) // world
            res["combine_overflow"] = int(flags[1])
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
