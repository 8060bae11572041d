#!/usr/bin/env python3
"""In-process kernel microbenchmarks with interleaved variants (rule: A/B in one process).

Times partition / window_agg / window_fire variants with HIP events on the bench shape
(16.7M events, 1M keys) and prints median/min microseconds per variant.
"""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mxstream.ops import expr as E  # noqa: E402
from mxstream.ops import kernels as K  # noqa: E402
from mxstream.runtime.window_operator import KeyedWindowOperator  # noqa: E402


def timeit(fn, rounds):
    ts = []
    for _ in range(rounds):
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    return ts


def main():
    dev = torch.device("cuda", 0)
    n = int(os.environ.get("N", 1 << 24))
    nkeys = int(os.environ.get("KEYS", 1_000_000))
    rounds = int(os.environ.get("ROUNDS", 10))
    keys = torch.empty(n, dtype=torch.int64, device=dev)
    ts = torch.empty_like(keys)
    vals = torch.empty_like(keys)
    K.gen_events(keys, ts, vals, seed=1, stream_id=0, idx0=0, nkeys=nkeys, ts_base=0,
                 ts_span=5000, disorder=2000, val_lo=0, val_span=20000)
    kg = torch.zeros(128, dtype=torch.int32, device=dev)
    results = {}
    variants = {}
    for nsub_log2 in (9,):
        nb = 1 << nsub_log2
        bcap = (int(n / nb * 1.5) + 8 * 1024 + 7) & ~7
        cursor = torch.zeros(nb, dtype=torch.int32, device=dev)
        out = torch.empty(nb * bcap * 3, dtype=torch.int64, device=dev)
        stats = K.new_stats(dev)
        from mxstream.ops.native import load
        m = load()
        for ablate in [int(x) for x in os.environ.get("KB_ABLATE", "0,1").split(",")]:
            for var in [int(x) for x in os.environ.get("KB_VARIANTS", "0,1,4,5").split(",")]:
                plan = K.PartitionPlan(max_parallelism=128, nsub_log2=nsub_log2, nranks=1,
                                       window_mode=1, drop_late=1, hash_mode=0, bucket_cap=bcap,
                                       late_ts=-5000, tbase=-60000, pane=60000, ablate=ablate,
                                       rec_words=int(os.environ.get("KB_RECW", 3)))

                def f(plan=plan, cursor=cursor, out=out, stats=stats, var=var):
                    K.step_begin(cursor, stats)
                    m.gpu_partition_variant(keys.data_ptr(), ts.data_ptr(), vals.data_ptr(), 0, n,
                                            plan.as_dict(), kg.data_ptr(), cursor.data_ptr(),
                                            out.data_ptr(), stats.data_ptr(),
                                            torch.cuda.current_stream().cuda_stream, var)
                variants[f"partition nb={nb} ablate={ablate} v={var}"] = f
    # fire: a populated 1M-key state
    op = KeyedWindowOperator(size=60000, agg=K.AGG_SUM_I64, device=dev, max_keys=nkeys,
                             batch_capacity=n, ooo_bound=2000,
                             map_prog=E.compile_expr(E.var(0) * 8.0 / 60 / 1024 / 1024),
                             filter_prog=E.compile_expr(E.var(6) < 0.3))
    op.process(keys, ts, vals)
    torch.cuda.synchronize()
    p0 = op.min_live_pane
    for ablate, (mp, fp) in {"full": (op.map_prog, op.filter_prog), "noexpr": (E.EMPTY, E.EMPTY),
                             "vmskip": (op.map_prog, op.filter_prog)}.items():
        def g(mp=mp, fp=fp, ab=(1 if ablate == "vmskip" else 0)):
            op.out_n.zero_()
            K.window_fire(op.keys_g, op.acc_g, op.cnt_g, op.dirty_g, agg=op.agg, npanes=1,
                          ring=op.ring, p0=p0, wstart=0, wend=60000, only_dirty=False,
                          map_prog=mp, filt_prog=fp, out_keys=op.out_keys, out_vals=op.out_vals,
                          out_raw=op.out_raw, out_cnt=op.out_cnt, out_n=op.out_n, ablate=ab)
        variants[f"fire {ablate}"] = g
    flt = os.environ.get("KB_FILTER")
    if flt:
        variants = {k: v for k, v in variants.items() if flt in k}
    for name, f in variants.items():
        f()
    torch.cuda.synchronize()
    for r in range(rounds):
        for name, f in variants.items():
            results.setdefault(name, []).extend(timeit(f, 1))
    out = {k: {"median_us": statistics.median(v), "min_us": min(v)} for k, v in results.items()}
    for k, v in out.items():
        print(f"{k:40s} median {v['median_us']:9.1f} us   min {v['min_us']:9.1f} us")
    print(json.dumps(out))


if __name__ == "__main__":
    main()
