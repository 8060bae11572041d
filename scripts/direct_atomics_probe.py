"""Experiment: can global atomics from the source columns replace partition + window_agg for
dense ids on one rank? Times the probe kernel (modes: 2 atomics / 1 atomic / none) against the
operator's steady-state partition + aggregation kernels on the headline batch."""
import json
import sys

import torch

sys.path.insert(0, ".")
from mxstream.ops import kernels as K  # noqa: E402
from mxstream.ops.native import load  # noqa: E402

dev = torch.device("cuda", 0)
m = load()
n, nkeys = 1 << 24, 1_000_000
keys = torch.empty(n, dtype=torch.int64, device=dev)
ts = torch.empty_like(keys)
vals = torch.empty_like(keys)
K.gen_events(keys, ts, vals, seed=1, stream_id=0, idx0=0, nkeys=nkeys, ts_base=0, ts_span=5000,
             disorder=2000, val_lo=0, val_span=20000)
bits = 20  # 2^20 slots >= 1M ids
mul = 0x9E3779B1 | 1
ring, nslots = 4, 1 << bits
acc = torch.zeros(ring * nslots, dtype=torch.int64, device=dev)
cnt = torch.zeros(ring * nslots, dtype=torch.int32, device=dev)
sink = torch.zeros(1, dtype=torch.int64, device=dev)
st = torch.cuda.current_stream(dev).cuda_stream
res = {}
for mode in (2, 1, 0):
    for grid in (0, 2048, 8192):
        for _ in range(3):
            m.gpu_direct_agg_probe(keys.data_ptr(), ts.data_ptr(), vals.data_ptr(), n, -2000, 60000,
                                   ring, nslots, mul, bits, 0, acc.data_ptr(), cnt.data_ptr(), mode,
                                   sink.data_ptr(), grid, st)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            m.gpu_direct_agg_probe(keys.data_ptr(), ts.data_ptr(), vals.data_ptr(), n, -2000, 60000,
                                   ring, nslots, mul, bits, 0, acc.data_ptr(), cnt.data_ptr(), mode,
                                   sink.data_ptr(), grid, st)
        e1.record()
        torch.cuda.synchronize()
        res[f"mode{mode}_grid{grid}_us"] = e0.elapsed_time(e1) / 10 * 1e3
print(json.dumps(res))
