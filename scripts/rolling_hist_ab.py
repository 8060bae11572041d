"""Per-kernel timing of the sort-free rolling COUNT (config 2 shape) for the ablation given in
MXS_RH_ABLATE (csrc/rolling_hist_hip.hip): prints one JSON line with ms per step."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mxstream.ops import expr as E  # noqa: E402
from mxstream.ops import kernels as K  # noqa: E402
from mxstream.runtime.rolling_operator import KeyedRollingOperator  # noqa: E402

n, keys_n = 1 << 24, int(os.environ.get("KEYS", 10_000))
dev = torch.device("cuda", 0)
filt = E.compile_expr(E.var(E.VAR_COUNT) % 100_000 == 0) if os.environ.get("FILT", "1") == "1" \
    else E.EMPTY
op = KeyedRollingOperator(agg=K.AGG_COUNT, device=dev, max_keys=keys_n, batch_capacity=n,
                          filter_prog=filt, emit_capacity=1 << 20,
                          dense_keys=os.environ.get("DENSE", "0") == "1")
op.sort_free = os.environ.get("SORT_FREE", "1") == "1"
kt = torch.empty(n, dtype=torch.int64, device=dev)
K.gen_events(kt, torch.empty_like(kt), torch.empty_like(kt), seed=2, stream_id=0, idx0=0,
             nkeys=keys_n, ts_base=0, ts_span=1000, disorder=0, val_lo=0, val_span=100)
for _ in range(3):
    op.process(kt, kt, to_host=False)
torch.cuda.synchronize()
t0 = time.perf_counter()
steps = 20
for _ in range(steps):
    op.process(kt, kt, to_host=False)
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / steps
print(json.dumps({"ablate": os.environ.get("MXS_RH_ABLATE", "0"), "sort_free": op.sort_free,
                  "dense": op.dense, "filter": bool(filt.as_args()[0]),
                  "keys": keys_n, "nslots": op.nslots, "ms_per_step": dt * 1e3,
                  "events_per_s": n / dt}))
