"""Per-step fired rows of the unpipelined and the pipelined session operator (debug aid)."""
import sys
from collections import Counter

import numpy as np
import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__file__)))
from mxstream.ops import kernels as K  # noqa: E402
from mxstream.runtime.session_operator import KeyedSessionOperator  # noqa: E402

snap = len(sys.argv) > 1 and sys.argv[1] == "snap"
rng = np.random.default_rng(4)
ops = [KeyedSessionOperator(gap=100, lateness=0, agg=K.AGG_SUM_I64, device="cuda",
                            max_keys=1 << 10, batch_capacity=512, ooo_bound=50, pipeline=p)
       for p in (False, True)]
fired = [Counter(), Counter()]
for step in range(6):
    k = torch.from_numpy(rng.integers(0, 30, 500)).cuda()
    t = torch.from_numpy(np.sort(rng.integers(step * 400, step * 400 + 400, 500))).cuda()
    v = torch.from_numpy(rng.integers(0, 9, 500)).cuda()
    for i, op in enumerate(ops):
        r = op.process(k, t, v)
        rows = sorted(zip(r.keys.tolist(), r.start.tolist(), r.end.tolist(), r.raw.tolist()))
        print(f"step {step} op{i} wm {op.wm} rows {len(rows)} {rows[:6]}", flush=True)
        fired[i].update(rows)
    if step == 3 and snap:
        for op in ops:
            s = op.snapshot()
            print("snap", len(s["key"]), sorted(zip(s["key"].tolist(), s["start"].tolist(),
                                                    s["acc"].tolist()))[:8])
for i, op in enumerate(ops):
    r = op.finish()
    rows = sorted(zip(r.keys.tolist(), r.start.tolist(), r.end.tolist(), r.raw.tolist()))
    print(f"finish op{i} rows {len(rows)}", flush=True)
    fired[i].update(rows)
print("only unpipelined", sorted((fired[0] - fired[1]).items())[:20])
print("only pipelined", sorted((fired[1] - fired[0]).items())[:20])
