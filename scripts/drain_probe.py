"""Where the headline's timed region spends its fixed cost (steps 20 / warm-up 5): host time
of each step, of the drain's flush and of the final device sync, printed per phase."""
import sys
import time

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__file__)))
from mxstream.models.bench_tumbling import TumblingBenchConfig, TumblingWindowBench  # noqa: E402
from mxstream.parallel.comm import LocalComm  # noqa: E402

dev = torch.device("cuda", 0)
for rep in range(3):
    b = TumblingWindowBench(TumblingBenchConfig(), LocalComm(), dev)
    for _ in range(5):
        b.step()
    b.drain()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    st = []
    for _ in range(20):
        b.step()
        st.append(time.perf_counter())
    t1 = time.perf_counter()
    b.op._s.flush(b.op._stream())
    tf = time.perf_counter()
    fl = b.op._collect()
    t2 = time.perf_counter()
    torch.cuda.synchronize()
    t3 = time.perf_counter()
    steps = [round((y - x) * 1e3, 3) for x, y in zip([t0] + st[:-1], st)]
    print(f"rep {rep}: steps {steps}\n  flush {1e3 * (t2 - t1):.3f} ms (native {1e3 * (tf - t1):.3f})"
          f"  sync {1e3 * (t3 - t2):.3f} ms"
          f"  total {1e3 * (t3 - t0):.3f} ms -> {16777216 * 20 / (t3 - t0) / 1e9:.2f} G", flush=True)
    # the same flush with the device idle first: the host cost alone
    for _ in range(3):
        b.step()
    torch.cuda.synchronize()
    ta = time.perf_counter()
    b.op._s.flush(b.op._stream())
    tb = time.perf_counter()
    print(f"  idle-device flush {1e3 * (tb - ta):.3f} ms", flush=True)
    del b
