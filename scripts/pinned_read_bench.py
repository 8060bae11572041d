"""Host read speed of pinned (page-locked) vs pageable buffers after a D2H copy."""
import time

import numpy as np
import torch

n = 6 * 600_000
src = torch.arange(n, dtype=torch.int64, device="cuda")
pin = torch.empty(n, dtype=torch.int64).pin_memory()
pag = torch.empty(n, dtype=torch.int64)
for name, dst in (("pinned", pin), ("pageable", pag)):
    dst.copy_(src, non_blocking=(name == "pinned"))
    torch.cuda.synchronize()
    a = dst.numpy()
    t0 = time.perf_counter()
    for _ in range(5):
        s = int(a.sum())
    t1 = time.perf_counter()
    for _ in range(5):
        b = a.copy()
    t2 = time.perf_counter()
    t3 = time.perf_counter()
    for _ in range(5):
        dst.copy_(src, non_blocking=(name == "pinned"))
        torch.cuda.synchronize()
    t4 = time.perf_counter()
    print(f"{name}: sum {(t1 - t0) / 5 * 1e3:.2f} ms, copy {(t2 - t1) / 5 * 1e3:.2f} ms, "
          f"d2h {(t4 - t3) / 5 * 1e3:.2f} ms for {n * 8 / 1e6:.1f} MB")
