"""Host-to-device bandwidth of the text sources' upload: SDMA (hipMemcpyAsync via torch) vs the
copy kernel reading the pinned buffer over PCIe (gpu_h2d_kernel), for batch-sized copies.

    python scripts/h2d_bench.py [--mb 48 192] [--reps 20]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from mxstream.ops.native import load  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", type=int, nargs="+", default=[12, 48, 192])
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--blocks", type=int, nargs="+", default=[256, 1024, 2048])
    a = ap.parse_args()
    m = load()
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    out = []
    for mb in a.mb:
        n = mb << 20
        src = torch.randint(0, 255, (n,), dtype=torch.uint8).pin_memory()
        dst = torch.empty(n, dtype=torch.uint8, device=dev)

        def timed(fn):
            fn()
            torch.cuda.synchronize()
            t = time.perf_counter()
            for _ in range(a.reps):
                fn()
            torch.cuda.synchronize()
            return (time.perf_counter() - t) / a.reps

        t_sdma = timed(lambda: dst.copy_(src, non_blocking=True))
        row = {"mb": mb, "sdma_gbs": n / t_sdma / 1e9}
        for blk in a.blocks:
            def kern():
                rc = m.gpu_h2d_kernel(dst.data_ptr(), src.data_ptr(), n, st.cuda_stream, blk)
                if rc:
                    raise RuntimeError(f"gpu_h2d_kernel: hip error {rc}")
            t_k = timed(kern)
            row[f"kernel_{blk}_gbs"] = n / t_k / 1e9
        ok = bool(torch.equal(dst.cpu(), src))
        row["kernel_copy_exact"] = ok
        out.append(row)
        print(json.dumps(row), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
