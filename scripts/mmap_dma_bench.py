"""Page cache -> HBM without a CPU copy: the text file's pages, mmapped and page-locked with
hipHostRegister (ReadOnly), go to the device by DMA. Compared against the pread reader
(csrc/text_ring.h, ~23 GB/s on the box): the config 7 reader ceiling.

    python scripts/mmap_dma_bench.py [--mb 768] [--chunk-mb 48]
"""
import argparse
import json
import mmap
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from mxstream.ops.native import load  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", type=int, default=768)
    ap.add_argument("--chunk-mb", type=int, default=48)
    a = ap.parse_args()
    m = load()
    line = b"2019-08-28T10:00:00 www.channel0001.com 12345678\n"
    n = (a.mb << 20) // len(line)
    fd, path = tempfile.mkstemp(suffix=".txt")
    with os.fdopen(fd, "wb") as f:
        f.write(line * n)
    size = os.path.getsize(path)
    with open(path, "rb") as f:  # page cache warm
        while f.read(1 << 26):
            pass
    chunk = a.chunk_mb << 20
    dev = torch.empty(chunk, dtype=torch.uint8, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    fd = os.open(path, os.O_RDONLY)
    mm = mmap.mmap(fd, size, prot=mmap.PROT_READ, flags=mmap.MAP_SHARED)
    base = np.frombuffer(mm, dtype=np.uint8).ctypes.data
    for flags, name in ((8, "readonly"), (8 | 2, "readonly_mapped")):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        t_reg = t_unreg = 0.0
        ok = True
        for off in range(0, size, chunk):
            ln = min(chunk, size - off)
            r0 = time.perf_counter()
            rc = m.gpu_host_register_flags(base + off, ln, flags)
            t_reg += time.perf_counter() - r0
            if rc:
                print(json.dumps({"mode": name, "register_error": rc}), flush=True)
                ok = False
                break
            e = m.gpu_h2d_async(dev.data_ptr(), base + off, ln, st)
            if e:
                print(json.dumps({"mode": name, "copy_error": e}), flush=True)
                ok = False
            torch.cuda.synchronize()
            u0 = time.perf_counter()
            m.gpu_host_unregister(base + off)
            t_unreg += time.perf_counter() - u0
        dt = time.perf_counter() - t0
        if ok:
            print(json.dumps({"mode": name, "bytes": size, "seconds": dt, "gb_per_s": size / dt / 1e9,
                              "register_s": t_reg, "unregister_s": t_unreg,
                              "dma_s": dt - t_reg - t_unreg}), flush=True)
    # one registration of the whole file, then back-to-back DMA chunks
    r0 = time.perf_counter()
    rc = m.gpu_host_register_flags(base, size, 8)
    t_reg = time.perf_counter() - r0
    if rc == 0:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for off in range(0, size, chunk):
            m.gpu_h2d_async(dev.data_ptr(), base + off, min(chunk, size - off), st)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        m.gpu_host_unregister(base)
        print(json.dumps({"mode": "whole_file_registered", "register_s": t_reg, "dma_s": dt,
                          "dma_gb_per_s": size / dt / 1e9}), flush=True)
    del base
    mm.close()
    os.close(fd)
    os.unlink(path)


if __name__ == "__main__":
    main()
