"""Throughput of the text file reader alone (csrc/text_ring.h: pread into pinned slots + line
count), without parsing: the ceiling it puts on the file-replay configs (7, 9).

    python scripts/ring_read_bench.py [--mb 768] [--chunk-mb 48] [--threads 16]
"""
import argparse
import json
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
    ap.add_argument("--threads", type=int, nargs="+", default=[4, 8, 16])
    ap.add_argument("--pageable", action="store_true", help="read into pageable slots")
    ap.add_argument("--registered", action="store_true",
                    help="read into page-locked pageable slots (hipHostRegister)")
    a = ap.parse_args()
    line = b"2019-08-28T10:00:00 www.channel0001.com 12345678\n"
    n = (a.mb << 20) // len(line)
    fd, path = tempfile.mkstemp(suffix=".txt")
    with os.fdopen(fd, "wb") as f:
        f.write(line * n)
    size = os.path.getsize(path)
    chunk = a.chunk_mb << 20
    pin = torch.cuda.is_available() and not a.pageable
    if a.registered:
        from mxstream.runtime.sources import _registered_slot

        slots = [_registered_slot(chunk) for _ in range(4)]
        pin = "registered"
    else:
        slots = [torch.empty(chunk, dtype=torch.uint8, pin_memory=pin) for _ in range(4)]
    try:
        for th in a.threads:
            for rep in range(2):  # the first pass also warms the page cache
                ring = load().TextFileRing(path, 0, size, [(t.data_ptr(), t.numel()) for t in slots],
                                           chunk, th)
                t0 = time.perf_counter()
                ring.start()
                got = lines = 0
                while True:
                    slot, nbytes, nl, end, eof, _ = ring.next(1000)
                    if slot < 0:
                        if eof:
                            break
                        continue
                    got += nbytes
                    lines += nl
                    ring.release(slot)
                dt = time.perf_counter() - t0
                ring.close()
            print(json.dumps({"threads": th, "pinned": pin, "bytes": got, "lines": lines, "seconds": dt,
                              "gb_per_s": got / dt / 1e9, "lines_per_s": lines / dt}), flush=True)
    finally:
        os.unlink(path)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
