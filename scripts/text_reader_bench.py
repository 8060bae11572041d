"""The device ingest's reader alone: a text file (in the page cache) streamed into HBM chunk by
chunk through csrc/text_ring.h, without parsing -- the config 7 reader ceiling per mode:

  pread           parallel pread into pinned slots, one DMA per chunk (the default until r5)
  mapped          file mapping page-locked read-only once; the reader threads count each
                  chunk's newlines from the mapping (first touch of its pages), one DMA per chunk
  mapped_seg      as mapped, the mapping page-locked segment by segment by the reader thread
  mapped_nocount  as mapped, without the host pass over the bytes (lines counted on the device)

Every mode opens a fresh ring (a fresh mapping: no page-table entries yet).

    python scripts/text_reader_bench.py [--mb 768] [--chunk-mb 48] [--modes pread,mapped]
"""
import argparse
import json
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from mxstream.ops.native import load  # noqa: E402


def run(m, mode, path, size, chunk, threads, dev_bufs, stream):
    slots = []
    t0 = time.perf_counter()
    if mode == "pread":
        slots = [torch.empty(chunk, dtype=torch.uint8, pin_memory=True) for _ in range(len(dev_bufs))]
        ring = m.TextFileRing(path, 0, size, [(t.data_ptr(), t.numel()) for t in slots], chunk,
                              threads)
    else:
        ring = m.TextFileRing.mapped(path, 0, size, len(dev_bufs), chunk, threads,
                                     mode != "mapped_nocount")
    t_open = time.perf_counter() - t0
    t_reg = 0.0
    seg = 0
    if mode == "mapped_seg":
        seg = max(64 << 20, chunk)
        ring.register_segments(seg, 8)
    elif mode != "pread":
        r0 = time.perf_counter()
        rc = ring.register_mapping(8)
        t_reg = time.perf_counter() - r0
        if rc:
            ring.close()
            return {"mode": mode, "register_error": rc}
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    ring.start()
    inflight, nbytes, lines, chunks = [], 0, 0, 0
    t_wait = 0.0
    while True:
        w0 = time.perf_counter()
        slot, nb, nl, end, eof, ptr = ring.next(5000)
        t_wait += time.perf_counter() - w0
        if slot < 0:
            if eof:
                break
            continue
        src = ptr if ptr else slots[slot].data_ptr()
        cut = nb
        if seg:
            off = ptr - ring.map_base
            cut = min(nb, (off // seg + 1) * seg - off)
        for a, b in ((0, cut), (cut, nb)):
            if b > a:
                rc = m.gpu_h2d_async(dev_bufs[slot].data_ptr() + a, src + a, b - a,
                                     stream.cuda_stream)
                if rc:
                    raise RuntimeError(f"h2d failed: {rc}")
        ev = torch.cuda.Event()
        ev.record(stream)
        inflight.append((slot, ev))
        nbytes += nb
        lines += max(nl, 0)
        chunks += 1
        while inflight and (inflight[0][1].query() or len(inflight) >= len(dev_bufs) - 1):
            s, e = inflight.pop(0)
            e.synchronize()
            ring.release(s)
    for s, e in inflight:
        e.synchronize()
        ring.release(s)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t1
    c0 = time.perf_counter()
    ring.close()
    t_close = time.perf_counter() - c0
    assert nbytes == size, (nbytes, size)
    return {"mode": mode, "gb_per_s": size / dt / 1e9, "seconds": dt, "chunks": chunks,
            "lines": lines, "open_s": t_open, "register_s": t_reg, "close_s": t_close,
            "consumer_wait_s": t_wait}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", type=int, default=768)
    ap.add_argument("--chunk-mb", type=int, default=48)
    ap.add_argument("--slots", type=int, default=8)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--modes", default="pread,mapped,mapped_seg,pread,mapped,mapped_seg")
    a = ap.parse_args()
    m = load()
    line = b"2019-08-28T10:00:00 www.channel0001.com 12345678\n"
    n = (a.mb << 20) // len(line)
    fd, path = tempfile.mkstemp(suffix=".txt")
    with os.fdopen(fd, "wb") as f:
        f.write(line * n)
    size = os.path.getsize(path)
    chunk = a.chunk_mb << 20
    dev_bufs = [torch.empty(chunk, dtype=torch.uint8, device="cuda") for _ in range(a.slots)]
    stream = torch.cuda.Stream()
    try:
        for mode in a.modes.split(","):
            print(json.dumps(run(m, mode, path, size, chunk, a.threads, dev_bufs, stream)),
                  flush=True)
    finally:
        os.unlink(path)


if __name__ == "__main__":
    main()
