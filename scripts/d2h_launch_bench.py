"""Host cost of launching a counted D2H (window_operator.CountedHostRows) on the MI355X box, by
piece: event record + stream wait, the copy-kernel launch, the whole constructor. Config 5's
session eviction spent 1.2 ms per step in the constructor (profiles/r4x_cfg5.json)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from mxstream.ops.native import load  # noqa: E402
from mxstream.runtime.window_operator import CountedHostRows, PinnedSlabPool  # noqa: E402


def timed(fn, reps=50):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    dt = (time.perf_counter() - t) / reps * 1e3
    torch.cuda.synchronize()
    return dt


def main():
    dev = torch.device("cuda", 0)
    m = load()
    R = 1 << 22
    rows = torch.zeros(6, R, dtype=torch.int64, device=dev)
    ctr = torch.zeros(16, dtype=torch.int32, device=dev)
    ctr[7] = 300_000
    side = torch.cuda.Stream(dev)
    pool = PinnedSlabPool(max_slabs=2)
    out = {}

    def ev_wait():
        e = torch.cuda.Event()
        e.record(torch.cuda.current_stream(dev))
        side.wait_event(e)
    out["event_record_wait_ms"] = timed(ev_wait)
    hr = CountedHostRows(pool, [rows[j] for j in range(6)], ctr[7:8], [ctr], copy_stream=side)
    hr.wait()
    t = hr.t
    copies = [(rows[j].data_ptr(), R * 8, j * R * 8, 8) for j in range(6)]
    out["d2h_counted_launch_ms"] = timed(lambda: m.gpu_d2h_counted(t.data_ptr(), copies,
                                                                     ctr[7:8].data_ptr(),
                                                                     side.cuda_stream, 64))
    del hr

    def ctor():
        h = CountedHostRows(pool, [rows[j] for j in range(6)], ctr[7:8], [ctr], copy_stream=side)
        h.wait()
    out["counted_host_rows_incl_copy_ms"] = timed(ctor, 20)

    def ctor_nowait():
        CountedHostRows(pool, [rows[j] for j in range(6)], ctr[7:8], [ctr], copy_stream=side)
    out["counted_host_rows_launch_ms"] = timed(ctor_nowait, 20)
    out["slab_allocs"] = pool.allocs
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
