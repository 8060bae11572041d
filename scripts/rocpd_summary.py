#!/usr/bin/env python3
"""Summarise a rocprofv3 rocpd database: per-kernel totals (and per-step averages).

  python scripts/rocpd_summary.py gpurun_out/prof_x [--steps N] [--timeline K]
"""
import argparse
import glob
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--steps", type=int, default=0, help="divide totals by this many steps")
    ap.add_argument("--timeline", type=int, default=0, help="print the last K dispatches")
    ap.add_argument("--width", type=int, default=70)
    a = ap.parse_args()
    db = sorted(glob.glob(f"{a.dir}/**/*.db", recursive=True))[0]
    c = sqlite3.connect(db)
    rows = list(c.execute("select name, count(*), sum(duration), avg(duration) from kernels "
                          "group by name order by sum(duration) desc"))
    tot = sum(r[2] for r in rows)
    print(f"| kernel | calls | total us | avg us | % |" + (" us/step |" if a.steps else ""))
    print("|---|---|---|---|---|" + ("---|" if a.steps else ""))
    for n, cnt, s, avg in rows:
        line = f"| `{n[:a.width]}` | {cnt} | {s/1e3:.1f} | {avg/1e3:.1f} | {100*s/tot:.1f} |"
        if a.steps:
            line += f" {s/1e3/a.steps:.1f} |"
        print(line)
    print(f"\ntotal kernel time {tot/1e3:.1f} us")
    if a.timeline:
        ks = list(c.execute("select name, start, end, stream_id from kernels order by start"))
        ks = ks[-a.timeline:]
        t0 = ks[0][1]
        for n, s, e, st in ks:
            print(f"{(s-t0)/1e3:9.1f} {(e-s)/1e3:8.1f} st{st} {n[:a.width]}")


if __name__ == "__main__":
    main()
