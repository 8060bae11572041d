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
    ap.add_argument("--busy", type=int, default=0,
                    help="GPU busy/idle over the last K dispatches: union of kernel intervals, "
                         "largest idle gaps and the kernel before each")
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
    if a.busy:
        ks = list(c.execute("select name, start, end from kernels order by start"))[-a.busy:]
        t0, t1 = ks[0][1], max(e for _, _, e in ks)
        busy, cur_s, cur_e, gaps = 0, ks[0][1], ks[0][2], []
        prev = ks[0][0]
        for n, s, e in ks[1:]:
            if s > cur_e:
                busy += cur_e - cur_s
                gaps.append((s - cur_e, prev, n))
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
            prev = n
        busy += cur_e - cur_s
        span = t1 - t0
        print(f"\nspan {span/1e3:.1f} us, busy {busy/1e3:.1f} us ({100*busy/span:.1f} %), "
              f"idle {(span-busy)/1e3:.1f} us in {len(gaps)} gaps")
        agg = {}
        for g, p0, n in gaps:
            k = (p0[:40], n[:40])
            agg[k] = (agg.get(k, (0, 0))[0] + g, agg.get(k, (0, 0))[1] + 1)
        print("| idle us | gaps | after | before |\n|---|---|---|---|")
        for (p0, n), (g, cnt) in sorted(agg.items(), key=lambda x: -x[1][0])[:15]:
            print(f"| {g/1e3:.1f} | {cnt} | `{p0}` | `{n}` |")


if __name__ == "__main__":
    main()
