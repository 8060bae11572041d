"""Kernel table from a rocprofv3 results.db (rocpd SQLite): per kernel, dispatches and time over
the LAST `timed` steps (steps delimited by the dispatches of a once-per-step marker kernel), in
microseconds per step, plus the GPU-busy union per step.

usage: python scripts/rocpd_table.py DB --marker gen_events --timed 40 [--md out.md]
"""
import argparse
import sqlite3
from collections import defaultdict


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--marker", default="gen_events")
    ap.add_argument("--timed", type=int, default=20)
    ap.add_argument("--md", default=None)
    ap.add_argument("--first", type=int, default=None,
                    help="the timed steps start at this marker dispatch (default: the last ones)")
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, start, end from kernels order by start").fetchall()
    marks = [s for n, s, _ in rows if a.marker in n]
    if len(marks) < a.timed:
        raise SystemExit(f"only {len(marks)} marker dispatches")
    i0 = len(marks) - a.timed if a.first is None else a.first
    t0 = marks[i0]
    t_end = marks[i0 + a.timed] if i0 + a.timed < len(marks) else float("inf")
    sel = [(n, s, e) for n, s, e in rows if t0 <= s < t_end]
    t1 = max(e for _, _, e in sel)
    per = defaultdict(lambda: [0, 0])
    for n, s, e in sel:
        short = n.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "").strip()
        per[short][0] += 1
        per[short][1] += e - s
    busy, cur_s, cur_e = 0, None, None  # union of dispatch intervals
    for _, s, e in sorted((x for x in sel), key=lambda x: x[1]):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    tot = sum(v[1] for v in per.values())
    lines = [f"timed region: {a.timed} steps from marker #{i0} ({a.marker} dispatches), wall "
             f"{(t1 - t0) / 1e3 / a.timed:.1f} us/step, GPU busy (union) {busy / 1e3 / a.timed:.1f} "
             f"us/step, kernel sum {tot / 1e3 / a.timed:.1f} us/step", "",
             "| kernel | calls/step | us/step | share |", "|---|---|---|---|"]
    for n, (k, d) in sorted(per.items(), key=lambda kv: -kv[1][1])[:a.top]:
        lines.append(f"| `{n[:80]}` | {k / a.timed:.2f} | {d / 1e3 / a.timed:.1f} | {100 * d / tot:.1f}% |")
    out = "\n".join(lines)
    print(out)
    if a.md:
        open(a.md, "w").write(out + "\n")


if __name__ == "__main__":
    main()
