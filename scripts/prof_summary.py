#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel-trace database (rocpd sqlite) into a markdown table."""
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
cur = db.cursor()
rows = cur.execute("select name, total_calls, total_duration, average, percentage from top_kernels").fetchall()
print("| kernel | calls | total us | avg us | % |")
print("|---|---|---|---|---|")
for name, calls, tot, avg, pct in rows:
    short = name.replace("(anonymous namespace)::", "")
    short = short.split("(")[0] if not short.startswith("void ") else short[5:].split("(")[0]
    if len(short) > 90:
        short = short[:87] + "..."
    print(f"| `{short}` | {calls} | {tot:.1f} | {avg:.1f} | {pct:.1f} |")
