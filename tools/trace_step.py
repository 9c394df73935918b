#!/usr/bin/env python3
"""One learner step of a rocprofv3 kernel trace (between two launches of a marker kernel, default the priority update): per-kernel
start gap, duration and queue, plus wall / busy-union / gap totals over the last N steps.
Usage: tools/trace_step.py <kernel_trace.csv> [steps] [marker]"""
import csv
import re
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
mark = sys.argv[3] if len(sys.argv) > 3 else "prio_update_fused"
adam = [i for i, r in enumerate(rows) if mark in r["Kernel_Name"]]
a, b = adam[-steps - 1], adam[-1]
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows[a + 1:b + 1])
union, gaps, (cs, ce) = 0, 0, iv[0]
for s, e in iv[1:]:
    if s > ce:
        union += ce - cs
        gaps += s - ce
        cs, ce = s, e
    else:
        ce = max(ce, e)
union += ce - cs
wall = int(rows[b]["End_Timestamp"]) - int(rows[a]["End_Timestamp"])
print(f"per step: wall {wall / steps / 1e3:.1f} us, busy {union / steps / 1e3:.1f} us, "
      f"idle {gaps / steps / 1e3:.1f} us")
prev = int(rows[adam[-2]]["End_Timestamp"])
for r in rows[adam[-2] + 1:adam[-1] + 1]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    n = re.sub(r"acme::|\(anonymous namespace\)::|gemm::|conv::", "", r["Kernel_Name"])[:80]
    print(f"{(s - prev) / 1e3:8.2f} {(e - s) / 1e3:8.2f} q{r['Queue_Id']} {n}")
    prev = max(prev, e)
