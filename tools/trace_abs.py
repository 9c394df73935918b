#!/usr/bin/env python3
"""Absolute timeline of one step of a rocprofv3 kernel trace (µs from the step's first kernel),
per queue, averaged over the last N steps (steps delimited by the marker kernel).
Usage: tools/trace_abs.py <kernel_trace.csv> [steps] [marker]"""
import csv, re, sys, collections
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
mark = sys.argv[3] if len(sys.argv) > 3 else "prio_update_fused"
idx = [i for i, r in enumerate(rows) if mark in r["Kernel_Name"]]
acc = collections.OrderedDict()
for s in range(steps):
    a, b = idx[-steps - 1 + s], idx[-steps + s]
    t0 = int(rows[a]["End_Timestamp"])
    seen = collections.Counter()
    for r in rows[a + 1:b + 1]:
        n = re.sub(r"acme::|\(anonymous namespace\)::|gemm::|conv::", "", r["Kernel_Name"])[:60]
        seen[n] += 1
        k = (n, seen[n])
        st, en = (int(r["Start_Timestamp"]) - t0) / 1e3, (int(r["End_Timestamp"]) - t0) / 1e3
        q = r.get("Queue_Id", r.get("Stream_Id", "?"))
        e = acc.setdefault(k, [0.0, 0.0, q])
        e[0] += st / steps; e[1] += en / steps
for (n, c), (st, en, q) in sorted(acc.items(), key=lambda kv: kv[1][0]):
    print(f"q{q:>2} {st:8.1f} {en:8.1f} {en - st:7.1f}  {n}")
