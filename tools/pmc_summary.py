#!/usr/bin/env python3
"""Mean per-dispatch PMC counters by kernel (rocprofv3 --pmc CSV output), for quick
bottleneck reading.  Usage: tools/pmc_summary.py <dir> [kernel-regex]"""
import collections
import csv
import glob
import re
import sys

d = sys.argv[1]
pat = re.compile(sys.argv[2]) if len(sys.argv) > 2 else None
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        k = row["Kernel_Name"]
        if pat and not pat.search(k):
            continue
        acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
for k, cs in sorted(acc.items(), key=lambda kv: kv[0]):
    short = re.sub(r"acme::(gemm|conv)::", "", k)[:150]
    vals = "  ".join(f"{c}={sum(v)/len(v):.4g}" for c, v in sorted(cs.items()))
    n = max(len(v) for v in cs.values())
    print(f"{short}\n    n={n} {vals}")
