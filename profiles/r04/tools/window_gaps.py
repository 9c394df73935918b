#!/usr/bin/env python3
"""Reads a rocprofv3 kernel_trace.csv of tools/window_trace.py and prints, per window
(between spin_kernel markers): its GPU span, the time with no kernel running, and the
first `n` kernels' start offsets / durations (us from the first kernel after the marker)."""
import csv
import sys


def main():
    path = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 60
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                         r.get("Queue_Id", r.get("Stream_Id", ""))))
    rows.sort()
    marks = [i for i, r in enumerate(rows) if "spin_kernel" in r[2]]
    for w in range(0, len(marks) - 1, 2):
        a, b = marks[w], marks[w + 1]
        ks = rows[a + 1:b]
        if not ks:
            continue
        t0, t1 = ks[0][0], max(k[1] for k in ks)
        busy, cur_s, cur_e = 0, None, None
        for s, e, _, _ in ks:
            if cur_e is None or s > cur_e:
                if cur_e is not None:
                    busy += cur_e - cur_s
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
        busy += cur_e - cur_s
        print(f"window {w // 2}: {len(ks)} kernels, span {(t1 - t0) / 1e3:.1f} us, "
              f"idle {(t1 - t0 - busy) / 1e3:.1f} us; marker->first kernel "
              f"{(t0 - rows[a][1]) / 1e3:.1f} us")
        if w == 0:
            for s, e, name, q in ks[:n]:
                print(f"  {(s - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f} q{q} {name[:90]}")


if __name__ == "__main__":
    main()
