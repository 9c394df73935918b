#!/usr/bin/env python3
"""bench.main() for the insert workload with the learner's step wrapped: host time per
step call over the run, in windows of 100 calls."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

stamps = []
_setup = bench.setup_dqn


def setup(*a, **k):
    out = list(_setup(*a, **k))
    step = out[0]

    def timed_step():
        stamps.append(time.perf_counter())
        step()
    out[0] = timed_step
    return tuple(out)


bench.setup_dqn = setup
sys.argv = ["bench.py", "--workload", "insert", "--steps", "300", "--warmup", "30"]
bench.main()
for i in range(0, len(stamps) - 100, 100):
    print(f"calls {i}-{i + 100}: {1e3 * (stamps[i + 100] - stamps[i]) / 100:.4f} ms/call",
          file=sys.stderr)
