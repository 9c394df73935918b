#!/usr/bin/env python3
"""The learner's step time in one process: setup_dqn alone, then (a second learner and table)
bench.insert_bench's own prologue and timing."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    sys.argv = ["bench.py", "--workload", "insert", "--steps", "300", "--warmup", "30"]
    args = bench.parse()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    if len(sys.argv) and os.environ.get("DIAG_FIRST", "1") == "1":
        step = bench.setup_dqn(args, 1, 0, dev)[0]
        for _ in range(30):
            step()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(300):
            step()
        torch.cuda.synchronize(dev)
        print(f"setup_dqn alone: {1e3 * (time.perf_counter() - t0) / 300:.4f} ms/step",
              file=sys.stderr, flush=True)
    bench.insert_bench(args, dev)


if __name__ == "__main__":
    main()
