#!/usr/bin/env python3
"""The bench's DQN setup and settling, then `reps` timed windows of `steps` steps, each
bracketed by torch.cuda._sleep marker kernels (spin_kernel) for a rocprofv3 kernel trace:
  rocprofv3 --kernel-trace --output-format csv -d gpurun_out/wt -- python3 tools/window_trace.py
then tools/window_gaps.py <kernel_trace.csv> prints each window's GPU idle time and the
first steps' timeline.  Usage: tools/window_trace.py [steps] [reps]"""
import gc
import os
import sys
import time
from types import SimpleNamespace

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    dev = torch.device("cuda", 0)
    args = SimpleNamespace(batch=512, replay_size=1_000_000, num_actions=18, prefetch=4,
                           cpu_baseline_seconds=0.0)
    step = bench.setup_dqn(args, 1, 0, dev)[0]
    gc.collect()
    for _ in range(5):
        step()
    torch.cuda.synchronize()
    t = time.perf_counter()
    while time.perf_counter() - t < 0.5:
        step()
    torch.cuda.synchronize()
    for r in range(reps):
        gc.disable()
        torch.cuda._sleep(100)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(steps):
            step()
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        torch.cuda._sleep(100)
        torch.cuda.synchronize()
        gc.enable()
        print(f"window {r}: {1e3 * wall / steps:.4f} ms/step", flush=True)
        for _ in range(30):
            step()
        torch.cuda.synchronize()


if __name__ == "__main__":
    main()
