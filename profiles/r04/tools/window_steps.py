#!/usr/bin/env python3
"""Where a short timed window loses time: the bench's DQN setup and settling, then a
20-step window with a timing event recorded on the learner's stream after every step
(each record costs the stream ~6 us, the same for every step), printed as per-step GPU
durations; the host's issue time of each step beside them.  Usage: tools/window_steps.py
[steps] [repeats]"""
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
    for r in range(reps):
        for _ in range(5):
            step()
        torch.cuda.synchronize()
        t = time.perf_counter()
        while time.perf_counter() - t < 0.5:
            step()
        torch.cuda.synchronize()
        gc.disable()
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)]
        host = []
        t0 = time.perf_counter()
        evs[0].record()
        for i in range(steps):
            h = time.perf_counter()
            step()
            host.append(1e6 * (time.perf_counter() - h))
            evs[i + 1].record()
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        gc.enable()
        gpu = [1e3 * evs[i].elapsed_time(evs[i + 1]) for i in range(steps)]
        print(f"rep {r}: wall {1e3 * wall / steps:.4f} ms/step; first-event lag from t0 n/a")
        print("  gpu us/step:", " ".join(f"{x:.0f}" for x in gpu))
        print("  host us/step:", " ".join(f"{x:.0f}" for x in host))


if __name__ == "__main__":
    main()
