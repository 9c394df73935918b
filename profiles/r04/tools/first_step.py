#!/usr/bin/env python3
"""Why the first step of a short timed window issues slowly: the bench's DQN setup and
settling, then windows of `steps` steps started after (a) torch.cuda.synchronize() alone and
(b) a busy poll of an event on the learner's stream before it (the host thread kept running
while the GPU drains), alternating.  Prints the host time of the first steps split into the
dataset draw (next(iterator)), the native step call and the rest, and the window's wall time.
Usage: tools/first_step.py [steps] [repeats]"""
import gc
import os
import sys
import time
from types import SimpleNamespace

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


class _TimedIter:
    def __init__(self, it, rec):
        self._it, self._rec = it, rec

    def __iter__(self):
        return self

    def __next__(self):
        t = time.perf_counter()
        x = next(self._it)
        self._rec.append(("draw", time.perf_counter() - t))
        return x

    def __getattr__(self, name):
        return getattr(self._it, name)


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    dev = torch.device("cuda", 0)
    args = SimpleNamespace(batch=512, replay_size=1_000_000, num_actions=18, prefetch=4,
                           cpu_baseline_seconds=0.0)
    step = bench.setup_dqn(args, 1, 0, dev)[0]
    learner = step.__self__
    rec = []
    learner._iterator = _TimedIter(learner._iterator, rec)
    native_step = learner._native.step

    def timed_native(*a, **k):
        t = time.perf_counter()
        r = native_step(*a, **k)
        rec.append(("native", time.perf_counter() - t))
        return r

    learner._native.step = timed_native
    for _ in range(30):
        step()
    torch.cuda.synchronize()
    t = time.perf_counter()
    while time.perf_counter() - t < 0.5:
        step()
    torch.cuda.synchronize()
    gc.collect()
    for r in range(reps):
        for mode in ("sync", "spin"):
            for _ in range(5):
                step()
            if mode == "spin":
                ev = torch.cuda.Event()
                ev.record()
                while not ev.query():
                    pass
            torch.cuda.synchronize()
            gc.disable()
            rec.clear()
            host = []
            t0 = time.perf_counter()
            for i in range(steps):
                h = time.perf_counter()
                step()
                host.append(1e6 * (time.perf_counter() - h))
            torch.cuda.synchronize()
            wall = time.perf_counter() - t0
            gc.enable()
            draws = [1e6 * v for k, v in rec if k == "draw"]
            nat = [1e6 * v for k, v in rec if k == "native"]
            print(f"rep {r} {mode}: {1e3 * wall / steps:.4f} ms/step; host us first 4 "
                  + " ".join(f"{x:.0f}" for x in host[:4])
                  + " | draw " + " ".join(f"{x:.0f}" for x in draws[:4])
                  + " | native " + " ".join(f"{x:.0f}" for x in nat[:4])
                  + f" | steady host {sorted(host)[len(host) // 2]:.0f}", flush=True)


if __name__ == "__main__":
    main()
