"""Fill and drain of a timed window of DQN steps (bench.py's configs[1] path): after a
synchronize, K steps are issued and the GPU drained again, as bench.py times them; the wall
time T(K) = fill + K * step fits a line whose intercept is what a short window pays once.
Also the host time of the window's first step() call (the GPU idles until its first
kernel is issued) and of the later calls.  Run under gpurun: python3 tools/window_fill.py"""
import os
import sys
import time

import numpy as np
import torch

MODE = sys.argv[1] if len(sys.argv) > 1 else "window"
sys.argv = [sys.argv[0]]
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    args = bench.parse()
    dev = torch.device("cuda", 0)
    step, B, meta, loss_fn, _ = bench.setup_dqn(args, 1, 0, dev)
    for _ in range(30):
        step()
    torch.cuda.synchronize()
    rows = []
    for rep in range(4):
        for K in (1, 2, 5, 20, 50):
            torch.cuda.synchronize()
            host = []
            t0 = time.perf_counter()
            for _ in range(K):
                a = time.perf_counter()
                step()
                host.append(time.perf_counter() - a)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            rows.append((K, t1 - t0, host[0], np.mean(host[1:]) if K > 1 else float("nan")))
            print(f"rep {rep} K {K:3d}: window {1e6 * (t1 - t0):8.1f} us  "
                  f"({1e6 * (t1 - t0) / K:6.1f} per step)  first call {1e6 * host[0]:6.1f} us  "
                  f"later calls {1e6 * rows[-1][3]:6.1f} us", flush=True)
    K = np.array([r[0] for r in rows], float)
    T = np.array([r[1] for r in rows], float)
    b, a = np.polyfit(K, T, 1)
    print(f"fit: T(K) = {1e6 * a:.1f} us + K x {1e6 * b:.1f} us")


if __name__ == "__main__" and MODE == "window":
    main()


def breakdown():
    """Host time of the parts of DQNLearner.step() on the first call after a synchronize
    and on later calls: python3 tools/window_fill.py breakdown"""
    args = bench.parse()
    dev = torch.device("cuda", 0)
    step, B, meta, loss_fn, _ = bench.setup_dqn(args, 1, 0, dev)
    learner = step.__self__
    for _ in range(30):
        step()
    torch.cuda.synchronize()
    acc = {}

    def timed(name, fn):
        def w(*a, **k):
            t = time.perf_counter()
            r = fn(*a, **k)
            acc.setdefault(name, []).append(time.perf_counter() - t)
            return r
        return w

    learner._check_guard = timed("check_guard", learner._check_guard)
    learner._issue = timed("issue", learner._issue)
    it = learner._iterator
    nxt = it.__next__
    learner._iterator = type("It", (), {"__next__": lambda self: timed("next", nxt)(),
                                        "__getattr__": lambda self, n: getattr(it, n)})()
    for rep in range(5):
        torch.cuda.synchronize()
        acc.clear()
        t0 = time.perf_counter()
        for _ in range(5):
            step()
        tot = time.perf_counter() - t0
        torch.cuda.synchronize()
        print(f"rep {rep}: " + ", ".join(
            f"{k} first {1e6 * v[0]:.1f} later {1e6 * np.mean(v[1:]):.1f} us" for k, v in acc.items()),
            flush=True)


if __name__ == "__main__" and MODE == "breakdown":
    breakdown()
