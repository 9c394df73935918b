"""Host-side cost of one DQN learner step (bench.py's configs[1] path): the Python +
launch time of learner.step() calls (no synchronisation inside the loop) against the
wall time of the same steps with the GPU drained at the end.  If the host time per call
approaches the wall time per step, the host bounds the step.  Run under gpurun."""
import sys
import time

import os

import torch

sys.argv = [sys.argv[0]]
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

args = bench.parse()
dev = torch.device("cuda", 0)
step, B, meta, loss_fn, _ = bench.setup_dqn(args, 1, 0, dev)
for _ in range(30):
    step()
torch.cuda.synchronize()
n = 300
t_host = 0.0
t0 = time.perf_counter()
for _ in range(n):
    a = time.perf_counter()
    step()
    t_host += time.perf_counter() - a
t_issue = time.perf_counter() - t0
torch.cuda.synchronize()
t_wall = time.perf_counter() - t0
print(f"host per step {1e6 * t_host / n:.1f} us, issue loop {1e6 * t_issue / n:.1f} us, "
      f"wall per step {1e6 * t_wall / n:.1f} us")
