#!/usr/bin/env python3
"""Per-step phase times of R2D2's one-launch LSTM kernels (workgroup 0, wall_clock64 at
100 MHz; ACME_V_RGTRACE=1): the bench shape B = 32, T = 121, burn-in 40, H = 512 on the flat
torso (the LSTM kernels do not depend on the torso).  Prints the median of each phase in us:
forward wait (h_{t-1} hand-off), mat-vec (+ the slice reduction barrier), cell, loop rest;
BPTT the same phases."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from acme_amd._lib import lib  # noqa: E402
from acme_amd.native import NativeR2D2  # noqa: E402


def main():
    B, T, BI, H = 32, 121, 40, 512
    lib().acme_tune_set(b"RGTRACE", 1)
    n = NativeR2D2(num_actions=18, max_batch=B, max_sequence_length=T, burn_in_length=BI,
                   torso="flat", obs_dim=64, lstm_size=H, head_size=512, n_step=5)
    lib().acme_tune_set(b"RGTRACE", 0)
    rng = np.random.default_rng(0)
    shapes = {k: v.shape for k, v in n.views(n.params).items()}
    p = {k: (rng.standard_normal(s) / np.sqrt(s[0] if len(s) > 1 else 1)).astype(np.float32)
         for k, s in shapes.items()}
    n.set_params(p, p)
    dev = torch.device("cuda", 0)
    obs = torch.randn(B, T, 64, device=dev)
    pa = torch.randint(0, 18, (B, T), dtype=torch.int32, device=dev)
    pr = torch.randn(B, T, device=dev)
    st = torch.zeros(B, T, 2, H, device=dev)
    probs = torch.full((B,), 1.0 / B, dtype=torch.float64, device=dev)
    disc = torch.ones(B, T, device=dev)
    for _ in range(3):
        n.step(obs, pa, pr, pa, pr, disc, probs, st[:, 0, 0], st[:, 0, 1])
    torch.cuda.synchronize()
    tr = n.debug_buffer("lstm_trace").view(np.uint64).astype(np.int64).reshape(2, 256, 4)
    for name, rows in (("forward", range(0, T)), ("bptt", range(T - 1, BI - 1, -1))):
        x = tr[0 if name == "forward" else 1]
        rows = list(rows)
        wait = [x[t, 1] - x[t, 0] for t in rows]
        mv = [x[t, 2] - x[t, 1] for t in rows]
        cell = [x[t, 3] - x[t, 2] for t in rows]
        nxt = [x[rows[i + 1], 0] - x[rows[i], 3] for i in range(len(rows) - 1)]
        tot = (x[rows[-1], 3] - x[rows[0], 0]) / len(rows)
        med = lambda v: float(np.median(v)) / 100.0  # noqa: E731  (100 MHz ticks -> us)
        print(f"{name}: per step {tot / 100.0:.2f} us; median wait {med(wait):.2f} mat-vec "
              f"{med(mv):.2f} cell/publish {med(cell):.2f} rest {med(nxt):.2f}")


if __name__ == "__main__":
    main()
