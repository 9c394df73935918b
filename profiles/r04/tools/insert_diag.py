#!/usr/bin/env python3
"""Learner step time in the insert workload's setting: after setup, after the adder's
add_first, after a few adder.add calls, after table.flush(), after the staging ring's
creation and after one staged commit."""
import os
import sys
import time
from types import SimpleNamespace

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    from acme_amd import dm_env, replay as rp
    from acme_amd.adders import reverb as adders
    dev = torch.device("cuda", 0)
    args = SimpleNamespace(batch=512, replay_size=1_000_000, num_actions=18, prefetch=4,
                           cpu_baseline_seconds=0.0)
    step, B, meta, _, _ = bench.setup_dqn(args, 1, 0, dev)
    table = meta["_table"]

    def timed(tag, n=300):
        for _ in range(30):
            step()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(n):
            step()
        torch.cuda.synchronize(dev)
        print(f"{tag}: {1e3 * (time.perf_counter() - t0) / n:.4f} ms/step", flush=True)

    timed("fresh")
    timed("fresh again")
    obs = np.random.default_rng(0).integers(0, 256, (8, 84, 84, 4), dtype=np.uint8)
    adder = adders.NStepTransitionAdder(rp.Client(rp.Server([table])), n_step=5, discount=0.99)
    adder.add_first(dm_env.restart(obs[0]))
    timed("after add_first")
    for i in range(8):
        adder.add(np.int32(1), dm_env.transition(np.float32(0.5), obs[i], np.float32(0.99)))
    timed("after 8 adds")
    table.flush()
    timed("after flush")
    nat = table.native
    cap = nat.stage_capacity()
    timed(f"after stage_capacity ({cap})")
    rows = [obs.reshape(8, -1), np.zeros((8, 4), np.uint8), np.zeros((8, 4), np.uint8),
            np.zeros((8, 4), np.uint8), obs.reshape(8, -1)]
    bufs = nat.stage(8)
    for b, src in zip(bufs, rows):
        np.copyto(b, src)
    nat.commit(8, None)
    nat.sync_inserts()
    timed("after one staged commit")


if __name__ == "__main__":
    main()
