#!/usr/bin/env python3
"""insert_bench's prologue piece by piece, the learner's step time after each piece."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    from acme_amd import dm_env, replay as rp
    from acme_amd.adders import reverb as adders
    sys.argv = ["bench.py", "--workload", "insert", "--steps", "300", "--warmup", "30"]
    args = bench.parse()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    step, B, meta, _, _ = bench.setup_dqn(args, 1, 0, dev)
    table = meta["_table"]
    nat = table.native

    def timed(tag, n=300):
        for _ in range(30):
            step()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(n):
            step()
        torch.cuda.synchronize(dev)
        print(f"{tag}: {1e3 * (time.perf_counter() - t0) / n:.4f} ms/step", flush=True)

    timed("after setup")
    rng = np.random.default_rng(0)
    pool = 512
    obs = rng.integers(0, 256, (pool, 84, 84, 4), dtype=np.uint8)
    timed("after obs pool")
    acts = [np.int32(i % 18) for i in range(pool)]
    steps_ts = [dm_env.transition(np.float32(0.5), obs[i], np.float32(0.99)) for i in range(pool)]
    adder = adders.NStepTransitionAdder(rp.Client(rp.Server([table])), n_step=5, discount=0.99)
    adder.add_first(dm_env.restart(obs[0]))
    timed("after adder")
    rows = [obs.reshape(pool, -1), np.arange(pool, dtype=np.int32).view(np.uint8).reshape(pool, 4),
            np.full(pool, 0.5, np.float32).view(np.uint8).reshape(pool, 4),
            np.full(pool, 0.99 ** 4, np.float32).view(np.uint8).reshape(pool, 4),
            np.roll(obs.reshape(pool, -1), -5, axis=0)]
    chunk = min(nat.stage_capacity(), pool)
    timed(f"after rows + stage_capacity ({chunk})")
    for t in range(64):
        adder.add(acts[t], steps_ts[t])
    timed("after 64 adds")
    bufs = nat.stage(chunk)
    for b, src in zip(bufs, rows):
        np.copyto(b, src[:chunk])
    nat.commit(chunk, None)
    nat.sync_inserts()
    timed("after one chunk commit")


if __name__ == "__main__":
    main()
