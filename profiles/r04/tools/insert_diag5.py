#!/usr/bin/env python3
"""Which piece of insert_bench's prologue, done before the learner's first step, slows the
learner: PRE=obs,adder,stage (comma list) are done before the first timed window."""
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
    pre = set(filter(None, os.environ.get("PRE", "").split(",")))
    sys.argv = ["bench.py", "--workload", "insert", "--steps", "300", "--warmup", "30"]
    args = bench.parse()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    step, B, meta, _, _ = bench.setup_dqn(args, 1, 0, dev)
    table = meta["_table"]
    nat = table.native
    keep = []
    if "obs" in pre:
        keep.append(np.random.default_rng(0).integers(0, 256, (512, 84, 84, 4), dtype=np.uint8))
    if "adder" in pre:
        adder = adders.NStepTransitionAdder(rp.Client(rp.Server([table])), n_step=5,
                                            discount=0.99)
        adder.add_first(dm_env.restart(np.zeros((84, 84, 4), np.uint8)))
        keep.append(adder)
    if "stage" in pre:
        keep.append(nat.stage_capacity())
    if "pin" in pre:  # pinned host memory of the staging ring's size
        keep.append(torch.empty(4 * 33 << 20, dtype=torch.uint8, pin_memory=True))
    if "devmem" in pre:  # device memory of the staging mirrors' size
        keep.append(torch.empty(4 * 33 << 20, dtype=torch.uint8, device=dev))
    if "streams" in pre:  # two non-blocking streams created on the HIP runtime directly
        import ctypes
        hip = ctypes.CDLL("libamdhip64.so")
        for _ in range(2):
            s = ctypes.c_void_p()
            assert hip.hipStreamCreateWithFlags(ctypes.byref(s), 1) == 0
            keep.append(s)
    for _ in range(30):
        step()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(300):
        step()
    torch.cuda.synchronize(dev)
    print(f"PRE={sorted(pre)}: {1e3 * (time.perf_counter() - t0) / 300:.4f} ms/step", flush=True)


if __name__ == "__main__":
    main()
