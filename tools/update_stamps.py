"""Phase stamps of the DQN step's fused priority write-back (replay.hip prio_update_fused_kernel,
ACME_V_STAMPS=1): the bench's DQN path (GPU table -> dataset -> DQNLearner.step() ->
update_priorities) runs some steps, then every workgroup's s_memrealtime stamps (100 MHz,
comparable across workgroups) of the last launch are summarised against the launch's first
entry: workgroup 0 runs the step's rescale (entry, done), the update workgroups their phases
(entry, keys resolved, node list, verdict, round-2 loads landed, levels, exit, LDS work
done before the verdict wait).
Run under gpurun: python3 tools/update_stamps.py [--steady]
--steady: the steps run back to back (the host ahead of the GPU, as in the bench's timed
region) and only the last launch is summarised; otherwise each step is synchronised."""
import os
import sys

import numpy as np

os.environ["ACME_V_STAMPS"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

PHASES = ("entry", "keys", "nodes", "verdict", "round2", "levels", "exit", "lds")


def main():
    import torch
    steady = "--steady" in sys.argv
    if "--abs" in sys.argv:
        os.environ["STAMPS_ABS"] = "1"
    sys.argv = [sys.argv[0], "--no-cpu-baseline"]
    import bench
    args = bench.parse()
    dev = torch.device("cuda", 0)
    step, B, meta, loss, _ = bench.setup_dqn(args, 1, 0, dev)
    learner = step.__self__
    for i in range(30):
        step()
        if steady and i < 29:
            continue
        torch.cuda.synchronize()
        st = learner.native.debug_buffer("gemm_stamps").view(np.int64).reshape(5, 4096, 8)[4]
        used = st[:257]
        if i < 25:
            continue
        t0 = used[used[:, 0] != 0, 0].min()  # every workgroup stamps its entry each launch
        rel = np.where(used >= t0, (used - t0) * 0.01, np.nan)  # us; older launches' stamps out
        print(f"step {i}: launch span {np.nanmax(rel):.2f} us")
        if "--abs" in sys.argv[1:] or os.environ.get("STAMPS_ABS"):
            last = used[used >= t0].max()
            print(f"  abs first entry {int(t0)} last stamp {int(last)} (100 MHz ticks)")
        print(f"  workgroup 0 (rescale): entry {rel[0, 0]:.2f}, done {rel[0, 1]:.2f}")
        upd = rel[1:]
        busy = ~np.isnan(upd[:, 2])
        print(f"  update workgroups with work: {busy.sum()} of {len(upd)}")
        for p, name in enumerate(PHASES):
            col = upd[busy, p] if p in (2, 3, 4, 5, 7) else upd[:, p]
            col = col[~np.isnan(col)]
            if len(col):
                print(f"  {name:8s} min {col.min():6.2f}  median {np.median(col):6.2f}  "
                      f"max {col.max():6.2f}")


if __name__ == "__main__":
    main()
