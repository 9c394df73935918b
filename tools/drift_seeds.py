"""Free-running drift of the DQN engines against float64 over several seeds (round 6): how much
the single-seed metrics of tests/test_step_guard_gpu.py::test_long_horizon_drift vary between
seeds for each engine.  A ReLU whose pre-activation lies within the engines' rounding of zero
switches on one side and not the other, and after it the trajectories part chaotically, so one
seed's maximum loss error is a draw, not a property of the engine.

  python tools/drift_seeds.py --seeds 4 --out gpurun_out/drift_seeds
"""

import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.drift_diag import _batch, _rel  # noqa: E402

CASES = {64: 100, 256: 50, 512: 20}


def run_seed(B, steps, seed):
    from acme_amd._lib import lib
    from acme_amd.native import NativeDQN
    from acme_amd.networks import DQNAtariNetwork
    from oracle.dqn_torch import TorchDQN
    net = DQNAtariNetwork(18)
    p0, t0 = net.init(11 + 2 * seed), net.init(12 + 2 * seed)

    def batches():
        rng = np.random.default_rng(1000 + B + 7919 * seed)
        for _ in range(steps):
            yield _batch(rng, B, 18)

    ref = TorchDQN(p0, 18, target=t0, dtype=torch.float64, device="cuda")
    ref_loss = []
    for b in batches():
        dev = {k: torch.as_tensor(b[k]).cuda() for k in ("o_tm1", "a_tm1", "r_t", "d_t", "o_t")}
        loss, _ = ref.step(dev["o_tm1"], dev["a_tm1"], dev["r_t"].double(), dev["d_t"].double(),
                           dev["o_t"], b["probabilities"])
        ref_loss.append(loss)
    ref_p = {k: v.detach().cpu().numpy() for k, v in ref.p.items()}
    ref_loss = np.array(ref_loss)
    out = {}
    for eng, code in (("plane", 1), ("f32", 0)):
        lib().acme_set_matmul_engine(code)
        try:
            d = NativeDQN(network="nature", num_actions=18, max_batch=B, obs_dtype="uint8")
            d.set_params(p0, t0)
            losses = []
            for b in batches():
                d.step(*[torch.as_tensor(b[k]).cuda().contiguous()
                         for k in ("o_tm1", "a_tm1", "r_t", "d_t", "o_t", "probabilities")])
                losses.append(d.loss.clone())
            torch.cuda.synchronize()
            g = d.guard_state()
            pe = d.get_params("params")
        finally:
            lib().acme_set_matmul_engine(1)
        e = np.abs(np.array([x.item() for x in losses]) - ref_loss) / np.abs(ref_loss)
        out[eng] = dict(drift=_rel(pe, ref_p, p0), loss_max=float(e.max()),
                        loss_median=float(np.median(e)), step1=float(e[1]),
                        skipped=int(g["skipped"]))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", type=int, default=4)
    ap.add_argument("--batches", default="64,256,512")
    ap.add_argument("--out", default="gpurun_out/drift_seeds")
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    res = {}
    for B in [int(x) for x in a.batches.split(",")]:
        steps = CASES[B]
        rows = []
        for s in range(a.seeds):
            r = run_seed(B, steps, s)
            rows.append(r)
            print(f"B={B} seed {s}: " + "  ".join(
                f"{eng} drift {v['drift']:.3e} loss max {v['loss_max']:.3e} median "
                f"{v['loss_median']:.3e} step1 {v['step1']:.2e} skipped {v['skipped']}"
                for eng, v in r.items()), flush=True)
        for m in ("drift", "loss_max", "loss_median"):
            pl = np.mean([r["plane"][m] for r in rows])
            f3 = np.mean([r["f32"][m] for r in rows])
            print(f"B={B} mean over {a.seeds} seeds: {m} plane {pl:.3e} f32 {f3:.3e} "
                  f"ratio {pl / f3:.2f}", flush=True)
        res[B] = rows
    with open(os.path.join(a.out, "drift_seeds.json"), "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
