"""Free-running drift of the DQN engines against the float64 trajectory, per step.

Runs the same batches as tests/test_step_guard_gpu.py::test_long_horizon_drift through the
float64 torch restatement (oracle/dqn_torch.py, cached in OUT/ref_B{B}.npz), the exact-f32
engine and the plane engine of the loaded library (ACME_LIB_PATH selects a variant build,
e.g. -DP3_FOUR_TERMS=1), and writes every step's loss and, every `--every` steps, the
parameter drift relative to how far training moved the parameters.

  python tools/drift_diag.py --out gpurun_out/drift --tag 3t --B 64 --steps 100
"""

import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _batch(rng, B, A):
    o1 = rng.integers(0, 256, (B, 84, 84, 4), dtype=np.uint8)
    o2 = rng.integers(0, 256, (B, 84, 84, 4), dtype=np.uint8)
    rr = (rng.standard_normal(B) * 1.5).astype(np.float32)
    dd = np.where(rng.random(B) < 0.2, 0.0, 0.99 ** 4).astype(np.float32)
    return dict(o_tm1=o1, a_tm1=rng.integers(0, A, B).astype(np.int32), r_t=rr, d_t=dd, o_t=o2,
                probabilities=rng.uniform(1e-6, 1e-3, B))


def _rel(a, b, base):
    num = sum(float(np.sum((a[k].astype(np.float64) - b[k]) ** 2)) for k in a)
    den = sum(float(np.sum((b[k] - base[k].astype(np.float64)) ** 2)) for k in a)
    return (num / max(den, 1e-300)) ** 0.5


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/drift")
    ap.add_argument("--tag", default="base")
    ap.add_argument("--B", type=int, default=64)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--every", type=int, default=10)
    ap.add_argument("--engines", default="plane,f32")
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    from acme_amd._lib import lib
    from acme_amd.native import NativeDQN
    from acme_amd.networks import DQNAtariNetwork
    from oracle.dqn_torch import TorchDQN
    net = DQNAtariNetwork(18)
    p0, t0 = net.init(11), net.init(12)
    B, steps = a.B, a.steps

    def batches():
        rng = np.random.default_rng(1000 + B)
        for _ in range(steps):
            yield _batch(rng, B, 18)

    marks = [i for i in range(steps) if (i + 1) % a.every == 0 or i == steps - 1]
    ref_path = os.path.join("/tmp", f"acme_drift_ref_B{B}_S{steps}.npz")  # not under gpurun_out: 100s of MB
    if not os.path.exists(ref_path):
        ref = TorchDQN(p0, 18, target=t0, dtype=torch.float64, device="cuda")
        ref_loss, snaps = [], {}
        for i, b in enumerate(batches()):
            dev = {k: torch.as_tensor(b[k]).cuda() for k in ("o_tm1", "a_tm1", "r_t", "d_t", "o_t")}
            loss, _ = ref.step(dev["o_tm1"], dev["a_tm1"], dev["r_t"].double(),
                               dev["d_t"].double(), dev["o_t"], b["probabilities"])
            ref_loss.append(loss)
            if i in marks:
                for k, v in ref.p.items():
                    snaps[f"{i}|{k}"] = v.detach().cpu().numpy()
        np.savez(ref_path, loss=np.array(ref_loss), **snaps)
        print(f"reference trajectory written ({time_ref(ref_path)})", flush=True)
    z = np.load(ref_path)
    ref_loss = z["loss"]
    names = sorted({k.split("|", 1)[1] for k in z.files if "|" in k})
    res = {"B": B, "steps": steps, "ref_loss": ref_loss.tolist(), "marks": marks}
    for eng in a.engines.split(","):
        if eng == "torch32":  # an independent float32 implementation (torch / MIOpen)
            t32 = TorchDQN(p0, 18, target=t0, dtype=torch.float32, device="cuda")
            losses, drift = [], []
            for i, b in enumerate(batches()):
                dev = {k: torch.as_tensor(b[k]).cuda() for k in ("o_tm1", "a_tm1", "r_t", "d_t", "o_t")}
                loss, _ = t32.step(dev["o_tm1"], dev["a_tm1"], dev["r_t"], dev["d_t"], dev["o_t"],
                                   b["probabilities"])
                losses.append(loss)
                if i in marks:
                    got = {k: v.detach().cpu().numpy() for k, v in t32.p.items()}
                    drift.append(_rel(got, {k: z[f"{i}|{k}"] for k in names}, p0))
            loss = np.array(losses)
            err = np.abs(loss - ref_loss) / np.abs(ref_loss)
            res[eng] = {"loss": loss.tolist(), "rel_err": err.tolist(), "drift": drift,
                        "max_rel_err": float(err.max()), "argmax": int(err.argmax())}
            print(f"{a.tag} {eng} B={B}: max loss rel err {err.max():.3e} at step {err.argmax()}; "
                  f"median {np.median(err):.3e}; drift at marks {[round(x, 4) for x in drift]}",
                  flush=True)
            continue
        code = {"plane": 1, "f32": 0}[eng]
        lib().acme_set_matmul_engine(code)
        try:
            d = NativeDQN(network="nature", num_actions=18, max_batch=B, obs_dtype="uint8")
            d.set_params(p0, t0)
            losses, drift = [], []
            for i, b in enumerate(batches()):
                d.step(*[torch.as_tensor(b[k]).cuda().contiguous()
                         for k in ("o_tm1", "a_tm1", "r_t", "d_t", "o_t", "probabilities")])
                losses.append(d.loss.clone())
                if i in marks:
                    torch.cuda.synchronize()
                    got = d.get_params("params")
                    drift.append(_rel(got, {k: z[f"{i}|{k}"] for k in names}, p0))
            torch.cuda.synchronize()
            g = d.guard_state()
        finally:
            lib().acme_set_matmul_engine(1)
        loss = np.array([x.item() for x in losses])
        err = np.abs(loss - ref_loss) / np.abs(ref_loss)
        res[eng] = {"loss": loss.tolist(), "rel_err": err.tolist(), "drift": drift,
                    "guard": g, "max_rel_err": float(err.max()),
                    "argmax": int(err.argmax())}
        print(f"{a.tag} {eng} B={B}: max loss rel err {err.max():.3e} at step {err.argmax()}; "
              f"median {np.median(err):.3e}; drift at marks {[round(x, 4) for x in drift]}; "
              f"guard {g}", flush=True)
    with open(os.path.join(a.out, f"drift_{a.tag}_B{B}.json"), "w") as f:
        json.dump(res, f)


def time_ref(p):
    return os.path.basename(p)


if __name__ == "__main__":
    main()
