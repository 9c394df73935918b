"""Diagnostics of the f16 plane engine (round 4): (1) the overflow-skip-recover sequence of
tests/test_step_guard_gpu.py with every gradient tensor's error and the scale records after
each step; (2) a free-running trajectory (plane / f32 engines / f64 torch) with per-step
losses.  Writes gpurun_out/diag/*.json."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import dqn_oracle as O  # noqa: E402
from tests.test_step_guard_gpu import HEAD, _batch, _dev, _masks  # noqa: E402

OUT = "gpurun_out/diag"
os.makedirs(OUT, exist_ok=True)
REC = ["X1", "X2", "X3", "T1", "T2", "T3", "Dzh", "Dz3", "Dz2", "Dz1", "Params", "Target"]


def scales(d):
    s = d.scale_state().reshape(-1, 4)
    return {REC[i]: [float(x) for x in s[i]] for i in range(len(REC))}


def overflow_seq():
    from acme_amd.native import NativeDQN
    from acme_amd.networks import DQNAtariNetwork
    net = DQNAtariNetwork(18)
    B = 64
    p0, t0 = net.init(1), net.init(2)
    for k in HEAD:
        p0[k] = p0[k] * 1e-4
        t0[k] = t0[k] * 1e-4
    d = NativeDQN(network="nature", num_actions=18, max_batch=B, obs_dtype="uint8")
    d.set_params(p0, t0)
    rng = np.random.default_rng(3)
    small = _batch(rng, B, 18, r=0.0, d=0.0)
    large = _batch(rng, B, 18, r=1.0, d=0.0)
    rep = {}
    cfg = O.DQNConfig(num_actions=18, network="nature")
    prev = (p0, t0)
    for i, b in enumerate((small, large, large, large)):
        q = torch.empty(B, 18, device="cuda")
        d.step(*_dev(b), q_tm1=q)
        torch.cuda.synchronize()
        g = d.guard_state()
        e = {"guard": g, "scales": scales(d)}
        for name in ("dzh", "dz3", "dz2", "dz1"):
            x = d.debug_buffer(name)
            e[f"{name}_max"] = float(np.nanmax(np.abs(x))) if np.isfinite(x).any() else None
            e[f"{name}_nan"] = int(np.isnan(x).sum())
        if not g["last_skipped"]:
            masks = _masks(d, prev[0], b["o_tm1"])
            out, grads = O.dqn_loss_and_grads(cfg, prev[0], prev[1], b, np.float64, masks=masks)
            gg = d.get_params("grads")
            e["loss"] = [d.loss.item(), out["loss"]]
            e["grad_err"] = {k: [float(np.abs(gg[k].reshape(v.shape) - v).max()),
                                 float(np.abs(v).max())] for k, v in grads.items()}
        rep[f"step{i + 1}"] = e
        prev = (d.get_params("params"), d.get_params("target"))
    json.dump(rep, open(f"{OUT}/overflow_seq.json", "w"), indent=1)
    print(json.dumps({k: {kk: vv for kk, vv in v.items() if kk in ("guard", "loss", "grad_err")}
                      for k, v in rep.items()}, indent=1))


def trajectory(B=64, steps=100):
    from acme_amd._lib import lib
    from acme_amd.native import NativeDQN
    from acme_amd.networks import DQNAtariNetwork
    from oracle.dqn_torch import TorchDQN
    net = DQNAtariNetwork(18)
    p0, t0 = net.init(11), net.init(12)

    def batches():
        rng = np.random.default_rng(1000 + B)
        for _ in range(steps):
            yield _batch(rng, B, 18)

    ref = TorchDQN(p0, 18, target=t0, dtype=torch.float64, device="cuda")
    ref_loss = []
    for b in batches():
        dv = {k: torch.as_tensor(b[k]).cuda() for k in ("o_tm1", "a_tm1", "r_t", "d_t", "o_t")}
        loss, _ = ref.step(dv["o_tm1"], dv["a_tm1"], dv["r_t"].double(), dv["d_t"].double(),
                           dv["o_t"], b["probabilities"])
        ref_loss.append(loss)
    res = {"ref": ref_loss}
    for name, eng in (("plane", 1), ("f32", 0)):
        lib().acme_set_matmul_engine(eng)
        try:
            d = NativeDQN(network="nature", num_actions=18, max_batch=B, obs_dtype="uint8")
            d.set_params(p0, t0)
            ls, sc = [], []
            for b in batches():
                d.step(*_dev(b))
                ls.append(d.loss.item())
                if eng == 1:
                    sc.append(scales(d))
            res[name] = ls
            if eng == 1:
                res["plane_scales"] = sc
            res[name + "_guard"] = d.guard_state()
        finally:
            lib().acme_set_matmul_engine(1)
    tag = os.environ.get("DIAG_TAG", "")
    json.dump(res, open(f"{OUT}/trajectory_{B}{tag}.json", "w"))
    r = np.array(ref_loss)
    for name in ("plane", "f32"):
        e = np.abs(np.array(res[name]) - r) / np.abs(r)
        print(name, "rel loss err per 10 steps:", [f"{x:.1e}" for x in e[::10]], "max", e.max(),
              "argmax", int(e.argmax()))


if __name__ == "__main__":
    what = sys.argv[1:] or ["overflow", "traj"]
    if "overflow" in what:
        overflow_seq()
    if "traj" in what:
        trajectory()
