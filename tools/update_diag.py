"""Where the second step's loss error comes from (round 6): one learner step of each DQN engine
from the same parameters, compared tensor by tensor with the float64 torch restatement
(oracle/dqn_torch.py): the step-0 gradients, the Adam update (its norm error and the elements
whose update direction differs), and the float64 loss of the step-1 batch at the engine's
post-step parameters (the error the update alone makes), also with one tensor at a time
taken from the engine and the rest from float64 (which tensor's update carries it).

  python tools/update_diag.py --B 256
"""

import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.drift_diag import _batch  # noqa: E402


def loss_at(params, target, b, A=18):
    """float64 loss of batch b at (params, target) (no update)."""
    from oracle.dqn_torch import TorchDQN, huber
    t = TorchDQN(params, A, target=target, dtype=torch.float64, device="cuda")
    dev = {k: torch.as_tensor(b[k]).cuda() for k in ("o_tm1", "a_tm1", "r_t", "d_t", "o_t")}
    with torch.no_grad():
        q_tm1 = t.q(t.p, dev["o_tm1"])
        q_t_value = t.q(t.t, dev["o_t"])
        q_t_selector = t.q(t.p, dev["o_t"])
        r = torch.clamp(dev["r_t"].double(), -1.0, 1.0)
        d = dev["d_t"].double() * t.discount
        best = q_t_selector.argmax(dim=1)
        tgt = r + d * q_t_value.gather(1, best[:, None])[:, 0]
        td = tgt - q_tm1.gather(1, dev["a_tm1"].long()[:, None])[:, 0]
        iw = (1.0 / b["probabilities"]) ** t.beta
        w = torch.from_numpy((iw / iw.max()).astype(np.float32)).cuda().double()
        return float((w * huber(td)).mean())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=256)
    a = ap.parse_args()
    from acme_amd._lib import lib
    from acme_amd.native import NativeDQN
    from acme_amd.networks import DQNAtariNetwork
    from oracle.dqn_torch import TorchDQN
    net = DQNAtariNetwork(18)
    p0, t0 = net.init(11), net.init(12)
    B = a.B
    rng = np.random.default_rng(1000 + B)
    b0, b1 = _batch(rng, B, 18), _batch(rng, B, 18)
    ref = TorchDQN(p0, 18, target=t0, dtype=torch.float64, device="cuda")
    dev0 = {k: torch.as_tensor(b0[k]).cuda() for k in ("o_tm1", "a_tm1", "r_t", "d_t", "o_t")}
    q_tm1 = ref.q(ref.p, dev0["o_tm1"])
    ref.step(dev0["o_tm1"], dev0["a_tm1"], dev0["r_t"].double(), dev0["d_t"].double(),
             dev0["o_t"], b0["probabilities"])
    del q_tm1
    p1 = {k: v.detach().cpu().numpy() for k, v in ref.p.items()}
    g_ref = {k: ref.m[k].cpu().numpy() / 0.1 for k in ref.names}  # m = 0.1 g at t = 1
    L1 = loss_at(p1, p1, b1)
    print(f"B={B}: float64 step-1 loss {L1:.9f}")
    for eng, code in (("plane", 1), ("f32", 0)):
        lib().acme_set_matmul_engine(code)
        try:
            d = NativeDQN(network="nature", num_actions=18, max_batch=B, obs_dtype="uint8")
            d.set_params(p0, t0)
            d.step(*[torch.as_tensor(b0[k]).cuda().contiguous()
                     for k in ("o_tm1", "a_tm1", "r_t", "d_t", "o_t", "probabilities")])
            torch.cuda.synchronize()
            pe, ge = d.get_params("params"), d.get_params("grads")
            d.step(*[torch.as_tensor(b1[k]).cuda().contiguous()
                     for k in ("o_tm1", "a_tm1", "r_t", "d_t", "o_t", "probabilities")])
            torch.cuda.synchronize()
            Le = float(d.loss.item())
        finally:
            lib().acme_set_matmul_engine(1)
        Lp = loss_at(pe, pe, b1)
        print(f" {eng}: step-1 loss {Le:.9f} (rel err {abs(Le - L1) / abs(L1):.2e}); float64 "
              f"loss at its post-step parameters {Lp:.9f} (rel err {abs(Lp - L1) / abs(L1):.2e})",
              flush=True)
        for k in ref.names:
            r1, e1, r0 = p1[k], pe[k].reshape(p1[k].shape).astype(np.float64), p0[k]
            du_r, du_e = r1 - r0, e1 - r0
            g, gr = ge[k].reshape(g_ref[k].shape).astype(np.float64), g_ref[k]
            flips = int(np.sum(np.sign(du_r) != np.sign(du_e)))
            mix = dict(p1)
            mix[k] = e1
            Lm = loss_at(mix, mix, b1)
            print(f"  {k:40s} grad fro {np.linalg.norm(g - gr) / np.linalg.norm(gr):.2e} | update "
                  f"fro {np.linalg.norm(du_e - du_r) / np.linalg.norm(du_r):.2e} flips {flips:6d} "
                  f"of {du_r.size:8d} | loss with this tensor's update {abs(Lm - L1) / abs(L1):.2e}",
                  flush=True)


if __name__ == "__main__":
    main()
