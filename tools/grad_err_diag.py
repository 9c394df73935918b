"""Per-tensor gradient error of the DQN engines against float64, teacher-forced.

From the same parameters (the initial ones, then those after `--warm` plane-engine steps of
tools/drift_diag.py's batch stream) both engines take one step's gradients on the next
batch; the float64 torch restatement (oracle/dqn_torch.py) gives the reference.  Prints,
per tensor, the relative Frobenius error and the fraction of elements whose error exceeds
1e-3 of their own magnitude (the elements Adam's per-element normalisation amplifies).

  python tools/grad_err_diag.py --B 64 --warm 30
"""

import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.drift_diag import _batch  # noqa: E402


def ref_grads(params, target, b, A=18):
    from oracle.dqn_torch import TorchDQN, huber
    t = TorchDQN(params, A, target=target, dtype=torch.float64, device="cuda")
    dev = {k: torch.as_tensor(b[k]).cuda() for k in ("o_tm1", "a_tm1", "r_t", "d_t", "o_t")}
    q_tm1 = t.q(t.p, dev["o_tm1"])
    with torch.no_grad():
        q_t_value = t.q(t.t, dev["o_t"])
        q_t_selector = t.q(t.p, dev["o_t"])
    r = torch.clamp(dev["r_t"].double(), -1.0, 1.0)
    d = dev["d_t"].double() * t.discount
    best = q_t_selector.argmax(dim=1)
    tgt = r + d * q_t_value.gather(1, best[:, None])[:, 0]
    td = tgt - q_tm1.gather(1, dev["a_tm1"].long()[:, None])[:, 0]
    iw = (1.0 / b["probabilities"]) ** t.beta
    w = torch.from_numpy((iw / iw.max()).astype(np.float32)).cuda().double()
    loss = (w * huber(td)).mean()
    g = torch.autograd.grad(loss, [t.p[k] for k in t.names])
    return {k: v.cpu().numpy() for k, v in zip(t.names, g)}, float(loss.detach())


def ref_tensors(params, target, b, A=18):
    """float64 pre-activation gradients dz1..dz3 / dzh and activations x1..x3 of the online
    o_tm1 rows (NHWC, flattened per row as the learner's debug buffers)."""
    import torch.nn.functional as F
    from oracle.dqn_torch import CONVS, TorchDQN, huber
    from oracle.dqn_oracle import same_pads
    t = TorchDQN(params, A, target=target, dtype=torch.float64, device="cuda")
    dev = {k: torch.as_tensor(b[k]).cuda() for k in ("o_tm1", "a_tm1", "r_t", "d_t", "o_t")}
    p = t.p
    x = (dev["o_tm1"].double() / 255.0).permute(0, 3, 1, 2)
    pre, acts = [], []
    for name, k, s_ in CONVS:
        out, pt, pb = same_pads(x.shape[-1], k, s_)
        x = F.pad(x, (pt, pb, pt, pb))
        z = F.conv2d(x, p[f"{name}/w"].permute(3, 2, 0, 1), p[f"{name}/b"], stride=s_)
        z.retain_grad()
        pre.append(z)
        x = F.relu(z)
        acts.append(x)
    xf = x.permute(0, 2, 3, 1).reshape(x.shape[0], -1)
    zh = xf @ p["duelling_q_network/hidden/w"] + p["duelling_q_network/hidden/b"]
    zh.retain_grad()
    h = F.relu(zh)
    v = h[:, :512] @ p["duelling_q_network/mlp/linear_1/w"] + p["duelling_q_network/mlp/linear_1/b"]
    adv = h[:, 512:] @ p["duelling_q_network/mlp_1/linear_1/w"] + \
        p["duelling_q_network/mlp_1/linear_1/b"]
    q_tm1 = v + adv - adv.mean(dim=1, keepdim=True)
    with torch.no_grad():
        q_t_value = t.q(t.t, dev["o_t"])
        q_t_selector = t.q(t.p, dev["o_t"])
    r = torch.clamp(dev["r_t"].double(), -1.0, 1.0)
    d = dev["d_t"].double() * t.discount
    best = q_t_selector.argmax(dim=1)
    tgt = r + d * q_t_value.gather(1, best[:, None])[:, 0]
    td = tgt - q_tm1.gather(1, dev["a_tm1"].long()[:, None])[:, 0]
    iw = (1.0 / b["probabilities"]) ** t.beta
    w = torch.from_numpy((iw / iw.max()).astype(np.float32)).cuda().double()
    (w * huber(td)).mean().backward()
    nhwc = lambda z: z.permute(0, 2, 3, 1).reshape(z.shape[0], -1).detach().cpu().numpy()  # noqa
    out = {"dz1": nhwc(pre[0].grad), "dz2": nhwc(pre[1].grad), "dz3": nhwc(pre[2].grad),
           "dzh": zh.grad.detach().cpu().numpy(),
           "x1": nhwc(acts[0]), "x2": nhwc(acts[1]), "x3": nhwc(acts[2]),
           "hid": h.detach().cpu().numpy()}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=64)
    ap.add_argument("--warm", type=int, default=0)
    ap.add_argument("--out", default="gpurun_out/graderr")
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    from acme_amd._lib import lib
    from acme_amd.native import NativeDQN
    from acme_amd.networks import DQNAtariNetwork
    net = DQNAtariNetwork(18)
    p0, t0 = net.init(11), net.init(12)
    B = a.B
    rng = np.random.default_rng(1000 + B)
    warm = [_batch(rng, B, 18) for _ in range(a.warm)]
    b = _batch(rng, B, 18)
    d = NativeDQN(network="nature", num_actions=18, max_batch=B, obs_dtype="uint8")
    d.set_params(p0, t0)
    for w in warm:
        d.step(*[torch.as_tensor(w[k]).cuda().contiguous()
                 for k in ("o_tm1", "a_tm1", "r_t", "d_t", "o_t", "probabilities")])
    torch.cuda.synchronize()
    params, target = d.get_params("params"), d.get_params("target")
    ref, ref_loss = ref_grads(params, target, b)
    res = {}
    for eng, code in (("plane", 1), ("f32", 0)):
        lib().acme_set_matmul_engine(code)
        try:
            e = NativeDQN(network="nature", num_actions=18, max_batch=B, obs_dtype="uint8")
            e.set_params(params, target)
            # forward_backward only: the gradients of this batch from these parameters
            e.forward_backward(*[torch.as_tensor(b[k]).cuda().contiguous()
                                 for k in ("o_tm1", "a_tm1", "r_t", "d_t", "o_t",
                                           "probabilities")])
            torch.cuda.synchronize()
            g = e.get_params("grads")
            if True:
                print(f" {eng}:", flush=True)
                rt = ref_tensors(params, target, b)
                for name, r in rt.items():
                    got = e.debug_buffer(name)[:r.size].reshape(r.shape).astype(np.float64)
                    err = np.abs(got - r)
                    mx = float(np.abs(r).max())
                    nz = np.abs(r[r != 0])
                    if name == "dz1":  # conv1's weight gradient from the engine's own dz1
                        import torch.nn.functional as F
                        from oracle.dqn_oracle import same_pads
                        x = torch.as_tensor(b["o_tm1"]).cuda().double().permute(0, 3, 1, 2) / 255.0
                        _, pt, pb = same_pads(84, 8, 4)
                        x = F.pad(x, (pt, pb, pt, pb))
                        go = torch.as_tensor(got).cuda().view(B, 21, 21, 32).permute(0, 3, 1, 2)
                        wg = torch.nn.grad.conv2d_weight(x, (32, 4, 8, 8), go, stride=4)
                        wg = wg.permute(2, 3, 1, 0).cpu().numpy()  # OIHW -> HWIO
                        mine = g["atari_torso/conv2_d/w"].reshape(wg.shape)
                        rw = ref["atari_torso/conv2_d/w"]
                        print(f"  conv1 wgrad vs f64 of its own dz1: fro "
                              f"{np.linalg.norm(mine - wg) / np.linalg.norm(wg):.2e}; own dz1's "
                              f"f64 wgrad vs reference {np.linalg.norm(wg - rw) / np.linalg.norm(rw):.2e}",
                              flush=True)
                    ev = got - r
                    sg = np.sign(r)
                    print(f"  {name} error structure: mean/rms {ev.mean() / np.sqrt((ev ** 2).mean()):+.3f}"
                          f"  corr(err, sign) {np.mean(ev * sg) / np.sqrt((ev ** 2).mean()):+.3f}"
                          f"  corr(err, x) {np.corrcoef(ev.ravel(), r.ravel())[0, 1]:+.3f}"
                          f"  err/|x| median {np.median(np.abs(ev[r != 0]) / np.abs(r[r != 0])):.2e}",
                          flush=True)
                    print(f"  {name}: fro {np.linalg.norm(err) / np.linalg.norm(r):.2e} "
                          f"maxerr/max {err.max() / mx:.2e}; |x| quantiles/max "
                          f"50% {np.quantile(nz, 0.5) / mx:.2e} 90% {np.quantile(nz, 0.9) / mx:.2e} "
                          f"99% {np.quantile(nz, 0.99) / mx:.2e}; rms/max "
                          f"{np.sqrt(np.mean(r ** 2)) / mx:.2e}", flush=True)
        finally:
            lib().acme_set_matmul_engine(1)
        rows = {}
        for k, r in ref.items():
            x = g[k].reshape(r.shape).astype(np.float64)
            err = np.abs(x - r)
            fro = float(np.linalg.norm(err) / max(np.linalg.norm(r), 1e-300))
            big = float(np.mean(err > 1e-3 * np.abs(r)))
            rmax = float(np.abs(r).max())
            rows[k] = dict(fro=fro, frac_rel_1e3=big, max_err_over_max=float(err.max() / rmax))
        res[eng] = rows
    for k in ref:
        p, f = res["plane"][k], res["f32"][k]
        print(f"{k:45s} fro plane {p['fro']:.2e} f32 {f['fro']:.2e} | >1e-3 rel: plane "
              f"{p['frac_rel_1e3']:.4f} f32 {f['frac_rel_1e3']:.4f} | maxerr/max plane "
              f"{p['max_err_over_max']:.2e} f32 {f['max_err_over_max']:.2e}", flush=True)
    with open(os.path.join(a.out, f"graderr_B{B}_w{a.warm}.json"), "w") as fh:
        json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
