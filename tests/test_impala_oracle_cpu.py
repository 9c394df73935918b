"""IMPALA oracle (oracle/impala_oracle.py) checked against an independent torch-autograd
restatement of IMPALALearner._step (acme/agents/tf/impala/learning.py:97-160) with the
IMPALAAtariNetwork / OAR embedding (acme/tf/networks/atari.py:115-144,
embedding.py:26-45), plus V-trace properties (on-policy V-trace = n-step TD(lambda=1)
returns).  Parity with TF/trfl itself is UNPINNED (no reference test holds IMPALA values).
"""

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import impala_oracle as O
from oracle.dqn_oracle import CONVS

P = O.PREFIX


def _cfg(torso="flat", **kw):
    base = dict(num_actions=4, torso=torso, obs_dim=6, lstm_size=8, head_size=8,
                entropy_cost=0.01, baseline_cost=0.5)
    base.update(kw)
    return O.IMPALAConfig(**base)


def _params(cfg, seed):
    rng = np.random.default_rng(seed)
    return {n: (rng.standard_normal(s) / np.sqrt(s[0] if len(s) < 4 else np.prod(s[:3])))
            .astype(np.float32) for n, s in O.tensor_shapes(cfg)}


def _batch(cfg, B, T, seed):
    rng = np.random.default_rng(seed)
    A, H = cfg.num_actions, cfg.lstm_size
    if cfg.torso == "atari":
        obs = rng.integers(0, 256, (B, T, 84, 84, 4), dtype=np.uint8)
    else:
        obs = rng.standard_normal((B, T, cfg.obs_dim)).astype(np.float32)
    return dict(obs=obs, prev_action=rng.integers(0, A, (B, T)).astype(np.int32),
                prev_reward=rng.standard_normal((B, T)).astype(np.float32),
                action=rng.integers(0, A, (B, T)).astype(np.int32),
                reward=rng.standard_normal((B, T)).astype(np.float32),
                discount=np.where(rng.random((B, T)) < 0.2, 0.0, 1.0).astype(np.float32),
                behaviour_logits=rng.standard_normal((B, T, A)).astype(np.float32),
                h0=(0.5 * rng.standard_normal((B, H))).astype(np.float32),
                c0=(0.5 * rng.standard_normal((B, H))).astype(np.float32))


def _t_torso(p, obs):
    x = torch.tensor((obs.reshape((-1,) + obs.shape[2:]) / 255.0).astype(np.float32),
                     dtype=torch.float64)  # float32(u8 / 255), the AtariWrapper dtype
    x = x.permute(0, 3, 1, 2)
    for (name, s, pads), short in zip(CONVS, ["conv2_d", "conv2_d_1", "conv2_d_2"]):
        w = p[f"{P}/atari_torso/{short}/w"].permute(3, 2, 0, 1)
        pt, pl, pb, pr = pads
        x = F.relu(F.conv2d(F.pad(x, (pl, pr, pt, pb)), w, p[f"{P}/atari_torso/{short}/b"],
                            stride=s))
    return x.permute(0, 2, 3, 1).reshape(x.shape[0], -1)


def _torch_loss_and_grads(cfg, params, b):
    p = {k: torch.tensor(v, dtype=torch.float64, requires_grad=True) for k, v in params.items()}
    B, T = b["action"].shape
    A, H = cfg.num_actions, cfg.lstm_size
    if cfg.torso == "atari":
        feats = _t_torso(p, b["obs"])
    else:
        feats = torch.tensor(b["obs"].reshape(B * T, -1), dtype=torch.float64)
    emb = torch.cat([feats, F.one_hot(torch.tensor(b["prev_action"].reshape(-1), dtype=torch.long),
                                      A).double(),
                     torch.tanh(torch.tensor(b["prev_reward"].reshape(-1, 1), dtype=torch.float64))],
                    1).reshape(B, T, -1)
    h = torch.tensor(b["h0"], dtype=torch.float64)
    c = torch.tensor(b["c0"], dtype=torch.float64)
    outs = []
    for t in range(T):
        z = emb[:, t] @ p[f"{P}/lstm/w_i"] + h @ p[f"{P}/lstm/w_h"] + p[f"{P}/lstm/b"]
        i, f, g, o = z.split(H, 1)
        c = torch.sigmoid(f) * c + torch.sigmoid(i) * torch.tanh(g)
        h = torch.sigmoid(o) * torch.tanh(c)
        outs.append(h)
    hs = torch.stack(outs, 0)  # [T, B, H]
    hh = F.relu(hs @ p[f"{P}/linear/w"] + p[f"{P}/linear/b"])
    pv = hh @ p[f"{P}/policy_value/w"] + p[f"{P}/policy_value/b"]
    logits, values = pv[..., :A], pv[..., A]
    act = torch.tensor(b["action"].T[:-1], dtype=torch.long)
    rew = torch.tensor(b["reward"].T[:-1], dtype=torch.float64)
    disc = float(np.float32(cfg.discount)) * torch.tensor(b["discount"].T[:-1], dtype=torch.float64)
    mu = torch.tensor(np.swapaxes(b["behaviour_logits"], 0, 1)[:-1], dtype=torch.float64)
    logp = torch.log_softmax(logits[:-1], -1)
    lp_a = logp.gather(-1, act[..., None])[..., 0]
    log_rhos = lp_a - torch.log_softmax(mu, -1).gather(-1, act[..., None])[..., 0]
    with torch.no_grad():
        vs, pg_adv = O.vtrace(log_rhos.detach().numpy(), disc.numpy(), rew.numpy(),
                              values[:-1].detach().numpy(), values[-1].detach().numpy())
    vs, pg_adv = torch.tensor(vs), torch.tensor(pg_adv)
    critic = (vs - values[:-1]) ** 2
    pg = -lp_a * pg_adv
    ent = -(logp.exp() * logp).sum(-1)
    loss = (pg + cfg.baseline_cost * critic - cfg.entropy_cost * ent).mean()
    names = list(p)
    gr = torch.autograd.grad(loss, [p[k] for k in names], allow_unused=True)
    return float(loss.detach()), {k: (g.numpy() if g is not None else np.zeros_like(params[k]))
                                  for k, g in zip(names, gr)}


@pytest.mark.parametrize("torso,B,T", [("flat", 3, 5), ("flat", 2, 1 + 1), ("atari", 2, 3)])
def test_oracle_matches_torch_autograd(torso, B, T):
    cfg = _cfg(torso)
    params = _params(cfg, 0)
    b = _batch(cfg, B, T, 1)
    out, g = O.loss_and_grads(cfg, params, b, np.float64)
    loss, gt = _torch_loss_and_grads(cfg, params, b)
    assert abs(out["loss"] - loss) <= 1e-11 * max(1.0, abs(loss))
    assert set(g) == set(gt)
    for k in g:
        np.testing.assert_allclose(g[k], gt[k], rtol=1e-8, atol=1e-12, err_msg=k)


def test_vtrace_on_policy_is_lambda1_return():
    """With log_rhos = 0 (on-policy), vs_t is the discounted n-step return bootstrapped
    from the final value, and pg advantages are the one-step TD errors of vs."""
    rng = np.random.default_rng(0)
    T, B = 6, 3
    r = rng.standard_normal((T, B))
    d = np.where(rng.random((T, B)) < 0.2, 0.0, 0.9)
    v = rng.standard_normal((T, B))
    boot = rng.standard_normal(B)
    vs, pg = O.vtrace(np.zeros((T, B)), d, r, v, boot)
    ret = boot.copy()
    for t in reversed(range(T)):
        ret = r[t] + d[t] * ret
        np.testing.assert_allclose(vs[t], ret, rtol=1e-12)
    vs_tp1 = np.concatenate([vs[1:], boot[None]])
    np.testing.assert_allclose(pg, r + d * vs_tp1 - v, rtol=1e-12)


def test_vtrace_truncates_large_rhos():
    rng = np.random.default_rng(1)
    T, B = 4, 2
    r, v, boot = rng.standard_normal((T, B)), rng.standard_normal((T, B)), rng.standard_normal(B)
    d = np.full((T, B), 0.9)
    a, _ = O.vtrace(np.full((T, B), 3.0), d, r, v, boot)   # rho = e^3 -> clipped to 1
    b, _ = O.vtrace(np.zeros((T, B)), d, r, v, boot)       # rho = 1
    np.testing.assert_allclose(a, b, rtol=1e-12)
