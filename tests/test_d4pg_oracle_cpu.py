"""D4PG oracle (oracle/d4pg_oracle.py) checked two ways: against an
independent torch-autograd restatement of D4PGLearner._step's losses
(acme/agents/tf/d4pg/learning.py:186-229, losses/distributional.py, losses/dpg.py), and
against the l2_project / clip properties the reference's math implies.  Parity with TF
itself is UNPINNED (no reference test holds a D4PG golden value)."""

import os

import numpy as np
import pytest
import torch

from oracle import d4pg_oracle as O

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "d4pg_step_b8.npz")


def _small_cfg(**kw):
    base = dict(obs_dim=5, act_dim=3, policy_sizes=(16, 12, 8), critic_sizes=(20, 12, 8),
                num_atoms=11, vmin=-4.0, vmax=4.0, action_min=(-1.0, -2.0, 0.0),
                action_max=(1.0, 2.0, 0.5))
    base.update(kw)
    return O.D4PGConfig(**base)


def _params(cfg, seed, scale=0.5):
    rng = np.random.default_rng(seed)
    out = {}
    for name, shape in O.d4pg_tensor_shapes(cfg):
        if name.endswith("/scale"):
            out[name] = (1.0 + 0.1 * rng.standard_normal(shape)).astype(np.float32)
        else:
            out[name] = (scale * rng.standard_normal(shape) / np.sqrt(shape[0])).astype(np.float32)
    return out


def _batch(cfg, B, seed):
    rng = np.random.default_rng(seed)
    return dict(o_tm1=rng.standard_normal((B, cfg.obs_dim)).astype(np.float32),
                a_tm1=rng.uniform(-1, 1, (B, cfg.act_dim)).astype(np.float32),
                r_t=rng.uniform(-3, 3, B).astype(np.float32),
                d_t=np.where(rng.random(B) < 0.2, 0.0, 0.99 ** 4).astype(np.float32),
                o_t=rng.standard_normal((B, cfg.obs_dim)).astype(np.float32))


# ------------------------------------------------------------------ torch restatement


def _t_lnmlp(p, prefix, x, n, eps):
    pre = f"{prefix}/layer_norm_mlp"
    z = x @ p[f"{pre}/linear/w"] + p[f"{pre}/linear/b"]
    y = torch.nn.functional.layer_norm(z, (z.shape[1],), p[f"{pre}/layer_norm/scale"],
                                       p[f"{pre}/layer_norm/offset"], eps)
    h = torch.tanh(y)
    for i in range(n - 1):
        h = torch.nn.functional.elu(h @ p[f"{pre}/mlp/linear_{i}/w"] + p[f"{pre}/mlp/linear_{i}/b"])
    return h


def _t_policy(cfg, p, o):
    h = _t_lnmlp(p, "policy", o, len(cfg.policy_sizes), cfg.ln_eps)
    u = h @ p["policy/near_zero_initialized_linear/w"] + p["policy/near_zero_initialized_linear/b"]
    lo = torch.tensor(cfg.action_min, dtype=o.dtype)
    hi = torch.tensor(cfg.action_max, dtype=o.dtype)
    return (torch.tanh(u) + 1) * 0.5 * (hi - lo) + lo


def _t_critic(cfg, p, o, a):
    h = _t_lnmlp(p, "critic", torch.cat([o, a], 1), len(cfg.critic_sizes), cfg.ln_eps)
    return h @ p["critic/discrete_valued_head/linear/w"] + p["critic/discrete_valued_head/linear/b"]


def _t_project(zp, P, zq):
    vmin, vmax = zq[0], zq[-1]
    d_pos = torch.cat([zq, vmin[None]])[1:] - zq
    d_neg = zq - torch.cat([vmax[None], zq])[:-1]
    dqp = torch.clamp(zp, vmin, vmax)[:, None, :] - zq[None, :, None]
    sg = (dqp >= 0).to(P.dtype)
    dh = sg * dqp / d_pos[None, :, None] - (1 - sg) * dqp / d_neg[None, :, None]
    return (torch.clamp(1 - dh, 0, 1) * P[:, None, :]).sum(2)


def _torch_losses_and_grads(cfg, params, target, batch):
    p = {k: torch.tensor(v, dtype=torch.float64, requires_grad=True) for k, v in params.items()}
    tp = {k: torch.tensor(v, dtype=torch.float64) for k, v in target.items()}
    b = {k: torch.tensor(v, dtype=torch.float64) for k, v in batch.items()}
    values = torch.tensor(O.support(cfg, np.float64))
    q_tm1 = _t_critic(cfg, p, b["o_tm1"], b["a_tm1"])
    with torch.no_grad():
        q_t = _t_critic(cfg, tp, b["o_t"], _t_policy(cfg, tp, b["o_t"]))
        z = b["r_t"][:, None] + (float(np.float32(cfg.discount)) * b["d_t"])[:, None] * values[None]
        tgt = _t_project(z, torch.softmax(q_t, 1), values)
    critic_loss = -(tgt * torch.log_softmax(q_tm1, 1)).sum(1).mean()
    a = _t_policy(cfg, p, b["o_t"])
    q = (torch.softmax(_t_critic(cfg, p, b["o_t"], a), 1) * values).sum(1)
    dqda = torch.autograd.grad(q.sum(), a, retain_graph=True)[0]
    n = dqda.norm(dim=1, keepdim=True)
    dqda = dqda / torch.clamp(n, min=1.0)
    policy_loss = (0.5 * (((dqda + a).detach() - a) ** 2).sum(1)).mean()
    pn = [k for k in p if k.startswith("policy/")]
    cn = [k for k in p if k.startswith("critic/")]
    gp = torch.autograd.grad(policy_loss, [p[k] for k in pn])
    gc = torch.autograd.grad(critic_loss, [p[k] for k in cn])
    grads = {k: g.numpy() for k, g in zip(pn + cn, list(gp) + list(gc))}
    return float(critic_loss.detach()), float(policy_loss.detach()), grads, dqda.detach().numpy()


@pytest.mark.parametrize("seed", [0, 1])
def test_oracle_matches_torch_autograd(seed):
    cfg = _small_cfg()
    params, target = _params(cfg, seed), _params(cfg, seed + 10)
    batch = _batch(cfg, 9, seed + 20)
    out, g = O.d4pg_loss_and_grads(cfg, params, target, batch, np.float64)
    cl, pl, gt, dqda = _torch_losses_and_grads(cfg, params, target, batch)
    assert abs(out["critic_loss"] - cl) <= 1e-12 * max(1.0, abs(cl))
    assert abs(out["policy_loss"] - pl) <= 1e-12 * max(1.0, abs(pl))
    np.testing.assert_allclose(out["dqda"], dqda, rtol=1e-10, atol=1e-14)
    assert set(g) == set(gt)
    for k in g:
        np.testing.assert_allclose(g[k], gt[k], rtol=1e-9, atol=1e-13, err_msg=k)


def test_l2_project_properties():
    cfg = _small_cfg()
    zq = O.support(cfg, np.float64)
    rng = np.random.default_rng(3)
    P = rng.dirichlet(np.ones(cfg.num_atoms), 6)
    # Support-aligned atoms project onto themselves.
    np.testing.assert_allclose(O.l2_project(np.tile(zq, (6, 1)), P, zq), P, atol=1e-15)
    # Mass is preserved for any shifted/scaled support (clipped to [vmin, vmax]).
    zp = 3.0 * rng.standard_normal((6, cfg.num_atoms))
    out = O.l2_project(zp, P, zq)
    np.testing.assert_allclose(out.sum(1), 1.0, rtol=1e-12)
    assert (out >= 0).all()
    # All mass beyond vmax lands on the last atom.
    out = O.l2_project(np.full((1, cfg.num_atoms), 100.0), P[:1], zq)
    np.testing.assert_allclose(out[0, -1], 1.0)


def test_global_norm_clip_semantics():
    g = {"a": np.full(3, 30.0, np.float32), "b": np.full(4, 20.0, np.float32)}
    clipped, G = O.global_norm_clip(g, 40.0, np.float32)
    assert abs(G - np.sqrt(3 * 900 + 4 * 400)) < 1e-9
    tot = np.sqrt(sum(float((v.astype(np.float64) ** 2).sum()) for v in clipped.values()))
    assert abs(tot - 40.0) < 1e-4
    small = {"a": np.full(2, 1.0, np.float32)}
    out, _ = O.global_norm_clip(small, 40.0, np.float32)
    np.testing.assert_array_equal(out["a"], small["a"])  # scale == 1.0 exactly in f32


def test_step_target_copy_at_start():
    cfg = _small_cfg(target_update_period=2)
    params, target = _params(cfg, 0), _params(cfg, 5)
    z = {k: np.zeros_like(v) for k, v in params.items()}
    state = dict(params=params, target=target, m=z, v=dict(z), num_steps=0)
    b = _batch(cfg, 4, 1)
    _, _, s1 = O.d4pg_step(cfg, state, b)
    for k in params:  # step 0 copied the PRE-update online weights (learning.py:171-174)
        np.testing.assert_array_equal(s1["target"][k], params[k])
    _, _, s2 = O.d4pg_step(cfg, s1, b)
    for k in params:  # step 1: no copy
        np.testing.assert_array_equal(s2["target"][k], s1["target"][k])
    _, _, s3 = O.d4pg_step(cfg, s2, b)
    for k in params:
        np.testing.assert_array_equal(s3["target"][k], s2["params"][k])


def test_golden_fixture_reproduces():
    """tests/golden/d4pg_step_b8.npz (made by tests/golden/make_d4pg_golden.py from this
    oracle): guards the restatement against silent drift."""
    from tests.golden.make_d4pg_golden import compute, golden_cfg
    z = np.load(GOLDEN)
    cfg = golden_cfg()
    got = compute(cfg, z)
    for k, v in got.items():
        np.testing.assert_allclose(v, z["out/" + k], rtol=1e-12, atol=1e-15, err_msg=k)
