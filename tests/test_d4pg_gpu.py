"""HIP D4PG learner step vs the numpy oracle (oracle/d4pg_oracle.py, float64).

Reference: D4PGLearner._step (acme/agents/tf/d4pg/learning.py:156-247).
Tolerances (fp32 kernels against an fp64 restatement):
  losses, actions, logits, dqda, global norms: rtol 1e-5 (+ a small atol at the fp32
      rounding floor of the tensor's scale)
  gradients: per tensor |g - g_ref| <= 1e-4 |g_ref| + 2e-5 max|g_ref|
  Adam-updated params: every element within 2 lr of the oracle's and 99% within
      1e-5 relative (Adam normalises each gradient element, so elements whose gradient
      sits at the fp32 rounding floor may take a different sign).
"""

import os

import numpy as np
import pytest
import torch

from oracle import d4pg_oracle as O

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "d4pg_step_b8.npz")


def _native(cfg, B, **kw):
    from acme_amd.native import NativeD4PG
    return NativeD4PG(obs_dim=cfg.obs_dim, act_dim=cfg.act_dim, max_batch=B,
                      policy_sizes=cfg.policy_sizes, critic_sizes=cfg.critic_sizes,
                      num_atoms=cfg.num_atoms, vmin=cfg.vmin, vmax=cfg.vmax,
                      action_min=cfg.action_min, action_max=cfg.action_max,
                      discount=cfg.discount, target_update_period=cfg.target_update_period,
                      policy_learning_rate=cfg.policy_lr, critic_learning_rate=cfg.critic_lr,
                      clipping=cfg.clipping, **kw)


def _dev(batch):
    return [torch.as_tensor(batch[k]).cuda().contiguous()
            for k in ("o_tm1", "a_tm1", "r_t", "d_t", "o_t")]


def _close(got, ref, rtol=1e-5, floor=2e-6, name=""):
    ref = np.asarray(ref, np.float64)
    got = np.asarray(got, np.float64).reshape(ref.shape)
    scale = max(float(np.abs(ref).max()), 1e-30)
    np.testing.assert_allclose(got, ref, rtol=rtol, atol=floor * scale, err_msg=name)


def _check_grads(native, g_ref):
    g = native.get_params("grads")
    for name, ref in g_ref.items():
        got = g[name].reshape(ref.shape).astype(np.float64)
        scale = np.abs(ref).max()
        err = np.abs(got - ref)
        bound = 1e-4 * np.abs(ref) + 2e-5 * scale + 1e-30
        assert (err <= bound).all(), (name, float(err.max()), float(scale))


def _check_params(got, ref, lr):
    for k, r in ref.items():
        gk = got[k].reshape(r.shape).astype(np.float64)
        err = np.abs(gk - r)
        assert err.max() <= 2 * lr + 1e-6, (k, float(err.max()))
        frac = np.mean(err <= 1e-5 * np.abs(r) + 1e-7)
        assert frac >= 0.99, (k, frac)


def _random_params(cfg, seed):
    rng = np.random.default_rng(seed)
    out = {}
    for name, shape in O.d4pg_tensor_shapes(cfg):
        if name.endswith("/scale"):
            v = 1.0 + 0.1 * rng.standard_normal(shape)
        elif name.endswith("/b") or name.endswith("/offset"):
            v = 0.1 * rng.standard_normal(shape)
        else:
            v = rng.standard_normal(shape) / np.sqrt(shape[0])
        out[name] = v.astype(np.float32)
    return out


def _batch(cfg, B, seed):
    rng = np.random.default_rng(seed)
    d = np.where(rng.random(B) < 0.05, 0.0, 0.99 ** 4).astype(np.float32)
    return dict(o_tm1=rng.standard_normal((B, cfg.obs_dim)).astype(np.float32),
                a_tm1=rng.uniform(-1, 1, (B, cfg.act_dim)).astype(np.float32),
                r_t=rng.uniform(0, 5, B).astype(np.float32), d_t=d,
                o_t=rng.standard_normal((B, cfg.obs_dim)).astype(np.float32))


def test_tensor_layout_matches_oracle():
    cfg = O.D4PGConfig()
    n = _native(cfg, 8)
    assert [(k, s) for k, _, s in n.tensors] == O.d4pg_tensor_shapes(cfg)
    assert n.policy_size == [o for k, o, _ in n.tensors if k.startswith("critic/")][0]


def test_golden_step():
    from tests.golden.make_d4pg_golden import golden_cfg, unpack
    z = np.load(GOLDEN)
    cfg = golden_cfg()
    params, target, batch = unpack(cfg, z)
    B = len(batch["r_t"])
    n = _native(cfg, B)
    n.set_params(params, target)
    n.num_steps = 1  # no start-of-step target copy; Adam t = 2
    n.step(*_dev(batch))
    torch.cuda.synchronize()
    out = lambda k: z["out/" + k]  # noqa: E731
    _close(n.critic_loss.item(), out("critic_loss"), name="critic_loss")
    _close(n.policy_loss.item(), out("policy_loss"), name="policy_loss")
    _close(n.debug_buffer("p_a")[:B * 6], out("dpg_a"), name="dpg_a")
    _close(n.debug_buffer("t_a")[:B * 6], out("a_target"), name="a_target")
    _close(n.debug_buffer("c_logits")[:B * 51], out("q_tm1"), name="q_tm1")
    _close(n.debug_buffer("t_logits")[:B * 51], out("q_t"), name="q_t")
    _close(n.debug_buffer("dqda")[:B * 6], out("dqda"), rtol=1e-4, name="dqda")
    _close(n.debug_buffer("norms"), out("norms"), rtol=1e-5, name="norms")
    _check_grads(n, {k[len("out/grad/"):]: z[k] for k in z.files if k.startswith("out/grad/")})
    _check_params(n.get_params("params"),
                  {k[len("out/new/"):]: z[k] for k in z.files if k.startswith("out/new/")},
                  cfg.policy_lr)


@pytest.mark.parametrize("B", [256, 37])
def test_full_size_steps_match_oracle(B):
    """Config-3 networks (policy 256x3, critic 512/512/256, 51 atoms): three steps with a
    target period of 2, so steps 0 and 2 copy online -> target at the start."""
    cfg = O.D4PGConfig(target_update_period=2)
    n = _native(cfg, 256)
    params, target = _random_params(cfg, 1), _random_params(cfg, 2)
    n.set_params(params, target)
    z = {k: np.zeros_like(v) for k, v in params.items()}
    state = dict(params=params, target=target, m=z, v=dict(z), num_steps=0)
    for s in range(3):
        batch = _batch(cfg, B, 10 + s)
        n.step(*_dev(batch))
        torch.cuda.synchronize()
        ref, raw, state = O.d4pg_step(cfg, state, batch, np.float64)
        _close(n.critic_loss.item(), ref["critic_loss"], name=f"critic_loss@{s}")
        _close(n.policy_loss.item(), ref["policy_loss"], rtol=1e-4, name=f"policy_loss@{s}")
        _close(n.debug_buffer("norms"), ref["norms"], rtol=1e-4, name=f"norms@{s}")
        _check_grads(n, raw)
        got = n.get_params("params")
        _check_params(got, state["params"], cfg.policy_lr)
        # Continue the oracle from the kernel's parameters so fp32 drift cannot compound.
        state["params"] = {k: got[k].astype(np.float32) for k in got}
        state["m"] = n.get_params("m")
        state["v"] = n.get_params("v")
        tgt = n.get_params("target")
        for k, r in state["target"].items():
            np.testing.assert_array_equal(tgt[k], np.asarray(r, np.float32), err_msg=k)
        state["target"] = tgt
    assert n.num_steps == 3


@pytest.mark.parametrize("B", [45, 600])
def test_odd_shapes_match_oracle(B):
    """Widths that are not multiples of the 32-wide tiles, a 1024-wide layer input (two
    passes of the register-operand engine's k loop), 21 atoms, 3 actions, 7 observations,
    a ragged batch and one past 512 rows (two k passes in the weight gradients): the direct
    engine's edges (rows and columns past M and N, k past K read as zero) and the widest
    LayerNorm instantiations, two steps against the float64 oracle."""
    cfg = O.D4PGConfig(obs_dim=7, act_dim=3, policy_sizes=(36, 100),
                       critic_sizes=(1024, 132, 44), num_atoms=21, vmin=-10.0, vmax=10.0,
                       action_min=(-1.0,) * 3, action_max=(1.0,) * 3, target_update_period=2)
    n = _native(cfg, B)
    params, target = _random_params(cfg, 7), _random_params(cfg, 8)
    n.set_params(params, target)
    z = {k: np.zeros_like(v) for k, v in params.items()}
    state = dict(params=params, target=target, m=z, v=dict(z), num_steps=0)
    for s in range(2):
        batch = _batch(cfg, B, 20 + s)
        n.step(*_dev(batch))
        torch.cuda.synchronize()
        ref, raw, state = O.d4pg_step(cfg, state, batch, np.float64)
        _close(n.critic_loss.item(), ref["critic_loss"], name=f"critic_loss@{s}")
        _close(n.policy_loss.item(), ref["policy_loss"], rtol=1e-4, name=f"policy_loss@{s}")
        _check_grads(n, raw)
        got = n.get_params("params")
        _check_params(got, state["params"], cfg.policy_lr)
        state["params"] = {k: got[k].astype(np.float32) for k in got}
        state["m"] = n.get_params("m")
        state["v"] = n.get_params("v")
        state["target"] = n.get_params("target")


def test_policy_forward_matches_oracle():
    cfg = O.D4PGConfig(action_min=(-2.0,) * 6, action_max=(0.5,) * 6)
    n = _native(cfg, 64)
    params = _random_params(cfg, 3)
    n.set_params(params, _random_params(cfg, 4))
    obs = np.random.default_rng(0).standard_normal((150, 24)).astype(np.float32)
    got = n.policy(torch.as_tensor(obs)).cpu().numpy()  # 150 rows > max_batch: chunked
    ref, _ = O.policy_forward(cfg, params, obs, np.float64)
    _close(got, ref, name="policy")
    assert (got >= -2.0).all() and (got <= 0.5).all()


def test_no_clipping_path():
    cfg = O.D4PGConfig(clipping=False, policy_sizes=(64, 64), critic_sizes=(128, 64))
    n = _native(cfg, 32)
    params, target = _random_params(cfg, 5), _random_params(cfg, 6)
    n.set_params(params, target)
    n.num_steps = 1
    batch = _batch(cfg, 32, 3)
    n.step(*_dev(batch))
    torch.cuda.synchronize()
    z = {k: np.zeros_like(v) for k, v in params.items()}
    ref, raw, st = O.d4pg_step(cfg, dict(params=params, target=target, m=z, v=dict(z),
                                         num_steps=1), batch, np.float64)
    _close(n.critic_loss.item(), ref["critic_loss"], name="critic_loss")
    _check_grads(n, raw)
    _check_params(n.get_params("params"), st["params"], cfg.policy_lr)


def test_learner_dropin_path():
    """D4PGLearner through the uniform GPU replay Table + make_reverb_dataset (config 3
    data layout), plus the reference's get_variables contract."""
    from acme_amd import replay, specs
    from acme_amd.adders import reverb as adders
    from acme_amd.agents.d4pg import D4PGLearner
    from acme_amd.datasets import make_reverb_dataset
    from acme_amd.networks import make_d4pg_networks
    from acme_amd.utils import loggers
    env_spec = specs.EnvironmentSpec(
        observations=specs.Array((24,), np.float32),
        actions=specs.BoundedArray((6,), np.float32, -1.0, 1.0),
        rewards=specs.Array((), np.float32), discounts=specs.BoundedArray((), np.float32, 0, 1))
    table = replay.Table(adders.DEFAULT_PRIORITY_TABLE, replay.selectors.Uniform(),
                         replay.selectors.Fifo(), 4096, replay.rate_limiters.MinSize(1),
                         signature=adders.NStepTransitionAdder.signature(env_spec), seed=7)
    table.native.fill_synthetic(4096, layout=1, num_actions=1, seed=0)
    server = replay.Server([table])
    nets = make_d4pg_networks(24, env_spec.actions)
    learner = D4PGLearner(nets["policy"], nets["critic"], nets["policy"], nets["critic"],
                          discount=0.99, target_update_period=100,
                          dataset=make_reverb_dataset(server, batch_size=256),
                          logger=loggers.NoOpLogger())
    for _ in range(3):
        learner.step()
    torch.cuda.synchronize()
    assert learner.num_steps == 3
    assert np.isfinite(learner.native.critic_loss.item())
    crit, pol = learner.get_variables(["critic", "policy"])
    assert all(k.startswith("critic/") for k in crit) and len(crit) == 10
    assert all(k.startswith("policy/") for k in pol) and len(pol) == 10
    a = learner.policy(np.zeros((2, 24), np.float32))
    assert a.shape == (2, 6) and np.isfinite(a).all()


def test_graph_replay_matches_eager():
    """The captured step graph (default) and the eager launch sequence (forced by the
    section profiler) produce bit-identical parameters, including across the target copy
    and with the two alternating batch buffers the dataset iterator uses."""
    from acme_amd import _lib
    cfg = O.D4PGConfig(target_update_period=2, policy_sizes=(64, 64, 64),
                       critic_sizes=(128, 128, 64))
    params, target = _random_params(cfg, 11), _random_params(cfg, 12)
    batches = [_dev(_batch(cfg, 64, 20 + i)) for i in range(2)]
    results = []
    for eager in (True, False):
        n = _native(cfg, 64)
        n.set_params(params, target)
        _lib.lib().acme_profile_enable(1 if eager else 0)
        try:
            for s in range(5):
                n.step(*batches[s % 2])
        finally:
            _lib.lib().acme_profile_enable(0)
        torch.cuda.synchronize()
        results.append((n.get_params("params"), n.get_params("target"),
                        n.critic_loss.item(), n.policy_loss.item()))
    (p0, t0, c0, l0), (p1, t1, c1, l1) = results
    for k in p0:
        np.testing.assert_array_equal(p0[k], p1[k], err_msg=k)
        np.testing.assert_array_equal(t0[k], t1[k], err_msg=k)
    assert c0 == c1 and l0 == l1
