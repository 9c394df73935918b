"""HIP IMPALA learner step vs the numpy oracle (oracle/impala_oracle.py, float64).

Reference: IMPALALearner._step (acme/agents/tf/impala/learning.py:97-169).
Tolerances (fp32 kernels against an fp64 restatement):
  losses / logits / values / vs / pg advantages: rtol 1e-5 (+ 2e-6 of the tensor's scale)
  gradients: per tensor |g - g_ref| <= 1e-4 |g_ref| + 2e-5 max|g_ref|, conditional on the
      kernel's own ReLU pattern (torso x1..x3 and the head's hh; see _relu_masks)
  Adam-updated params: every element within 2 lr, 99% within 1e-5 relative.
"""

import numpy as np
import pytest
import torch

from oracle import impala_oracle as O

pytestmark = pytest.mark.gpu


def _native(cfg, B, T, **kw):
    from acme_amd.native import NativeIMPALA
    return NativeIMPALA(num_actions=cfg.num_actions, max_batch=B, max_sequence_length=T,
                        torso=cfg.torso, obs_dim=cfg.obs_dim, lstm_size=cfg.lstm_size,
                        head_size=cfg.head_size, discount=cfg.discount,
                        entropy_cost=cfg.entropy_cost, baseline_cost=cfg.baseline_cost,
                        learning_rate=cfg.learning_rate, **kw)


def _params(cfg, seed):
    rng = np.random.default_rng(seed)
    out = {}
    for n, s in O.tensor_shapes(cfg):
        fan = np.prod(s[:-1]) if len(s) > 1 else s[0]
        out[n] = (rng.standard_normal(s) / np.sqrt(fan)).astype(np.float32)
        if n.endswith("/b"):
            out[n] = (0.1 * rng.standard_normal(s)).astype(np.float32)
    return out


def _batch(cfg, B, T, seed):
    rng = np.random.default_rng(seed)
    A, H = cfg.num_actions, cfg.lstm_size
    if cfg.torso == "atari":
        obs = rng.integers(0, 256, (B, T, 84, 84, 4), dtype=np.uint8)
    else:
        obs = rng.standard_normal((B, T, cfg.obs_dim)).astype(np.float32)
    state = (0.5 * rng.standard_normal((B, T, 2, H))).astype(np.float32)
    return dict(obs=obs, prev_action=rng.integers(0, A, (B, T)).astype(np.int32),
                prev_reward=rng.standard_normal((B, T)).astype(np.float32),
                action=rng.integers(0, A, (B, T)).astype(np.int32),
                reward=(2 * rng.standard_normal((B, T))).astype(np.float32),
                discount=np.where(rng.random((B, T)) < 0.1, 0.0, 1.0).astype(np.float32),
                behaviour_logits=rng.standard_normal((B, T, A)).astype(np.float32),
                state=state, h0=state[:, 0, 0].copy(), c0=state[:, 0, 1].copy())


def _run(n, b):
    d = lambda k: torch.as_tensor(b[k]).cuda().contiguous()  # noqa: E731
    st = torch.as_tensor(b["state"]).cuda()
    # core_state[:, 0] views of a [B, T, 2, H] extras tensor: row stride T * 2 * H.
    n.step(d("obs"), d("prev_action"), d("prev_reward"), d("action"), d("reward"),
           d("discount"), d("behaviour_logits"), st[:, 0, 0], st[:, 0, 1])
    torch.cuda.synchronize()


def _close(got, ref, rtol=1e-5, floor=2e-6, name=""):
    ref = np.asarray(ref, np.float64)
    got = np.asarray(got, np.float64).reshape(ref.shape)
    scale = max(float(np.abs(ref).max()), 1e-30)
    np.testing.assert_allclose(got, ref, rtol=rtol, atol=floor * scale, err_msg=name)


def _check_grads(n, g_ref, frob_only=()):
    g = n.get_params("grads")
    for name, ref in g_ref.items():
        got = g[name].reshape(ref.shape).astype(np.float64)
        if any(name.startswith(p) for p in frob_only):
            rel = np.linalg.norm(got - ref) / max(np.linalg.norm(ref), 1e-30)
            assert rel <= 1e-4, (name, rel)
            continue
        scale = np.abs(ref).max()
        err = np.abs(got - ref)
        assert (err <= 1e-4 * np.abs(ref) + 2e-5 * scale + 1e-30).all(), \
            (name, float(err.max()), float(scale))


def _check_params(got, ref, lr):
    for k, r in ref.items():
        gk = got[k].reshape(r.shape).astype(np.float64)
        err = np.abs(gk - r)
        assert err.max() <= 2 * lr + 1e-6, (k, float(err.max()))
        assert np.mean(err <= 1e-5 * np.abs(r) + 1e-7) >= 0.99, k


def _relu_masks(cfg, n, params, b):
    """The kernel's own ReLU pattern (forward activations checked first; flips only where
    the f64 pre-activation is within fp32 rounding of 0), so that gradients are compared
    conditional on the same branch decisions (as tests/test_dqn_gpu.py::_relu_masks)."""
    _, _, cache = O.forward(cfg, params, b, np.float64)
    names = ["hh"] + (["x1", "x2", "x3"] if cfg.torso == "atari" else [])
    masks = {}
    for name in names:
        ref = cache[name]
        got = n.debug_buffer(name)[:ref.size].reshape(ref.shape)
        scale = np.abs(ref).max()
        np.testing.assert_allclose(got, ref, rtol=1e-5, atol=2e-6 * scale, err_msg=name)
        m = got > 0
        flips = m != (ref > 0)
        assert (np.abs(ref[flips]) <= 2e-6 * scale).all(), name
        assert flips.mean() < 1e-4, (name, flips.mean())
        masks[name] = m
    return masks


def _compare(cfg, n, params, b, frob_only=()):
    z = {k: np.zeros_like(v) for k, v in params.items()}
    masks = _relu_masks(cfg, n, params, b)
    ref, raw, st = O.impala_step(cfg, dict(params=params, m=z, v=dict(z), num_steps=0), b,
                                 masks=masks)
    B, T = b["action"].shape
    A = cfg.num_actions
    m = n.metrics.cpu().numpy()
    _close(m[0], ref["loss"], name="loss")
    _close(m[1], ref["critic_loss"], name="critic_loss")
    _close(m[2], ref["entropy_loss"], name="entropy_loss")
    _close(m[3], ref["policy_gradient_loss"], name="pg_loss")
    pv = n.debug_buffer("pv")[:B * T * (A + 1)].reshape(B, T, A + 1)
    _close(pv[..., :A], ref["logits"], name="logits")
    _close(pv[..., A], ref["values"], name="values")
    _close(n.debug_buffer("vs")[:(T - 1) * B].reshape(T - 1, B), ref["vs"], name="vs")
    _close(n.debug_buffer("pg_adv")[:(T - 1) * B].reshape(T - 1, B), ref["pg_advantages"],
           name="pg_adv")
    _check_grads(n, raw, frob_only)
    _check_params(n.get_params("params"), st["params"], cfg.learning_rate)


@pytest.mark.parametrize("B,T,H", [(4, 6, 16), (16, 20, 256), (3, 2, 8), (64, 3, 256)])
def test_flat_torso_step_matches_oracle(B, T, H):
    cfg = O.IMPALAConfig(num_actions=5, torso="flat", obs_dim=12, lstm_size=H,
                         head_size=max(H // 2, 4) // 4 * 4, entropy_cost=0.01, baseline_cost=0.5)
    n = _native(cfg, B, T)
    params = _params(cfg, 1)
    n.set_params(params)
    b = _batch(cfg, B, T, 2)
    _run(n, b)
    _compare(cfg, n, params, b)


@pytest.mark.parametrize("B,T,f32", [(2, 5, False), (16, 20, False), (16, 20, True)])
def test_atari_torso_step_matches_oracle(B, T, f32):
    """IMPALAAtariNetwork at full width (LSTM 256, head 256, 18 actions); (16, 20) is the
    configs[3] learner batch (agents/tf/impala/agent.py:50, 20-step rollouts).  Steps of at
    least 64 frames run the torso and the W_i projection / gradients on the exact plane
    engine (the DQN kernels); f32: the f32 engine throughout (ACME_V_IMP3=1)."""
    from acme_amd._lib import lib
    cfg = O.IMPALAConfig(num_actions=18, torso="atari", entropy_cost=0.01, baseline_cost=0.5)
    lib().acme_tune_set(b"IMP3", 1 if f32 else 0)  # read once, at the learner's creation
    try:
        n = _native(cfg, B, T)
    finally:
        lib().acme_tune_set(b"IMP3", 0)
    params = _params(cfg, 3)
    n.set_params(params)
    b = _batch(cfg, B, T, 4)
    _run(n, b)
    _compare(cfg, n, params, b)


def test_policy_step_matches_unroll():
    cfg = O.IMPALAConfig(num_actions=6, torso="flat", obs_dim=10, lstm_size=32, head_size=16)
    n = _native(cfg, 8, 4)
    params = _params(cfg, 5)
    n.set_params(params)
    b = _batch(cfg, 8, 2, 6)
    logits, values, cache = O.forward(cfg, params, b, np.float64)
    d = lambda x: torch.as_tensor(np.ascontiguousarray(x)).cuda()  # noqa: E731
    lg, v, h, c = n.policy_step(d(b["obs"][:, 0]), d(b["prev_action"][:, 0]),
                                d(b["prev_reward"][:, 0]), d(b["h0"]), d(b["c0"]))
    _close(lg.cpu().numpy(), logits[:, 0], name="logits")
    _close(v.cpu().numpy(), values[:, 0], name="values")
    _close(h.cpu().numpy(), cache["hs"][:, 0], name="h")
    _close(c.cpu().numpy(), cache["cs"][:, 0], name="c")


def test_policy_step_on_planes_matches_oracle():
    """The actor-side policy step on the plane engine (acme_impala_set_policy_planes: Atari
    torso and W_i on f16 planes, scales calibrated on the first call and rescaled after each)
    against the f64 forward, for two consecutive 64-row calls (the second at the scales the
    first one set), with no plane overflow."""
    cfg = O.IMPALAConfig(num_actions=18, torso="atari", lstm_size=256, head_size=256)
    rows = 64
    n = _native(cfg, rows, 2)
    n.set_policy_planes(True)
    params = _params(cfg, 7)
    n.set_params(params)
    d = lambda x: torch.as_tensor(np.ascontiguousarray(x)).cuda()  # noqa: E731
    for call in range(2):
        b = _batch(cfg, rows, 1, 30 + call)
        logits, values, cache = O.forward(cfg, params, b, np.float64)
        lg, v, h, c = n.policy_step(d(b["obs"][:, 0]), d(b["prev_action"][:, 0]),
                                    d(b["prev_reward"][:, 0]), d(b["h0"]), d(b["c0"]))
        _close(lg.cpu().numpy(), logits[:, 0], name=f"logits {call}")
        _close(v.cpu().numpy(), values[:, 0], name=f"values {call}")
        _close(h.cpu().numpy(), cache["hs"][:, 0], name=f"h {call}")
        _close(c.cpu().numpy(), cache["cs"][:, 0], name=f"c {call}")
    assert not n.plane_overflow()


@pytest.mark.parametrize("B,T,H,torso", [(16, 20, 256, "flat"), (3, 7, 256, "flat"),
                                         (27, 5, 256, "flat"), (16, 2, 256, "flat"),
                                         (16, 20, 256, "atari")])
def test_persistent_lstm_unroll_matches_per_step(B, T, H, torso):
    """The one-launch LSTM forward and backward (lstm_fwd_rg_kernel / lstm_bwd_rg_kernel:
    workgroups own 4 sequences x 16 units with their W_h slice in registers across the
    unroll and exchange h_t and the dh partial products as tagged granules; the default for
    lstm_size 256 and at most 64 sequences) against the per-step launches: h, c, gate
    gradients, the policy/value outputs and the losses equal to fp32 rounding (the sums run
    in another order), no spin timeout.  Both are checked against the f64 oracle by the
    tests above (64 sequences, 256 co-resident workgroups, there only: the per-step forward
    holds every row's h in 64 KB of LDS); ragged row groups (B = 3, 27) and the shortest
    unroll (T = 2) included."""
    cfg = O.IMPALAConfig(num_actions=18 if torso == "atari" else 5, torso=torso, obs_dim=12,
                         lstm_size=H, head_size=64, entropy_cost=0.01, baseline_cost=0.5)
    params = _params(cfg, 5)
    b = _batch(cfg, B, T, 6)
    res = {}
    for per_step in (False, True):
        n = _native(cfg, B, T)
        n.set_lstm_unroll(per_step)
        n.set_params(params)
        _run(n, b)
        res[per_step] = {k: n.debug_buffer(k) for k in ("h", "c", "dgates", "pv")}
        res[per_step]["metrics"] = n.metrics.cpu().numpy()
        res[per_step]["grads"] = n.grads.cpu().numpy()
        res[per_step]["tmo"] = n.debug_buffer("lstm_timeout")[:1].view(np.uint32)
    assert res[False]["tmo"][0] == 0
    for k in ("h", "c", "dgates", "pv", "metrics", "grads"):
        scale = float(np.abs(res[True][k]).max())
        np.testing.assert_allclose(res[False][k], res[True][k], rtol=2e-5, atol=2e-6 * scale,
                                   err_msg=k)
