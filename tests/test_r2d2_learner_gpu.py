"""HIP R2D2 learner step (csrc/r2d2_learner.hip) vs the numpy oracle
(oracle/r2d2_oracle.py, float64).

Reference: R2D2Learner._step (acme/agents/tf/r2d2/learning.py:112-200) with
R2D2AtariNetwork (acme/tf/networks/atari.py:72-112) and transformed_n_step_loss
(acme/tf/losses/r2d2.py:29-169).  Tolerances (fp32 kernels against an fp64 restatement):
  q values (online / target suffix rows): rtol 1e-5 (+ 2e-6 of the tensor's scale)
  the loss kernel, bit for bit against TF's float32 loss arithmetic evaluated on the
      kernel's own q values (oracle transformed_loss, teacher-forced): errors, priorities,
      d loss / d q[a]
  errors / loss end to end against the f64 networks: 2.5e-4 absolute / 2e-4 relative (the
      f32 value transform h^-1 subtracts 500 from ~501: the reference's own f32 loss
      resolves ~6.1e-5, oracle signed_parabolic_f32)
  gradients: the f64 backward from the kernel's d loss / d q, per tensor |g - g_ref| <=
      1e-4 |g_ref| + 2e-5 max|g_ref|, conditional on the kernel's own ReLU pattern (torso
      x1..x3 and the duelling hidden layer)
  Adam-updated params: every element within 2 lr, 99% within 1e-5 relative; the target copy
      (num_steps % period == 0 after the update) bit-identical to the updated params.
"""

import numpy as np
import pytest
import torch

from oracle import r2d2_oracle as O

pytestmark = pytest.mark.gpu


def _cfg(**kw):
    base = dict(num_actions=5, torso="flat", obs_dim=12, lstm_size=16, head_size=8,
                burn_in_length=2, n_step=3, max_replay_size=1000, target_update_period=2)
    base.update(kw)
    return O.R2D2Config(**base)


def _native(cfg, B, T):
    from acme_amd.native import NativeR2D2
    return NativeR2D2(num_actions=cfg.num_actions, max_batch=B, max_sequence_length=T,
                      burn_in_length=cfg.burn_in_length, torso=cfg.torso, obs_dim=cfg.obs_dim,
                      lstm_size=cfg.lstm_size, head_size=cfg.head_size, n_step=cfg.n_step,
                      discount=cfg.discount,
                      importance_sampling_exponent=cfg.importance_sampling_exponent,
                      max_replay_size=cfg.max_replay_size,
                      max_priority_weight=cfg.max_priority_weight,
                      target_update_period=cfg.target_update_period,
                      learning_rate=cfg.learning_rate, adam_epsilon=cfg.adam_epsilon,
                      store_lstm_state=cfg.store_lstm_state)


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
                state=state, h0=state[:, 0, 0].copy(), c0=state[:, 0, 1].copy(),
                probabilities=(0.5 + rng.random(B)) / (B * 4.0))


def _run(n, b):
    d = lambda k: torch.as_tensor(b[k]).cuda().contiguous()  # noqa: E731
    st = torch.as_tensor(b["state"]).cuda()
    # core_state[:, 0] views of a [B, T, 2, H] extras tensor: row stride T * 2 * H.
    n.step(d("obs"), d("prev_action"), d("prev_reward"), d("action"), d("reward"),
           d("discount"), torch.as_tensor(b["probabilities"], dtype=torch.float64).cuda(),
           st[:, 0, 0], st[:, 0, 1])
    torch.cuda.synchronize()


def _close(got, ref, rtol=1e-5, floor=2e-6, name=""):
    ref = np.asarray(ref, np.float64)
    got = np.asarray(got, np.float64).reshape(ref.shape)
    scale = max(float(np.abs(ref).max()), 1e-30)
    np.testing.assert_allclose(got, ref, rtol=rtol, atol=floor * scale, err_msg=name)


def _check_grads(n, g_ref):
    g = n.get_params("grads")
    for name, ref in g_ref.items():
        got = g[name].reshape(ref.shape).astype(np.float64)
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


def _tm(x, B, T):
    """Time-major rows [T * B, ...] of a kernel buffer -> batch-major [B, T, ...]."""
    return np.swapaxes(x.reshape((T, B) + x.shape[1:]), 0, 1)


def _relu_masks(cfg, n, params, b):
    """The kernel's own ReLU pattern for the online network (checked against the f64 forward
    first; flips only where the f64 pre-activation is within fp32 rounding of 0)."""
    B, T = b["action"].shape
    BI = cfg.burn_in_length
    _, cache = O.forward(cfg, params, b, np.float64)
    masks = {}
    names = ["x1", "x2", "x3"] if cfg.torso == "atari" else []
    for name in names:
        ref = cache[name]  # [B*T, ...] batch-major
        per = ref.size // (B * T)
        got = _tm(n.debug_buffer(name)[:ref.size].reshape(B * T, per), B, T).reshape(ref.shape)
        scale = np.abs(ref).max()
        np.testing.assert_allclose(got, ref, rtol=1e-5, atol=2e-6 * scale, err_msg=name)
        m = got > 0
        flips = m != (ref > 0)
        assert (np.abs(ref[flips]) <= 2e-6 * scale).all(), name
        assert flips.mean() < 1e-4, (name, flips.mean())
        masks[name] = m
    ref = cache["hid"].reshape(B, T, -1)
    L = T - BI
    got = _tm(n.debug_buffer("hid")[:L * B * ref.shape[-1]].reshape(L * B, -1), B, L)
    scale = np.abs(ref).max()
    np.testing.assert_allclose(got, ref[:, BI:], rtol=1e-5, atol=2e-6 * scale, err_msg="hid")
    m = ref > 0
    m[:, BI:] = got > 0
    masks["hid"] = m.reshape(B * T, -1)
    return masks


def _compare(cfg, B, T, seed=0, steps=1, f32_engine=False):
    from acme_amd._lib import lib
    from oracle.dqn_oracle import adam_update
    if f32_engine:
        lib().acme_tune_set(b"R2P3", 1)  # read at the learner's creation
    try:
        n = _native(cfg, B, T)
    finally:
        if f32_engine:
            lib().acme_tune_set(b"R2P3", 0)
    p0, t0 = _params(cfg, 10 + seed), _params(cfg, 20 + seed)
    n.set_params(p0, t0)
    z = {k: np.zeros_like(v) for k, v in p0.items()}
    state = dict(params=p0, target=t0, m=z, v=dict(z), num_steps=0)
    BI, A = cfg.burn_in_length, cfg.num_actions
    L = T - BI
    prev_t = None
    for k in range(steps):
        b = _batch(cfg, B, T, 100 * seed + k)
        _run(n, b)
        masks = _relu_masks(cfg, n, state["params"], b)
        ref, _ = O.loss_and_grads(cfg, state["params"], state["target"], b, masks=masks)
        # Network forwards against the f64 restatement.
        q_ref = np.swapaxes(ref["q"][:, BI:], 0, 1).reshape(L * B, A)
        tq_ref = np.swapaxes(ref["target_q"][:, BI:], 0, 1).reshape(L * B, A)
        q_k = n.debug_buffer("q")[:L * B * A]
        tq_k = n.debug_buffer("target_q")[:L * B * A]
        _close(q_k, q_ref, name=f"q step {k}")
        _close(tq_k, tq_ref, name=f"target_q step {k}")
        # The loss kernel bit for bit against TF's f32 loss arithmetic on the kernel's own q
        # values (teacher-forced): errors, priorities, d loss / d q[a].
        err_tf, _ = O.transformed_loss(cfg, q_k.reshape(L, B, A), tq_k.reshape(L, B, A), b)
        np.testing.assert_array_equal(n.errors.cpu().numpy(), err_tf, err_msg=f"errors {k}")
        np.testing.assert_array_equal(n.priorities.cpu().numpy(),
                                      O.compute_priority(err_tf, cfg.max_priority_weight),
                                      err_msg=f"priorities {k}")
        w32 = O.importance_weights(b["probabilities"], cfg.max_replay_size,
                                   cfg.importance_sampling_exponent)
        g_tf = (w32[None, :] * err_tf) * np.float32(1.0 / B)
        g_k = n.debug_buffer("g")[:L * B].reshape(L, B)
        np.testing.assert_array_equal(g_k[:L - 1], g_tf, err_msg=f"g {k}")
        assert not g_k[L - 1].any()
        # End to end against the f64 networks: the f32 value transforms resolve ~6e-5.
        _close(n.errors.cpu().numpy(), ref["errors"], rtol=1e-4, floor=0, name=f"errors {k}")
        np.testing.assert_allclose(n.errors.cpu().numpy(), ref["errors"], atol=2.5e-4)
        np.testing.assert_allclose(n.loss.item(), ref["loss"], rtol=2e-4, err_msg=f"loss {k}")
        # Gradients: the f64 backward from the kernel's d loss / d q (teacher-forced).
        _, cache = O.forward(cfg, state["params"], b, np.float64)
        act = b["action"]
        dq = np.zeros((B, T, A))
        for t in range(L - 1):
            dq[np.arange(B), BI + t, act[:, BI + t]] += g_k[t]
        grads = O.backward(cfg, state["params"], b, cache, dq.reshape(B * T, A), np.float64,
                           masks)
        _check_grads(n, grads)
        got_p = n.get_params("params")
        new_p = {}
        for name in p0:
            new_p[name] = adam_update(state["params"][name], grads[name], state["m"][name],
                                      state["v"][name], k + 1, cfg.learning_rate,
                                      eps=cfg.adam_epsilon)[0]
        _check_params(got_p, new_p, cfg.learning_rate)
        # The target copy: identical to the updated parameters on copy steps, else kept.
        got_t = n.get_params("target")
        for name in got_t:
            want = got_p[name] if k % cfg.target_update_period == 0 else prev_t[name]
            np.testing.assert_array_equal(got_t[name], want, err_msg=name)
        prev_t = got_t
        assert n.num_steps == k + 1
        # Teacher forcing: the next step starts from the kernel's own state.
        shp = {kk: v.shape for kk, v in p0.items()}
        state = dict(params={kk: got_p[kk].reshape(shp[kk]) for kk in p0},
                     target={kk: got_t[kk].reshape(shp[kk]) for kk in p0},
                     m={kk: n.get_params("m")[kk].reshape(shp[kk]) for kk in p0},
                     v={kk: n.get_params("v")[kk].reshape(shp[kk]) for kk in p0},
                     num_steps=k + 1)
    g = n.guard_state()
    assert g["skipped"] == 0 and g["applied"] == steps, g
    return n


def test_r2d2_flat_step_matches_oracle():
    _compare(_cfg(), B=3, T=9, steps=3)


def test_r2d2_no_burn_in_and_zero_state():
    _compare(_cfg(burn_in_length=0, store_lstm_state=False), B=4, T=7, seed=1, steps=2)


def test_r2d2_n_step_longer_than_sequence():
    # Tm = T - burn_in - 1 = 3 < n - 1: only truncated bootstrap steps (r2d2.py:157-159).
    _compare(_cfg(n_step=5, burn_in_length=1), B=2, T=5, seed=2)


def test_r2d2_large_batch_row_chunks():
    # B * (H + 32) floats of h_prev exceed one workgroup's LDS at H = 512: the forward step
    # kernel splits the batch over workgroups (grid.y).
    _compare(_cfg(lstm_size=512, head_size=64, num_actions=18, obs_dim=24), B=80, T=6, seed=3)


@pytest.mark.parametrize("f32_engine", [False, True])
def test_r2d2_atari_step_matches_oracle(f32_engine):
    """R2D2AtariNetwork's sizes (A = 18, LSTM 512, duelling [512]) on uint8 frames: the
    torso and the OAR projection on the two-plane f16 engine (the default: scales calibrated
    on the first step, the step guard) and on f32 MFMA (ACME_V_R2P3=1)."""
    cfg = _cfg(torso="atari", num_actions=18, lstm_size=512, head_size=512, obs_dim=0,
               burn_in_length=2, n_step=2)
    _compare(cfg, B=3, T=6, seed=4, steps=2, f32_engine=f32_engine)


@pytest.mark.parametrize("H,B", [(512, 32), (256, 5)])
def test_r2d2_one_launch_unroll(H, B):
    """The LSTM unroll and BPTT in one launch each (lstm.h lstm_fwd_rg_kernel /
    lstm_bwd_rg_kernel, the default at H = 256 / 512 with <= 256 workgroups; B = 32 at
    H = 512 is the bench's full grid, B = 5 a ragged row group): against the f64 oracle at
    the bars above (two steps, BPTT stopping at the burn-in), then against the per-step
    kernels on the same inputs (the same arithmetic in another summation order: h, q rtol
    1e-5; errors 1e-5 absolute; every gradient within 1e-5 relative Frobenius)."""
    cfg = _cfg(lstm_size=H, head_size=64, num_actions=18, obs_dim=24, burn_in_length=3)
    T = 8
    n = _compare(cfg, B=B, T=T, seed=6, steps=2)
    assert n.debug_buffer("lstm_timeout")[0] == 0
    p0, t0 = _params(cfg, 30), _params(cfg, 31)
    b = _batch(cfg, B, T, 77)
    outs = []
    for per_step in (False, True):
        m = _native(cfg, B, T)
        m.set_lstm_unroll(per_step)
        m.set_params(p0, t0)
        _run(m, b)
        outs.append((m.debug_buffer("h"), m.debug_buffer("q"), m.errors.cpu().numpy().copy(),
                     m.get_params("grads")))
    (h1, q1, e1, g1), (h2, q2, e2, g2) = outs
    np.testing.assert_allclose(h1, h2, rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(q1, q2, rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(e1, e2, rtol=0, atol=1e-5)
    for k in g2:
        den = max(float(np.linalg.norm(g2[k])), 1e-30)
        assert float(np.linalg.norm(g1[k] - g2[k])) <= 1e-5 * den, k


@pytest.mark.parametrize("torso", ["flat", "atari"])
def test_r2d2_lstm_timeout_skips_update(torso):
    """A one-launch LSTM spin timeout (this step's timeout word set before the step, as the
    kernels set it) skips the update on both engines: parameters, Adam moments, Adam's count
    and the target unchanged bit for bit, the loss NaN, the skip counted (pinned host
    mirror, guard state, the sticky timeout count); the next step applies normally."""
    import ctypes

    from acme_amd import _lib
    from acme_amd.native import _memcpy_dtod
    cfg = _cfg(torso=torso, num_actions=18, lstm_size=512, head_size=64,
               obs_dim=0 if torso == "atari" else 24, burn_in_length=2, n_step=2,
               target_update_period=1)
    B, T = 3, 6
    n = _native(cfg, B, T)
    n.set_params(_params(cfg, 40), _params(cfg, 41))
    _run(n, _batch(cfg, B, T, 1))
    assert n.guard_state()["applied"] == 1
    before = {buf: n.get_params(buf) for buf in ("params", "target", "m", "v")}
    p, c = ctypes.c_void_p(), ctypes.c_int64()
    _lib.check(_lib.lib().acme_r2d2_debug_buffer(n._h, b"lstm_timeout_step", ctypes.byref(p),
                                                 ctypes.byref(c)))
    one = torch.ones(1, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    _memcpy_dtod(p.value, one.data_ptr(), 4)
    _run(n, _batch(cfg, B, T, 2))
    assert np.isnan(n.loss.item())
    g = n.guard_state()
    assert g["applied"] == 1 and g["skipped"] == 1 and g["last_skipped"] == 1, g
    assert n.skipped_steps == 1
    assert n.debug_buffer("lstm_timeout").view(np.uint32)[0] == 1
    for buf, ref in before.items():
        got = n.get_params(buf)
        for k in ref:
            np.testing.assert_array_equal(got[k], ref[k], err_msg=f"{buf}/{k}")
    _run(n, _batch(cfg, B, T, 3))
    assert np.isfinite(n.loss.item())
    g = n.guard_state()
    assert g["applied"] == 2 and g["skipped"] == 1 and g["last_skipped"] == 0, g
