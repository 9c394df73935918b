"""The R2D2 learner oracle (oracle/r2d2_oracle.py) checked on its own, on the CPU.

Parity with TF is UNPINNED (no reference test holds an R2D2 learner value, SURVEY.md
§8(c)); these pin the restatement's internal consistency:
  * gradients = central finite differences of the loss (burn_in = 0, where the whole
    unroll is inside the tape);
  * the burn-in stops the gradient (learning.py:134-137): the step with burn_in = k equals
    the step with burn_in = 0 on the sequences' suffix started from the burn-in's state;
  * the n-step targets (losses/r2d2.py:122-169) equal their closed form
    sum_i (prod_{j<i} pcont) r + (prod pcont) bootstrap[min(t + n - 1, T - 1)];
  * signed_parabolic inverts signed_hyperbolic (losses/r2d2.py:172-180).
"""

import numpy as np

from oracle import r2d2_oracle as O


def _cfg(**kw):
    base = dict(num_actions=5, torso="flat", obs_dim=12, lstm_size=16, head_size=8,
                burn_in_length=0, n_step=3, max_replay_size=100)
    base.update(kw)
    return O.R2D2Config(**base)


def _batch(B, T, seed, H=16, obs_dim=12, A=5):
    rng = np.random.default_rng(seed)
    return dict(obs=rng.standard_normal((B, T, obs_dim)),
                action=rng.integers(0, A, (B, T)).astype(np.int32),
                prev_action=rng.integers(0, A, (B, T)).astype(np.int32),
                prev_reward=rng.standard_normal((B, T)),
                reward=rng.standard_normal((B, T)),
                discount=(rng.random((B, T)) > 0.1).astype(np.float64),
                h0=0.3 * rng.standard_normal((B, H)), c0=0.3 * rng.standard_normal((B, H)),
                probabilities=rng.random(B) * 0.1 + 0.01)


def _f64(p):
    return {k: v.astype(np.float64) for k, v in p.items()}


def test_gradients_match_finite_differences():
    cfg = _cfg()
    b = _batch(3, 8, 0)
    p, tg = _f64(O.init_params(cfg, 0)), _f64(O.init_params(cfg, 1))
    _, g = O.loss_and_grads(cfg, p, tg, b, loss_dtype=np.float64)
    rng = np.random.default_rng(5)
    for name in p:
        for _ in range(3):
            idx = tuple(int(rng.integers(0, s)) for s in p[name].shape)
            e = 1e-6
            pp = {k: v.copy() for k, v in p.items()}
            pp[name][idx] += e
            lp = O.loss_and_grads(cfg, pp, tg, b, loss_dtype=np.float64)[0]["loss"]
            pp[name][idx] -= 2 * e
            lm = O.loss_and_grads(cfg, pp, tg, b, loss_dtype=np.float64)[0]["loss"]
            fd = (lp - lm) / (2 * e)
            assert abs(fd - g[name][idx]) <= 1e-6 + 1e-5 * abs(fd), (name, idx, fd, g[name][idx])


def test_burn_in_stops_the_gradient():
    BI, B, T = 3, 3, 10
    cfg = _cfg(burn_in_length=BI)
    b = _batch(B, T, 1)
    p, tg = _f64(O.init_params(cfg, 2)), _f64(O.init_params(cfg, 3))
    out, g = O.loss_and_grads(cfg, p, tg, b, loss_dtype=np.float64)
    # The suffix as its own batch, from the burn-in's states of each network.  The online
    # and target burn-ins end in different states, so the suffix step is split: the online
    # unroll from the online state, the target's from the target state.
    _, c_on = O.forward(cfg, p, b, np.float64)
    _, c_tg = O.forward(cfg, tg, b, np.float64)
    sl = {k: (v[:, BI:] if k not in ("h0", "c0", "probabilities") else v) for k, v in b.items()}
    s_on = dict(sl, h0=c_on["hs"][:, BI - 1], c0=c_on["cs"][:, BI - 1])
    s_tg = dict(sl, h0=c_tg["hs"][:, BI - 1], c0=c_tg["cs"][:, BI - 1])
    cfg0 = _cfg(burn_in_length=0)
    q_tg, _ = O.forward(cfg0, tg, s_tg, np.float64)
    q_on, _ = O.forward(cfg0, p, s_on, np.float64)
    np.testing.assert_allclose(q_on, out["q"][:, BI:], rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(q_tg, out["target_q"][:, BI:], rtol=1e-12, atol=1e-12)

    # Same step with the target network's suffix q forced: run the burn_in = 0 oracle with
    # a target whose unroll starts at the target's burn-in state (the loss only reads q_tg).
    orig = O.forward

    def fwd(c, params, batch, dtype):
        if params is tg:
            return orig(c, params, s_tg, dtype)
        return orig(c, params, batch, dtype)

    O.forward = fwd
    try:
        out0, g0 = O.loss_and_grads(cfg0, p, tg, s_on, loss_dtype=np.float64)
    finally:
        O.forward = orig
    np.testing.assert_allclose(out0["loss"], out["loss"], rtol=1e-12)
    np.testing.assert_allclose(out0["errors"], out["errors"], rtol=1e-10, atol=1e-12)
    for k in g:
        np.testing.assert_allclose(g0[k], g[k], rtol=1e-9, atol=1e-12, err_msg=k)


def test_n_step_targets_closed_form():
    rng = np.random.default_rng(3)
    for T, n in ((9, 3), (4, 5), (6, 1), (5, 5)):
        B = 2
        r = rng.standard_normal((T, B))
        pc = rng.random((T, B))
        boot = rng.standard_normal((T, B))
        got = O.n_step_targets(r, pc, boot, n)
        want = np.zeros((T, B))
        for t in range(T):
            acc, disc = 0.0, np.ones(B)
            for i in range(n):
                k = t + i
                if k < T:
                    acc = acc + disc * r[k]
                    disc = disc * pc[k]
            want[t] = acc + disc * boot[min(t + n - 1, T - 1)]
        np.testing.assert_allclose(got, want, rtol=1e-12, atol=1e-12, err_msg=f"T={T} n={n}")


def test_f32_transforms_follow_tf_rounding():
    """The float32 restatements round like the f64 transforms up to their f32 resolution
    (ulp(512) = 6.1e-5 absolute for h^-1 near 0, relative 2^-23 scale elsewhere)."""
    x = np.linspace(-50, 50, 4001).astype(np.float32)
    p32 = O.signed_parabolic_f32(x).astype(np.float64)
    p64 = O.signed_parabolic(x.astype(np.float64))
    assert np.all(np.abs(p32 - p64) <= 1.3e-4 * (1 + np.abs(p64)))
    h32 = O.signed_hyperbolic_f32(x).astype(np.float64)
    h64 = O.signed_hyperbolic(x.astype(np.float64))
    assert np.all(np.abs(h32 - h64) <= 1e-6 * (1 + np.abs(h64)))


def test_value_transforms_invert():
    x = np.concatenate([np.linspace(-1000, 1000, 2001), [0.0, 1e-6, -1e-6]])
    np.testing.assert_allclose(O.signed_parabolic(O.signed_hyperbolic(x)), x, rtol=1e-9,
                               atol=1e-9)
    np.testing.assert_allclose(O.signed_hyperbolic(O.signed_parabolic(x)), x, rtol=1e-9,
                               atol=1e-9)
