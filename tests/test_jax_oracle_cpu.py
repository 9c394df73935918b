"""CPU checks of the oracles' JAX-learner modes.

acme/agents/jax/dqn/learning.py:94-96 (f32 importance weights), :114-119 with
acme/jax/utils.py:148-154 (target copy at (steps + 1) % period), optix.adam; optix
clip_by_global_norm (acme/agents/jax/impala/agent.py:98-101).
"""

import numpy as np

from oracle import dqn_oracle as O
from oracle import impala_oracle as OI


def _mlp_state(seed=0):
    from acme_amd.networks import MLP
    net = MLP(4, [8], 2)
    p, t = net.init(seed), net.init(seed + 1)
    z = {k: np.zeros_like(v) for k, v in p.items()}
    return net, dict(params=p, target=t, m=z, v=dict(z), num_steps=0)


def _batch(rng, B):
    return dict(o_tm1=rng.standard_normal((B, 4)).astype(np.float32),
                a_tm1=rng.integers(0, 2, B).astype(np.int32),
                r_t=rng.standard_normal(B).astype(np.float32),
                d_t=np.full(B, 0.99, np.float32),
                o_t=rng.standard_normal((B, 4)).astype(np.float32),
                probabilities=10.0 ** rng.uniform(-9, -2, B))


def test_target_cadence_tf_vs_jax():
    rng = np.random.default_rng(0)
    batches = [_batch(rng, 16) for _ in range(5)]
    for sem, copies in (("tf", {0, 2, 4}), ("jax", {1, 3})):
        net, st = _mlp_state()
        cfg = O.DQNConfig(num_actions=2, network="mlp", obs_dim=4, hidden=(8,),
                          target_update_period=2, semantics=sem)
        for i, b in enumerate(batches):
            before = {k: v.copy() for k, v in st["target"].items()}
            _, _, st = O.dqn_step(cfg, st, b, np.float64)
            copied = all(np.array_equal(st["target"][k], st["params"][k]) for k in before)
            assert copied == (i in copies), (sem, i)
            assert st["num_steps"] == i + 1


def test_importance_weights_f32_vs_f64():
    rng = np.random.default_rng(1)
    net, st = _mlp_state()
    b = _batch(rng, 64)
    outs = {}
    for sem in ("tf", "jax"):
        cfg = O.DQNConfig(num_actions=2, network="mlp", obs_dim=4, hidden=(8,), semantics=sem)
        outs[sem], _ = O.dqn_loss_and_grads(cfg, st["params"], st["target"], b, np.float64)
    w_tf, w_jax = outs["tf"]["importance_weights"], outs["jax"]["importance_weights"]
    beta = np.float32(0.2)
    inv = (1.0 / b["probabilities"]).astype(np.float32)
    expect = (inv ** beta) / (inv ** beta).max()
    np.testing.assert_array_equal(w_jax, expect.astype(np.float64))
    assert w_jax.max() == 1.0 and w_tf.max() == 1.0
    np.testing.assert_allclose(w_jax, w_tf, rtol=1e-6)


def test_optix_adam_form():
    rng = np.random.default_rng(2)
    p, g = rng.standard_normal(1000).astype(np.float32), rng.standard_normal(1000).astype(np.float32)
    z = np.zeros(1000, np.float32)
    a, _, _ = O.adam_update(p, g, z, z, 1, 1e-3)
    b, _, _ = O.adam_update(p, g, z, z, 1, 1e-3, optix=True)
    np.testing.assert_allclose(a, b, rtol=1e-6)
    f = np.float32
    b1, b2 = f(0.9), f(0.999)
    mh = (b1 * z + (f(1) - b1) * g) / (f(1) - np.power(b1, f(1)))
    vh = (b2 * z + (f(1) - b2) * (g * g)) / (f(1) - np.power(b2, f(1)))
    np.testing.assert_array_equal(b, p - f(1e-3) * (mh / (np.sqrt(vh) + f(1e-8))))


def test_optix_clip_by_global_norm():
    rng = np.random.default_rng(3)
    g = {"a": rng.standard_normal(10).astype(np.float32),
         "b": rng.standard_normal((3, 4)).astype(np.float32)}
    G = np.sqrt(sum(float(np.sum(x.astype(np.float64) ** 2)) for x in g.values()))
    same, G1 = OI.clip_by_global_norm(g, 2 * G, np.float32, optix=True)
    assert G1 == G and all(np.array_equal(same[k], g[k]) for k in g)
    clipped, _ = OI.clip_by_global_norm(g, G / 4, np.float32, optix=True)
    tf, _ = OI.clip_by_global_norm(g, G / 4, np.float32)
    for k in g:
        np.testing.assert_array_equal(clipped[k], (g[k] / np.float32(G)) * np.float32(G / 4))
        np.testing.assert_allclose(clipped[k], tf[k], rtol=1e-6)
    inf, _ = OI.clip_by_global_norm(g, np.inf, np.float32, optix=True)
    assert all(np.array_equal(inf[k], g[k]) for k in g)
