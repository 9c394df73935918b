"""JAX learner semantics on the HIP learners.

References: acme/agents/jax/dqn/learning.py:74-178 (f32 importance weights :94-96, target
copy at (steps + 1) % period :114-119, optix.adam agents/jax/dqn/agent.py:110) and
acme/agents/jax/impala/learning.py:66-136 with optix.chain(clip_by_global_norm, adam)
(agents/jax/impala/agent.py:98-101).  Oracle: oracle/dqn_oracle.py and
oracle/impala_oracle.py with semantics="jax".  Tolerances as tests/test_dqn_gpu.py and
tests/test_impala_gpu.py (fp32 kernels vs the f64 restatement; Adam on identical gradients
rtol 1e-6).
"""

import numpy as np
import pytest
import torch

from oracle import dqn_oracle as O
from oracle import impala_oracle as OI
from tests import test_dqn_gpu as TD
from tests import test_impala_gpu as TI

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("netname,B", [("nature", 37), ("cartpole_mlp", 32), ("nature", 512)])
def test_jax_dqn_forward_backward_matches_oracle(netname, B):
    net = TD.NETS[netname]()
    rng = np.random.default_rng(B + 7)
    params, target = net.init(seed=1), net.init(seed=2)
    # probabilities spanning six decades: the f32 weights differ from the f64 ones here.
    probs = 10.0 ** rng.uniform(-9, -3, B)
    batch = TD._batch(rng, B, net.obs_shape, net.num_actions, u8=net.obs_dtype == "uint8",
                      probs=probs)
    d = TD._learner(net, B, semantics="jax")
    d.set_params(params, target)
    q = torch.empty(B, net.num_actions, device="cuda")
    d.forward_backward(*TD._dev(batch), q_tm1=q)
    torch.cuda.synchronize()
    masks = TD._relu_masks(d, net, batch, params, B)
    out, grads = O.dqn_loss_and_grads(TD._cfg(net, semantics="jax"), params, target, batch,
                                      np.float64, masks=masks)
    np.testing.assert_allclose(d.loss.item(), out["loss"], rtol=1e-5)
    np.testing.assert_allclose(d.td_error[:B].cpu().numpy(), out["td_error"], rtol=1e-5,
                               atol=1e-6)
    np.testing.assert_allclose(d.priorities[:B].cpu().numpy(), out["priorities"], rtol=1e-5,
                               atol=1e-6)
    TD._check_grads(d.get_params("grads"), grads)


def test_jax_dqn_optix_adam_and_target_cadence():
    """optix.adam on the kernel's own gradients, and the target copied after steps 1 and 3
    ((steps + 1) % 2 == 0), never at step 0 (the TF learner copies at steps 0 and 2)."""
    from acme_amd.networks import MLP
    net = MLP(4, [50, 50], 2)
    B = 32
    rng = np.random.default_rng(0)
    p0, t0 = net.init(seed=3), net.init(seed=4)
    d = TD._learner(net, B, target_update_period=2, learning_rate=1e-3, semantics="jax")
    d.set_params(p0, t0)
    m = {k: np.zeros_like(v) for k, v in p0.items()}
    v = {k: np.zeros_like(v) for k, v in p0.items()}
    params, target = p0, t0
    for step in range(4):
        batch = TD._batch(rng, B, net.obs_shape, net.num_actions, u8=False)
        d.forward_backward(*TD._dev(batch))
        g = d.get_params("grads")
        d.apply()
        torch.cuda.synchronize()
        newp = {}
        for k in params:
            newp[k], m[k], v[k] = O.adam_update(params[k], g[k], m[k], v[k], step + 1, 1e-3,
                                                optix=True)
        got = d.get_params("params")
        for k in newp:
            np.testing.assert_allclose(got[k], newp[k], rtol=1e-6, atol=1e-9)
        params = got
        if (step + 1) % 2 == 0:
            target = got
        tg = d.get_params("target")
        for k in target:
            np.testing.assert_array_equal(tg[k], target[k])
        assert d.num_steps == step + 1


def test_jax_dqn_nature_trajectory_matches_oracle():
    """Three Nature-CNN steps at B = 16, target period 2 (the JAX copy lands after step 1,
    never at step 0), teacher-forced: each step against the f64 JAX oracle from the kernel's
    own pre-step state, conditional on its ReLU pattern (a kink flip between fp32 and fp64
    would otherwise change a conv gradient by tens of percent, tests/test_dqn_gpu.py), and
    optix.adam on the kernel's gradients (tolerances of tests/test_dqn_headline_gpu.py)."""
    from acme_amd.networks import DQNAtariNetwork
    net = DQNAtariNetwork(18)
    B, lr = 16, 1e-3
    rng = np.random.default_rng(21)
    d = TD._learner(net, B, target_update_period=2, semantics="jax")
    d.set_params(net.init(seed=5), net.init(seed=6))
    cfg = TD._cfg(net, target_update_period=2, semantics="jax")
    for i in range(3):
        batch = TD._batch(rng, B, net.obs_shape, net.num_actions)
        pre = {w: d.get_params(w) for w in ("params", "target", "m", "v")}
        d.step(*TD._dev(batch))
        torch.cuda.synchronize()
        masks = TD._relu_masks(d, net, batch, pre["params"], B)
        out, grads = O.dqn_loss_and_grads(cfg, pre["params"], pre["target"], batch, np.float64,
                                          masks=masks)
        np.testing.assert_allclose(d.loss.item(), out["loss"], rtol=1e-5)
        g = d.get_params("grads")
        TD._check_grads(g, grads)
        post = {w: d.get_params(w) for w in ("params", "target", "m", "v")}
        t = i + 1
        for k in pre["params"]:
            p1, m1, v1 = O.adam_update(pre["params"][k], g[k], pre["m"][k], pre["v"][k], t, lr,
                                       optix=True)
            m_terms = 0.9 * np.abs(pre["m"][k]) + 0.1 * np.abs(g[k])
            assert (np.abs(post["m"][k] - m1) <= 1e-6 * m_terms + 1e-30).all(), k
            np.testing.assert_allclose(post["v"][k], v1, rtol=1e-6, atol=1e-30)
            vhat = np.asarray(v1, np.float64) / (1 - 0.999 ** t)
            upd_terms = lr * (m_terms / (1 - 0.9 ** t)) / (np.sqrt(vhat) + 1e-8)
            p_terms = np.abs(pre["params"][k]) + upd_terms
            assert (np.abs(post["params"][k] - p1) <= 1e-6 * p_terms + 1e-30).all(), k
            want = post["params"][k] if (i + 1) % 2 == 0 else pre["target"][k]
            np.testing.assert_array_equal(post["target"][k], want)
        assert d.num_steps == i + 1


def test_jax_dqn_learner_drop_in():
    """acme_amd.agents.jax.dqn.DQNLearner: the reference constructor (network, obs_spec, ...,
    iterator, optimizer=optix.adam, rng), separate target init, counts-only logging,
    priorities written back, get_variables -> [params]."""
    from acme_amd import replay, specs
    from acme_amd.adders import reverb as adders
    from acme_amd.agents.jax.dqn import DQNLearner
    from acme_amd.datasets import make_reverb_dataset
    from acme_amd.networks import MLP
    from acme_amd.optimizers import optix
    from acme_amd.utils import loggers
    env_spec = specs.EnvironmentSpec(
        observations=specs.Array((4,), np.float32), actions=specs.DiscreteArray(2, np.int32),
        rewards=specs.Array((), np.float32), discounts=specs.BoundedArray((), np.float32, 0, 1))
    table = replay.Table(adders.DEFAULT_PRIORITY_TABLE, replay.selectors.Prioritized(0.6),
                         replay.selectors.Fifo(), 1000, replay.rate_limiters.MinSize(1),
                         signature=adders.NStepTransitionAdder.signature(env_spec),
                         device=torch.device("cuda"))
    rng = np.random.default_rng(0)
    for i in range(300):
        table.insert((rng.standard_normal(4).astype(np.float32), np.int32(i % 2),
                      np.float32(rng.standard_normal()), np.float32(0.99),
                      rng.standard_normal(4).astype(np.float32)), 1.0)
    server = replay.Server([table])
    it = iter(make_reverb_dataset(server, batch_size=32))

    class Rec(loggers.Logger):
        def __init__(self):
            self.rows = []

        def write(self, data):
            self.rows.append(dict(data))

        def close(self):
            pass

    log = Rec()
    net = MLP(4, [50, 50], 2)
    learner = DQNLearner(net, env_spec.observations, discount=0.99,
                         importance_sampling_exponent=0.2, target_update_period=2,
                         iterator=it, optimizer=optix.adam(1e-3), rng=7,
                         replay_client=replay.Client(server), logger=log)
    n = learner.native
    assert n.semantics == "jax"
    p, t = n.get_params("params"), n.get_params("target")
    assert any(not np.array_equal(p[k], t[k]) for k in p)  # separate keys (:148-151)
    prio_before = table.native.debug_state()["raw"][:300].copy()
    for _ in range(3):
        learner.step()
    torch.cuda.synchronize()
    assert learner.num_steps == 3
    assert all("loss" not in r for r in log.rows) and log.rows[-1]["steps"] == 3
    assert not np.array_equal(table.native.debug_state()["raw"][:300], prio_before)
    (params,) = learner.get_variables([""])
    assert set(params) == set(n.get_params("params"))


@pytest.mark.parametrize("clip", [None, 0.05])
def test_jax_impala_step_matches_oracle(clip):
    """Flat-torso IMPALA (LSTM 16, T = 6, B = 4) with the optix chain: no clipping (the JAX
    agent's default max_gradient_norm = inf) and a norm small enough to clip."""
    cfg = OI.IMPALAConfig(num_actions=5, torso="flat", obs_dim=12, lstm_size=16, head_size=8,
                          entropy_cost=0.01, baseline_cost=0.5, semantics="jax",
                          max_gradient_norm=float("inf") if clip is None else clip)
    B, T = 4, 6
    n = TI._native(cfg, B, T, semantics="jax", max_gradient_norm=clip)
    params = TI._params(cfg, 1)
    n.set_params(params)
    b = TI._batch(cfg, B, T, 2)
    TI._run(n, b)
    TI._compare(cfg, n, params, b)
    G = n.debug_buffer("grad_norm")[0]
    if clip is not None:
        assert G > clip  # the clip branch was taken
