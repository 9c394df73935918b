"""IMPALA drop-in path on the GPU: the queue table + SequenceAdder + dataset feeding
IMPALALearner.step() (loss checked against the oracle on the very sequences the adder
wrote), and the IMPALA agent running in the EnvironmentLoop behind
ObservationActionRewardWrapper (acme/agents/tf/impala/agent_test.py:31-60 analogue)."""

import numpy as np
import pytest
import torch

from acme_amd import specs
from acme_amd.environment_loop import EnvironmentLoop
from acme_amd.testing import fakes
from acme_amd.utils import loggers
from acme_amd.wrappers import ObservationActionRewardWrapper
from oracle import impala_oracle as O

pytestmark = pytest.mark.gpu


def test_learner_step_through_queue_matches_oracle():
    from acme_amd import datasets, replay
    from acme_amd.adders import reverb as adders
    from acme_amd.agents.impala import IMPALALearner
    from acme_amd.networks import IMPALAAtariNetwork, LSTMState
    from acme_amd.wrappers import OAR
    A, H, T, B, obs_dim = 3, 16, 4, 5, 6
    net = IMPALAAtariNetwork(A, lstm_size=H, head_size=8, torso="flat", obs_dim=obs_dim)
    env = ObservationActionRewardWrapper(fakes.DiscreteEnvironment(num_actions=A,
                                                                   obs_shape=(obs_dim,)))
    spec = specs.make_environment_spec(env)
    extra = {"core_state": LSTMState(specs.Array((H,), np.float32), specs.Array((H,), np.float32)),
             "logits": specs.Array((A,), np.float32)}
    queue = replay.Table.queue(adders.DEFAULT_PRIORITY_TABLE, 100,
                               signature=adders.SequenceAdder.signature(spec, extras_spec=extra))
    server = replay.Server([queue])
    rng = np.random.default_rng(0)
    items = []
    writer = replay.Client(server).writer(T)
    for _ in range(B):
        for t in range(T):
            step = adders.Step(
                observation=OAR(rng.standard_normal(obs_dim).astype(np.float32),
                                np.int32(rng.integers(A)), np.float32(rng.standard_normal())),
                action=np.int32(rng.integers(A)), reward=np.float32(rng.standard_normal()),
                discount=np.float32(rng.choice([0.0, 1.0], p=[0.2, 0.8])),
                start_of_episode=np.bool_(t == 0),
                extras={"core_state": LSTMState(rng.standard_normal(H).astype(np.float32),
                                                rng.standard_normal(H).astype(np.float32)),
                        "logits": rng.standard_normal(A).astype(np.float32)})
            items.append(step)
            writer.append(step)
        writer.create_item(adders.DEFAULT_PRIORITY_TABLE, T, 1.0)
    ds = datasets.make_reverb_dataset(server_address=server, batch_size=B, sequence_length=T)
    learner = IMPALALearner(spec, net, ds, learning_rate=1e-3, entropy_cost=0.01,
                            baseline_cost=0.5, logger=loggers.NoOpLogger(), batch_size=B,
                            sequence_length=T, seed=3)
    params = learner.native.get_params("params")
    learner.step()
    torch.cuda.synchronize()
    st = lambda f: np.stack([f(s) for s in items]).reshape((B, T) + np.shape(f(items[0])))  # noqa
    batch = dict(obs=st(lambda s: s.observation.observation),
                 prev_action=st(lambda s: s.observation.action),
                 prev_reward=st(lambda s: s.observation.reward), action=st(lambda s: s.action),
                 reward=st(lambda s: s.reward), discount=st(lambda s: s.discount),
                 behaviour_logits=st(lambda s: s.extras["logits"]),
                 h0=st(lambda s: s.extras["core_state"].hidden)[:, 0],
                 c0=st(lambda s: s.extras["core_state"].cell)[:, 0])
    cfg = O.IMPALAConfig(num_actions=A, torso="flat", obs_dim=obs_dim, lstm_size=H, head_size=8,
                         entropy_cost=0.01, baseline_cost=0.5)
    ref, _ = O.loss_and_grads(cfg, params, batch, np.float64)
    np.testing.assert_allclose(learner.native.metrics[0].item(), ref["loss"], rtol=1e-5)
    assert learner.num_steps == 1
    assert queue.size() == 0  # consumed once


def test_impala_agent_runs_in_environment_loop():
    from acme_amd.agents.impala import IMPALA
    from acme_amd.networks import IMPALAAtariNetwork
    env = ObservationActionRewardWrapper(fakes.DiscreteEnvironment(num_actions=3, obs_shape=(5,),
                                                                   episode_length=10))
    spec = specs.make_environment_spec(env)
    net = IMPALAAtariNetwork(3, lstm_size=16, head_size=8, torso="flat", obs_dim=5)
    agent = IMPALA(spec, net, sequence_length=4, sequence_period=4, batch_size=2,
                   logger=loggers.NoOpLogger())
    loop = EnvironmentLoop(env, agent, logger=loggers.NoOpLogger())
    loop.run(num_episodes=4)
    learner = agent._learner  # noqa: SLF001
    assert learner.num_steps >= 1
    assert np.isfinite(learner.native.metrics.cpu().numpy()).all()


def test_actor_pool_feeds_device_queue_learner():
    """BASELINE configs[3] shape end to end at small scale: 6 actor threads (Atari-shaped
    environments, IMPALAActor, SequenceAdder) with batched GPU policy steps on the learner's
    parameters feed the device queue; the learner steps whenever a batch is queued."""
    import time
    from acme_amd import datasets, replay
    from acme_amd.adders import reverb as adders
    from acme_amd.agents.impala import IMPALALearner
    from acme_amd.agents.impala.actors import ActorPool, BatchedPolicy
    from acme_amd.environments.atari_like import AtariLike
    from acme_amd.networks import IMPALAAtariNetwork, LSTMState
    A, H, T, B = 18, 32, 5, 4
    env = ObservationActionRewardWrapper(AtariLike(seed=0, min_length=7, max_length=30))
    spec = specs.make_environment_spec(env)
    extra = {"core_state": LSTMState(specs.Array((H,), np.float32), specs.Array((H,), np.float32)),
             "logits": specs.Array((A,), np.float32)}
    queue = replay.Table.queue(adders.DEFAULT_PRIORITY_TABLE, 16,
                               signature=adders.SequenceAdder.signature(spec, extras_spec=extra))
    server = replay.Server([queue])
    net = IMPALAAtariNetwork(A, lstm_size=H, head_size=16)
    learner = IMPALALearner(spec, net, datasets.make_reverb_dataset(server, batch_size=B,
                                                                    sequence_length=T),
                            learning_rate=1e-3, entropy_cost=0.01, baseline_cost=0.5,
                            logger=loggers.NoOpLogger(), batch_size=B, sequence_length=T)
    policy = BatchedPolicy(learner.actor_policy(max_rows=4), max_rows=4)
    pool = ActorPool(lambda i: ObservationActionRewardWrapper(
                         AtariLike(seed=10 + i, min_length=7, max_length=30)),
                     lambda i: adders.SequenceAdder(replay.Client(server), sequence_length=T,
                                                    period=T),
                     policy, net.initial_state, num_actors=6)
    pool.start()
    try:
        deadline = time.time() + 120
        while learner.num_steps < 5 and time.time() < deadline:
            assert not pool.errors, pool.errors
            if queue.can_sample(B):
                learner.step()
            else:
                time.sleep(0.001)
    finally:
        pool.stop(timeout=10)
        policy.close()
    torch.cuda.synchronize()
    assert learner.num_steps >= 5
    assert pool.env_steps >= 5 * B * T
    assert policy.batches > 0 and policy.rows >= pool.env_steps
    assert np.isfinite(learner.native.metrics.cpu().numpy()).all()


def test_vector_actor_pool_feeds_device_queue_learner():
    """The same with VectorActorPool: 2 host threads x 3 environments, one policy call per
    thread step on the learner's parameters (chunks of 2 rows), into the device queue."""
    import time
    from acme_amd import datasets, replay
    from acme_amd.adders import reverb as adders
    from acme_amd.agents.impala import IMPALALearner
    from acme_amd.agents.impala.actors import VectorActorPool
    from acme_amd.environments.atari_like import AtariLike
    from acme_amd.networks import IMPALAAtariNetwork, LSTMState
    A, H, T, B = 18, 32, 5, 4
    env = ObservationActionRewardWrapper(AtariLike(seed=0, min_length=7, max_length=30))
    spec = specs.make_environment_spec(env)
    extra = {"core_state": LSTMState(specs.Array((H,), np.float32), specs.Array((H,), np.float32)),
             "logits": specs.Array((A,), np.float32)}
    queue = replay.Table.queue(adders.DEFAULT_PRIORITY_TABLE, 16,
                               signature=adders.SequenceAdder.signature(spec, extras_spec=extra))
    server = replay.Server([queue])
    net = IMPALAAtariNetwork(A, lstm_size=H, head_size=16)
    learner = IMPALALearner(spec, net, datasets.make_reverb_dataset(server, batch_size=B,
                                                                    sequence_length=T),
                            learning_rate=1e-3, entropy_cost=0.01, baseline_cost=0.5,
                            logger=loggers.NoOpLogger(), batch_size=B, sequence_length=T)
    pool = VectorActorPool(lambda i: ObservationActionRewardWrapper(
                               AtariLike(seed=10 + i, min_length=7, max_length=30)),
                           lambda i: adders.SequenceAdder(replay.Client(server), sequence_length=T,
                                                          period=T),
                           lambda t: learner.actor_policy(max_rows=2), net.initial_state,
                           num_actors=6, threads=2, max_rows=2)
    pool.start()
    try:
        deadline = time.time() + 120
        while learner.num_steps < 5 and time.time() < deadline:
            assert not pool.errors, pool.errors
            if queue.can_sample(B):
                learner.step()
            else:
                time.sleep(0.001)
    finally:
        pool.stop(timeout=10)
    torch.cuda.synchronize()
    assert not pool.errors, pool.errors
    assert learner.num_steps >= 5
    assert pool.env_steps >= 5 * B * T
    assert np.isfinite(learner.native.metrics.cpu().numpy()).all()


@pytest.mark.parametrize("rows", [5, 64])
def test_pipelined_policy_equals_actor_policy(rows):
    """IMPALALearner.pipelined_policy (the process pool's policy: packed transfers, a
    page-locked observation source, issue / result) returns exactly actor_policy's
    logits, values and LSTM state for the same inputs, at 64 rows on the one-launch LSTM
    step too; and two calls in flight on their own policies do not disturb each other."""
    import ctypes
    from acme_amd import _lib
    from acme_amd.agents.impala import IMPALALearner
    from acme_amd.networks import IMPALAAtariNetwork
    A, H = 18, 256
    net = IMPALAAtariNetwork(A, lstm_size=H, head_size=256)
    learner = IMPALALearner(None, net, iter(()), learning_rate=1e-3,
                            logger=loggers.NoOpLogger(), batch_size=2, sequence_length=4)
    rng = np.random.default_rng(rows)
    ins = [(rng.integers(0, 256, (rows, 84, 84, 4), dtype=np.uint8),
            rng.integers(0, A, rows).astype(np.int32), rng.standard_normal(rows).astype(np.float32),
            (0.3 * rng.standard_normal((rows, H))).astype(np.float32),
            (0.3 * rng.standard_normal((rows, H))).astype(np.float32)) for _ in range(2)]
    ref = [learner.actor_policy(max_rows=rows)(*x) for x in ins]
    pols = [learner.pipelined_policy(rows) for _ in range(2)]
    # The first call's observations from page-locked memory, the second's staged.
    obs0 = np.empty_like(ins[0][0])
    obs0[...] = ins[0][0]
    L = _lib.lib()
    _lib.check(L.acme_host_register(ctypes.c_void_p(obs0.ctypes.data), obs0.nbytes))
    try:
        pols[0].issue(obs0, *ins[0][1:], observation_pinned=True)
        pols[1].issue(*ins[1])
        got = [pols[0].result(), pols[1].result()]
    finally:
        L.acme_host_unregister(ctypes.c_void_p(obs0.ctypes.data))
    for g, r in zip(got, ref):
        for a, b in zip(g, r):
            np.testing.assert_array_equal(a, b)
