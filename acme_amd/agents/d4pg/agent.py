"""D4PG agent — drop-in for acme/agents/tf/d4pg/agent.py:37-180.

Same constructor (environment_spec, policy_network, critic_network,
observation_network=identity, discount=0.99, batch_size=256, prefetch_size=4,
target_update_period=100, policy_optimizer=None, critic_optimizer=None,
min_replay_size=1000, max_replay_size=1e6, samples_per_insert=32.0, n_step=5, sigma=0.3,
clipping=True, logger=None, counter=None, checkpoint=True, replay_table_name).  Uniform
GPU replay table instead of a Reverb server; the behaviour policy is the learner's online
policy + ClippedGaussian(sigma) + ClipToSpec (agent.py:132-138, tf/networks/noise.py:27-40,
rescaling.py:28-37)."""

from __future__ import annotations

import copy
from typing import Optional

import numpy as np

from acme_amd import datasets, replay, specs
from acme_amd.adders import reverb as adders
from acme_amd.agents import agent
from acme_amd.agents.actors import FeedForwardActor
from acme_amd.agents.d4pg import learning


class GaussianBehaviourPolicy:
    """a = clip_to_spec(clip(policy(o) + N(0, sigma), -1, 1))."""

    def __init__(self, policy_fn, sigma: float, minimum, maximum, seed: int = 0):
        self._policy = policy_fn
        self._sigma = float(sigma)
        self._min = np.asarray(minimum, np.float32)
        self._max = np.asarray(maximum, np.float32)
        self._rng = np.random.default_rng(seed)

    def __call__(self, batched_obs):
        a = np.asarray(self._policy(batched_obs), np.float32)
        a = np.clip(a + self._rng.normal(0.0, self._sigma, a.shape).astype(np.float32), -1.0, 1.0)
        return np.clip(a, self._min, self._max)


class D4PG(agent.Agent):

    def __init__(self, environment_spec: specs.EnvironmentSpec, policy_network, critic_network,
                 observation_network="identity", discount: float = 0.99, batch_size: int = 256,
                 prefetch_size: int = 4, target_update_period: int = 100,
                 policy_optimizer=None, critic_optimizer=None, min_replay_size: int = 1000,
                 max_replay_size: int = 1000000, samples_per_insert: float = 32.0,
                 n_step: int = 5, sigma: float = 0.3, clipping: bool = True, logger=None,
                 counter=None, checkpoint: bool = True,
                 replay_table_name: str = adders.DEFAULT_PRIORITY_TABLE, seed: int = 0):
        table = replay.Table(
            name=replay_table_name, sampler=replay.selectors.Uniform(),
            remover=replay.selectors.Fifo(), max_size=max_replay_size,
            rate_limiter=replay.rate_limiters.MinSize(1),
            signature=adders.NStepTransitionAdder.signature(environment_spec), seed=4321 + seed)
        self._server = replay.Server([table], port=None)
        address = f"localhost:{self._server.port}"
        adder = adders.NStepTransitionAdder(priority_fns={replay_table_name: lambda x: 1.},
                                            client=replay.Client(address), n_step=n_step,
                                            discount=discount)
        dataset = datasets.make_reverb_dataset(table=replay_table_name, server_address=address,
                                               batch_size=batch_size,
                                               prefetch_size=prefetch_size)
        learner = learning.D4PGLearner(
            policy_network=policy_network, critic_network=critic_network,
            target_policy_network=copy.deepcopy(policy_network),
            target_critic_network=copy.deepcopy(critic_network),
            observation_network=observation_network,
            target_observation_network=observation_network,
            policy_optimizer=policy_optimizer, critic_optimizer=critic_optimizer,
            clipping=clipping, discount=discount, target_update_period=target_update_period,
            dataset=dataset, counter=counter, logger=logger, checkpoint=checkpoint,
            batch_size=batch_size, seed=seed)
        acts = environment_spec.actions
        behaviour = GaussianBehaviourPolicy(learner.policy, sigma, acts.minimum, acts.maximum,
                                            seed=seed)
        actor = FeedForwardActor(behaviour, adder)
        super().__init__(actor=actor, learner=learner,
                         min_observations=max(batch_size, min_replay_size),
                         observations_per_step=float(batch_size) / samples_per_insert)
