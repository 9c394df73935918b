"""Actors (acme/agents/tf/actors.py:35-94 FeedForwardActor) and the epsilon-greedy DQN
policy (trfl.epsilon_greedy used at acme/agents/tf/dqn/agent.py:118-124)."""

from __future__ import annotations

from typing import Callable, Optional

import numpy as np

from acme_amd import core


class FeedForwardActor(core.Actor):
    """Runs `policy` on a batch of one observation; forwards experience to an adder."""

    def __init__(self, policy: Callable, adder=None, variable_client=None):
        self._policy = policy
        self._adder = adder
        self._variable_client = variable_client

    def select_action(self, observation):
        batched = np.asarray(observation)[None]
        return np.asarray(self._policy(batched))[0]

    def observe_first(self, timestep):
        if self._adder is not None:
            self._adder.add_first(timestep)

    def observe(self, action, next_timestep):
        if self._adder is not None:
            self._adder.add(action, next_timestep)

    def update(self):
        if self._variable_client is not None:
            self._variable_client.update()


class EpsilonGreedyPolicy:
    """a ~ (1 - eps) * uniform over argmax q + eps * uniform over actions (trfl semantics:
    greedy ties share the greedy mass)."""

    def __init__(self, q_fn: Callable, num_actions: int, epsilon: float = 0.05, seed: int = 0,
                 action_dtype=np.int32):
        self._q_fn = q_fn
        self._A = int(num_actions)
        self.epsilon = float(epsilon)
        self._rng = np.random.default_rng(seed)
        self._dtype = action_dtype

    def __call__(self, batched_obs):
        q = np.asarray(self._q_fn(batched_obs))
        out = np.empty(q.shape[0], self._dtype)
        for i, row in enumerate(q):
            greedy = np.flatnonzero(row == row.max())
            probs = np.full(self._A, self.epsilon / self._A)
            probs[greedy] += (1.0 - self.epsilon) / len(greedy)
            out[i] = self._rng.choice(self._A, p=probs / probs.sum())
        return out
