"""Test fakes (pattern of acme/testing/fakes.py and acme/adders/reverb/test_utils.py).

- FakeClient / FakeWriter: record what an adder writes (append / create_item / close).
- Environment / DiscreteEnvironment / ContinuousEnvironment: spec-driven environments
  with a fixed episode length that emit random observations.
- transition_dataset: a constant batch of ReplaySample(info=SampleInfo(key=0,
  probability=1.0, table_size=1, priority=1.0), data=transition) (fakes.py:233-262).
"""

from __future__ import annotations

from typing import Any, List, Optional

import numpy as np

from acme_amd import dm_env, specs
from acme_amd.utils import tree


class FakeWriter:
    def __init__(self, max_sequence_length, delta_encoded=False, chunk_length=None):
        self.max_sequence_length = max_sequence_length
        self.delta_encoded = delta_encoded
        self.chunk_length = chunk_length
        self.timesteps: List[Any] = []
        self.priorities: List[Any] = []  # (table, item, priority)
        self.closed = False

    def append(self, data):
        if self.closed:
            raise AssertionError("append on a closed writer")
        self.timesteps.append(data)

    def create_item(self, table, num_timesteps, priority):
        if self.closed:
            raise AssertionError("create_item on a closed writer")
        if num_timesteps > len(self.timesteps) or num_timesteps > self.max_sequence_length:
            raise AssertionError("item longer than the appended history / max_sequence_length")
        item = self.timesteps[-num_timesteps:]
        self.priorities.append((table, item[0] if num_timesteps == 1 else item, priority))

    def close(self):
        if self.closed:
            raise AssertionError("writer closed twice")
        self.closed = True


class FakeClient:
    def __init__(self):
        self.writers: List[FakeWriter] = []

    def writer(self, max_sequence_length, delta_encoded=False, chunk_length=None):
        w = FakeWriter(max_sequence_length, delta_encoded, chunk_length)
        self.writers.append(w)
        return w


def _random_like(spec, rng):
    if isinstance(spec, specs.DiscreteArray):
        return np.asarray(rng.integers(0, spec.num_values), spec.dtype)
    if isinstance(spec, specs.BoundedArray):
        lo = np.broadcast_to(spec.minimum, spec.shape)
        hi = np.broadcast_to(spec.maximum, spec.shape)
        if np.issubdtype(spec.dtype, np.integer):
            return rng.integers(lo, hi + 1, spec.shape).astype(spec.dtype)
        return rng.uniform(lo, hi, spec.shape).astype(spec.dtype)
    if np.issubdtype(spec.dtype, np.integer):
        return rng.integers(0, 256, spec.shape).astype(spec.dtype)
    return rng.standard_normal(spec.shape).astype(spec.dtype)


class Environment(dm_env.Environment):
    """Emits random observations for `episode_length` steps, reward/discount per spec."""

    def __init__(self, spec: specs.EnvironmentSpec, episode_length: int = 25, seed: int = 0):
        self._spec = spec
        self._episode_length = episode_length
        self._rng = np.random.default_rng(seed)
        self._step = 0

    def _obs(self):
        return tree.map_structure(lambda s: _random_like(s, self._rng), self._spec.observations)

    def reset(self):
        self._step = 0
        return dm_env.restart(self._obs())

    def step(self, action):
        tree.map_structure(lambda s, a: s.validate(a), self._spec.actions, action)
        self._step += 1
        reward = tree.map_structure(lambda s: _random_like(s, self._rng), self._spec.rewards)
        if self._step >= self._episode_length:
            return dm_env.termination(reward, self._obs())
        return dm_env.transition(reward, self._obs())

    def observation_spec(self):
        return self._spec.observations

    def action_spec(self):
        return self._spec.actions

    def reward_spec(self):
        return self._spec.rewards

    def discount_spec(self):
        return self._spec.discounts


class DiscreteEnvironment(Environment):
    def __init__(self, num_actions: int = 2, num_observations: int = 4, obs_shape=(4,),
                 obs_dtype=np.float32, action_dtype=np.int32, reward_dtype=np.float32,
                 discount_dtype=np.float32, episode_length: int = 25, seed: int = 0):
        spec = specs.EnvironmentSpec(
            observations=specs.Array(obs_shape, obs_dtype, "observation"),
            actions=specs.DiscreteArray(num_actions, action_dtype, "action"),
            rewards=specs.Array((), reward_dtype, "reward"),
            discounts=specs.BoundedArray((), discount_dtype, 0.0, 1.0, "discount"))
        del num_observations
        super().__init__(spec, episode_length, seed)


class ContinuousEnvironment(Environment):
    def __init__(self, obs_dim: int = 24, action_dim: int = 6, episode_length: int = 25,
                 seed: int = 0):
        spec = specs.EnvironmentSpec(
            observations=specs.Array((obs_dim,), np.float32, "observation"),
            actions=specs.BoundedArray((action_dim,), np.float32, -1.0, 1.0, "action"),
            rewards=specs.Array((), np.float32, "reward"),
            discounts=specs.BoundedArray((), np.float32, 0.0, 1.0, "discount"))
        super().__init__(spec, episode_length, seed)


def transition_dataset(environment, batch_size: int = 1, device: Optional[str] = None):
    """Infinite iterator of one constant batched transition (device tensors)."""
    import torch
    from acme_amd.replay import ReplaySample, SampleInfo
    spec = specs.make_environment_spec(environment)
    rng = np.random.default_rng(0)
    o = _random_like(spec.observations, rng)
    a = _random_like(spec.actions, rng)
    r = _random_like(spec.rewards, rng)
    d = np.asarray(1.0, spec.discounts.dtype)
    dev = device or "cuda"

    def batch(x):
        x = np.asarray(x)
        return torch.as_tensor(np.broadcast_to(x, (batch_size,) + x.shape).copy()).to(dev)

    data = tuple(batch(x) for x in (o, a, r, d, o))
    info = SampleInfo(key=torch.zeros(batch_size, dtype=torch.uint64, device=dev),
                      probability=torch.ones(batch_size, dtype=torch.float64, device=dev),
                      table_size=torch.ones(batch_size, dtype=torch.int64, device=dev),
                      priority=torch.ones(batch_size, dtype=torch.float64, device=dev))
    sample = ReplaySample(info=info, data=data)
    while True:
        yield sample
