"""An Atari-shaped environment for the IMPALA actor harness (BASELINE configs[3]: 64 CPU
actors feeding one GPU learner).  The ALE is not installed here, so this stands in for
`AtariWrapper(gym.make(...))` + frame stacking (acme/wrappers/atari_wrapper.py:155-158,
284-306; frame_stacking.py:78-83): uint8 [84, 84] grey frames stacked 4 deep on the last
axis, 18 discrete actions, clipped rewards in {-1, 0, 1}, episodes of a random length.
Frames are cheap deterministic functions of (seed, episode, step, action) — a scrolling
band pattern plus per-step noise rows — so an actor's host cost is dominated by what the
reference's actors also pay per step (policy call, adder), not by frame synthesis."""

from __future__ import annotations

import collections

import numpy as np

from acme_amd import dm_env, specs


class AtariLike(dm_env.Environment):

    def __init__(self, seed: int = 0, num_actions: int = 18, min_length: int = 200,
                 max_length: int = 1000, stack: int = 4):
        self._rng = np.random.default_rng(seed)
        self._A = int(num_actions)
        self._lengths = (int(min_length), int(max_length))
        self._stack = int(stack)
        self._frames = collections.deque(maxlen=self._stack)
        base = np.arange(84, dtype=np.int32)
        self._pattern = ((base[:, None] * 3 + base[None, :] * 5) % 256).astype(np.uint8)
        self._t = 0
        self._len = 0
        self._pos = 0

    def _frame(self) -> np.ndarray:
        f = np.roll(self._pattern, self._pos, axis=1)
        rows = self._rng.integers(0, 84, 4)
        f[rows] = self._rng.integers(0, 256, (4, 84), dtype=np.uint8)
        return f

    def _observation(self) -> np.ndarray:
        return np.stack(list(self._frames), axis=-1)

    def reset(self) -> dm_env.TimeStep:
        self._t = 0
        self._len = int(self._rng.integers(*self._lengths))
        self._pos = int(self._rng.integers(0, 84))
        self._frames.clear()
        for _ in range(self._stack - 1):
            self._frames.append(np.zeros((84, 84), np.uint8))  # zero padding at the start
        self._frames.append(self._frame())
        return dm_env.restart(self._observation())

    def step(self, action) -> dm_env.TimeStep:
        self._t += 1
        self._pos = (self._pos + int(action) - self._A // 2) % 84
        self._frames.append(self._frame())
        u = self._rng.random()
        reward = np.float32(1.0 if u < 0.02 else (-1.0 if u > 0.99 else 0.0))
        if self._t >= self._len:
            return dm_env.termination(reward, self._observation())
        return dm_env.transition(reward, self._observation())

    def observation_spec(self):
        return specs.Array((84, 84, self._stack), np.uint8, name="observation")

    def action_spec(self):
        return specs.DiscreteArray(self._A, np.int32, name="action")

    def reward_spec(self):
        return specs.Array((), np.float32, name="reward")

    def discount_spec(self):
        return specs.BoundedArray((), np.float32, 0.0, 1.0, name="discount")
