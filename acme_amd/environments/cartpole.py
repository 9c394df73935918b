"""CartPole-v1 as a dm_env environment (config 1 of BASELINE.json: the reference runs
gym's CartPole-v1 through GymWrapper + SinglePrecisionWrapper; gym is not installed here,
so the classic cart-pole dynamics of Barto, Sutton & Anderson (1983) are restated with
gym's published constants: Euler integration, tau 0.02, force 10, pole half-length 0.5,
termination at |x| > 2.4 or |theta| > 12 degrees, 500-step time limit (truncation)."""

from __future__ import annotations

import math

import numpy as np

from acme_amd import dm_env, specs


class CartPole(dm_env.Environment):
    GRAVITY, MASSCART, MASSPOLE, LENGTH, FORCE, TAU = 9.8, 1.0, 0.1, 0.5, 10.0, 0.02
    THETA_LIMIT = 12 * 2 * math.pi / 360
    X_LIMIT = 2.4

    def __init__(self, seed: int = 0, max_episode_steps: int = 500):
        self._rng = np.random.default_rng(seed)
        self._max_steps = max_episode_steps
        self._state = np.zeros(4)
        self._t = 0

    def reset(self):
        self._state = self._rng.uniform(-0.05, 0.05, 4)
        self._t = 0
        return dm_env.restart(self._state.astype(np.float32))

    def step(self, action):
        x, x_dot, th, th_dot = self._state
        total = self.MASSCART + self.MASSPOLE
        pml = self.MASSPOLE * self.LENGTH
        force = self.FORCE if int(action) == 1 else -self.FORCE
        c, s = math.cos(th), math.sin(th)
        temp = (force + pml * th_dot * th_dot * s) / total
        th_acc = (self.GRAVITY * s - c * temp) / (
            self.LENGTH * (4.0 / 3.0 - self.MASSPOLE * c * c / total))
        x_acc = temp - pml * th_acc * c / total
        x, x_dot = x + self.TAU * x_dot, x_dot + self.TAU * x_acc
        th, th_dot = th + self.TAU * th_dot, th_dot + self.TAU * th_acc
        self._state = np.array([x, x_dot, th, th_dot])
        self._t += 1
        obs = self._state.astype(np.float32)
        if abs(x) > self.X_LIMIT or abs(th) > self.THETA_LIMIT:
            return dm_env.termination(np.float32(1.0), obs)
        if self._t >= self._max_steps:
            return dm_env.truncation(np.float32(1.0), obs, np.float32(1.0))
        return dm_env.transition(np.float32(1.0), obs, np.float32(1.0))

    def observation_spec(self):
        return specs.Array((4,), np.float32, "observation")

    def action_spec(self):
        return specs.DiscreteArray(2, np.int32, "action")

    def reward_spec(self):
        return specs.Array((), np.float32, "reward")

    def discount_spec(self):
        return specs.BoundedArray((), np.float32, 0.0, 1.0, "discount")
