"""EnvironmentLoop — drop-in for acme/environment_loop.py:63-144.

reset -> observe_first -> (select_action, step, observe, update)* until the episode's
last timestep; counts episodes/steps, logs episode_length / episode_return /
steps_per_second merged with the counter's totals."""

from __future__ import annotations

import time
from typing import Optional

from acme_amd import core
from acme_amd.utils import counting, loggers


class EnvironmentLoop(core.Worker):

    def __init__(self, environment, actor: core.Actor, counter: Optional[counting.Counter] = None,
                 logger: Optional[loggers.Logger] = None, label: str = "environment_loop"):
        self._env = environment
        self._actor = actor
        self._counter = counter or counting.Counter()
        self._logger = logger or loggers.make_default_logger(label)

    def run_episode(self) -> dict:
        t0 = time.time()
        steps, ret = 0, 0
        ts = self._env.reset()
        self._actor.observe_first(ts)
        while not ts.last():
            action = self._actor.select_action(ts.observation)
            ts = self._env.step(action)
            self._actor.observe(action, next_timestep=ts)
            self._actor.update()
            steps += 1
            ret = ret + ts.reward
        result = {"episode_length": steps, "episode_return": ret,
                  "steps_per_second": steps / max(time.time() - t0, 1e-9)}
        result.update(self._counter.increment(episodes=1, steps=steps))
        return result

    def run(self, num_episodes: Optional[int] = None, num_steps: Optional[int] = None):
        if num_episodes is not None and num_steps is not None:
            raise ValueError('Either "num_episodes" or "num_steps" should be None.')
        episodes = steps = 0
        while not ((num_episodes is not None and episodes >= num_episodes) or
                   (num_steps is not None and steps >= num_steps)):
            result = self.run_episode()
            episodes += 1
            steps += result["episode_length"]
            self._logger.write(result)
