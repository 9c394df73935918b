"""Agent = actor + learner with the learner-step cadence of acme/agents/agent.py:45-89.

No learner step happens until `min_observations` observations have been made; after
that, every `observations_per_step` observations trigger one learner step (or, for a
ratio below one, `1 / observations_per_step` steps per observation)."""

from __future__ import annotations

from typing import List

from acme_amd import core


class Agent(core.Actor, core.VariableSource):

    def __init__(self, actor: core.Actor, learner: core.Learner, min_observations: int,
                 observations_per_step: float):
        self._actor = actor
        self._learner = learner
        self._countdown = -int(min_observations)  # observations still to wait for
        if observations_per_step >= 1.0:
            self._obs_per_update, self._steps_per_update = int(observations_per_step), 1
        else:
            self._obs_per_update, self._steps_per_update = 1, int(1.0 / observations_per_step)

    def select_action(self, observation):
        return self._actor.select_action(observation)

    def observe_first(self, timestep):
        self._actor.observe_first(timestep)

    def observe(self, action, next_timestep):
        self._countdown += 1
        self._actor.observe(action, next_timestep)

    def update(self):
        if self._countdown < 0 or self._countdown % self._obs_per_update != 0:
            return
        self._countdown = 0
        for _ in range(self._steps_per_update):
            self._learner.step()
        self._actor.update()

    def get_variables(self, names: List[str]) -> List:
        return self._learner.get_variables(names)
