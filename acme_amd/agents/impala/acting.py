"""IMPALAActor — drop-in for acme/agents/tf/impala/acting.py:30-95: a recurrent actor
that samples a ~ Categorical(logits), carries the LSTM state across steps, resets it at
episode starts and hands {'logits', 'core_state'} of the step to the adder as extras."""

from __future__ import annotations

from typing import Callable, Optional

import numpy as np

from acme_amd import core
from acme_amd.networks import LSTMState


class IMPALAActor(core.Actor):

    def __init__(self, policy_step: Callable, initial_state: Callable, adder=None,
                 variable_client=None, seed: int = 0):
        self._policy_step = policy_step      # (obs, prev_a, prev_r, h, c) -> logits, v, h, c
        self._initial_state = initial_state  # batch_size -> LSTMState
        self._adder = adder
        self._variable_client = variable_client
        self._rng = np.random.default_rng(seed)
        self._state: Optional[LSTMState] = None
        self._prev_state: Optional[LSTMState] = None
        self._prev_logits = None

    def select_action(self, observation):
        if self._state is None:
            self._state = self._initial_state(1)
        obs = observation
        logits, _, h, c = self._policy_step(np.asarray(obs.observation)[None],
                                            np.asarray(obs.action).reshape(1),
                                            np.asarray(obs.reward).reshape(1),
                                            self._state.hidden, self._state.cell)
        self._prev_logits = logits[0]
        self._prev_state = LSTMState(self._state.hidden[0].copy(), self._state.cell[0].copy())
        self._state = LSTMState(h, c)
        z = logits[0] - logits[0].max()
        p = np.exp(z)
        p /= p.sum()
        return np.int32(self._rng.choice(len(p), p=p))

    def observe_first(self, timestep):
        if self._adder:
            self._adder.add_first(timestep)
        self._state = None  # re-initialised at the next policy call

    def observe(self, action, next_timestep):
        if not self._adder:
            return
        extras = {"logits": self._prev_logits, "core_state": self._prev_state}
        self._adder.add(action, next_timestep, extras)

    def update(self):
        if self._variable_client:
            self._variable_client.update()
