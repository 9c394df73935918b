"""dm_env-compatible environment types.

The reference builds on DeepMind's `dm_env` (TimeStep, StepType, restart/transition/
termination, Environment and the specs module — imported at acme/core.py:26).  dm_env is
not installed in this image, so this module provides the same API surface; when the
real package is importable it is re-exported instead, so objects interoperate.
"""

from __future__ import annotations

import abc
import enum
from typing import Any, NamedTuple

import numpy as np

try:  # pragma: no cover - exercised only where dm_env exists
    import dm_env as _real  # type: ignore
except ImportError:  # the normal case in this image
    _real = None


if _real is not None:  # pragma: no cover
    StepType = _real.StepType
    TimeStep = _real.TimeStep
    restart, transition, termination, truncation = (_real.restart, _real.transition,
                                                    _real.termination, _real.truncation)
    Environment = _real.Environment
    specs = _real.specs
else:

    class StepType(enum.IntEnum):
        FIRST = 0
        MID = 1
        LAST = 2

        def first(self) -> bool:
            return self is StepType.FIRST

        def mid(self) -> bool:
            return self is StepType.MID

        def last(self) -> bool:
            return self is StepType.LAST

    class TimeStep(NamedTuple):
        step_type: Any
        reward: Any
        discount: Any
        observation: Any

        def first(self) -> bool:
            return self.step_type == StepType.FIRST

        def mid(self) -> bool:
            return self.step_type == StepType.MID

        def last(self) -> bool:
            return self.step_type == StepType.LAST

    def restart(observation):
        return TimeStep(StepType.FIRST, None, None, observation)

    def transition(reward, observation, discount=1.0):
        return TimeStep(StepType.MID, reward, discount, observation)

    def termination(reward, observation):
        return TimeStep(StepType.LAST, reward, 0.0, observation)

    def truncation(reward, observation, discount=1.0):
        return TimeStep(StepType.LAST, reward, discount, observation)

    class _Specs:
        """dm_env.specs: Array / BoundedArray / DiscreteArray."""

        class Array:
            def __init__(self, shape, dtype, name=None):
                self._shape = tuple(int(s) for s in shape)
                self._dtype = np.dtype(dtype)
                self._name = name

            shape = property(lambda self: self._shape)
            dtype = property(lambda self: self._dtype)
            name = property(lambda self: self._name)

            def generate_value(self):
                return np.zeros(self._shape, self._dtype)

            def validate(self, value):
                value = np.asarray(value)
                if value.shape != self._shape:
                    raise ValueError(f"expected shape {self._shape}, got {value.shape}")
                return value

            def __repr__(self):
                return f"Array(shape={self._shape}, dtype={self._dtype}, name={self._name!r})"

        class BoundedArray(Array):
            def __init__(self, shape, dtype, minimum, maximum, name=None):
                super().__init__(shape, dtype, name)
                self._minimum = np.broadcast_to(np.asarray(minimum, dtype), self._shape)
                self._maximum = np.broadcast_to(np.asarray(maximum, dtype), self._shape)

            minimum = property(lambda self: self._minimum)
            maximum = property(lambda self: self._maximum)

            def generate_value(self):
                return np.array(self._minimum, self._dtype, copy=True)

        class DiscreteArray(BoundedArray):
            def __init__(self, num_values, dtype=np.int32, name=None):
                super().__init__((), dtype, 0, num_values - 1, name)
                self._num_values = int(num_values)

            num_values = property(lambda self: self._num_values)

    specs = _Specs()

    class Environment(abc.ABC):
        @abc.abstractmethod
        def reset(self) -> TimeStep:
            ...

        @abc.abstractmethod
        def step(self, action) -> TimeStep:
            ...

        @abc.abstractmethod
        def observation_spec(self):
            ...

        @abc.abstractmethod
        def action_spec(self):
            ...

        def reward_spec(self):
            return specs.Array((), np.float64, name="reward")

        def discount_spec(self):
            return specs.BoundedArray((), np.float64, 0.0, 1.0, name="discount")

        def close(self):
            pass
