"""Core interfaces, drop-in for acme/core.py:31-152.

Actor / VariableSource / Worker / Learner / Saveable keep the reference's method names
and contracts so existing agent code constructs unchanged: `Learner.step()` performs
one update, `Learner.run()` loops on it forever, `get_variables(names)` returns host
(numpy) copies and must be callable from another thread.
"""

import abc
from typing import Generic, List, NoReturn, TypeVar

T = TypeVar("T")


class Actor(abc.ABC):
    """Acts in an environment: select_action / observe_first / observe / update."""

    @abc.abstractmethod
    def select_action(self, observation):
        """Returns an action for the observation."""

    @abc.abstractmethod
    def observe_first(self, timestep):
        """Records the first timestep of an episode."""

    @abc.abstractmethod
    def observe(self, action, next_timestep):
        """Records an action and the timestep it produced."""

    @abc.abstractmethod
    def update(self):
        """Refreshes the actor's parameters."""


class VariableSource(abc.ABC):
    @abc.abstractmethod
    def get_variables(self, names: List[str]) -> List:
        """Returns the named collections of variables as (nested) numpy arrays."""


class Worker(abc.ABC):
    @abc.abstractmethod
    def run(self):
        """Runs the worker."""


class Learner(VariableSource, Worker):
    """A learner performs updates from a dataset; `run` repeats `step` forever."""

    @abc.abstractmethod
    def step(self):
        """One update of the learner's parameters."""

    def run(self) -> NoReturn:
        while True:
            self.step()


class Saveable(abc.ABC, Generic[T]):
    @abc.abstractmethod
    def save(self) -> T:
        """Returns the state to checkpoint."""

    @abc.abstractmethod
    def restore(self, state: T):
        """Restores a state returned by save()."""
