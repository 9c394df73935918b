"""Shared machinery of the replay adders (semantics of acme/adders/reverb/base.py:62-213
and acme/adders/reverb/utils.py:69-104).

An adder holds a bounded window of `Step`s plus the dangling next observation of the
current trajectory, and talks to a writer obtained lazily from `client.writer(...)`:
`writer.append(data)` then `writer.create_item(table, num_timesteps, priority)`.  The
client may be the GPU replay client (acme_amd.replay.Client) or any object with the
same writer surface (e.g. the reference's FakeClient pattern used by the tests).
"""

from __future__ import annotations

import abc
import collections
from typing import Any, Callable, Dict, Mapping, NamedTuple, Optional, Sequence

import numpy as np

from acme_amd import specs
from acme_amd.adders import base
from acme_amd.utils import tree

DEFAULT_PRIORITY_TABLE = "priority_table"


class Step(NamedTuple):
    observation: Any
    action: Any
    reward: Any
    discount: Any
    start_of_episode: Any
    extras: Any


class PriorityFnInput(NamedTuple):
    """Steps stacked along time; the priority function's argument."""
    observations: Any
    actions: Any
    rewards: Any
    discounts: Any
    start_of_episode: Any
    extras: Any


PriorityFn = Callable[[PriorityFnInput], float]
PriorityFnMapping = Mapping[str, PriorityFn]


def zeros_like(x):
    """Zero of the same (d)type and shape; keeps python/numpy scalar types."""
    if isinstance(x, (bool, int, float, np.number, np.bool_)):
        return type(x)(0)
    if isinstance(x, np.ndarray):
        return np.zeros_like(x)
    if hasattr(x, "new_zeros"):  # torch tensor
        return x.new_zeros(x.shape)
    raise ValueError(f"cannot build a zero like {type(x)}: need a numpy array, int or float")


def final_step_like(step: Step, next_observation) -> Step:
    """The closing step of a trajectory: next observation, everything else zero."""
    return Step(observation=next_observation,
                action=tree.map_structure(zeros_like, step.action),
                reward=tree.map_structure(zeros_like, step.reward),
                discount=tree.map_structure(zeros_like, step.discount),
                start_of_episode=False,
                extras=tree.map_structure(zeros_like, step.extras))


def stack_steps(steps: Sequence[Step]):
    """Stacks each leaf of a sequence of identically structured steps along axis 0."""
    return tree.map_structure(lambda *xs: np.stack([np.asarray(x) for x in xs]), *steps)


def uniform_priority(_) -> float:
    """The default priority function (adders/reverb/base.py:91-92: lambda x: 1.)."""
    return 1.


def calculate_priorities(priority_fns: PriorityFnMapping, steps) -> Dict[str, float]:
    """`steps`: the window, or a callable returning it.  The stacked window
    (acme/adders/reverb/utils.py:97-103) is only built when some function reads it:
    stacking an Atari window copies its frames (112 KB per transition) to feed the default
    uniform_priority, which ignores its input."""
    stacked = None
    out = {}
    for table, fn in priority_fns.items():
        if fn is uniform_priority:
            out[table] = 1.
            continue
        if stacked is None:
            stacked = PriorityFnInput(*stack_steps(steps() if callable(steps) else steps))
        out[table] = fn(stacked)
    return out


class ReverbAdder(base.Adder):
    """Trajectory window + lazily created writer; subclasses decide what to write."""

    def __init__(self, client, buffer_size: int, max_sequence_length: int,
                 delta_encoded: bool = False, chunk_length: Optional[int] = None,
                 priority_fns: Optional[PriorityFnMapping] = None):
        self._client = client
        self._priority_fns = (dict(priority_fns) if priority_fns
                              else {DEFAULT_PRIORITY_TABLE: uniform_priority})
        self._max_sequence_length = max_sequence_length
        self._writer_kwargs = dict(delta_encoded=delta_encoded, chunk_length=chunk_length)
        self._active_writer = None
        self._buffer: collections.deque = collections.deque(maxlen=buffer_size)
        self._next_observation = None
        self._start_of_episode = False

    @property
    def _writer(self):
        if self._active_writer is None:
            self._active_writer = self._client.writer(self._max_sequence_length,
                                                      **self._writer_kwargs)
        return self._active_writer

    def add_priority_table(self, table_name: str, priority_fn: PriorityFn):
        if table_name in self._priority_fns:
            raise ValueError(f"A priority function already exists for {table_name}.")
        self._priority_fns[table_name] = priority_fn

    def reset(self):
        if self._active_writer is not None:
            self._active_writer.close()
            self._active_writer = None
        self._buffer.clear()
        self._next_observation = None

    def add_first(self, timestep):
        if not timestep.first():
            raise ValueError("adder.add_first with an initial timestep (i.e. one for "
                             "which timestep.first() is True")
        if self._next_observation is not None:
            raise ValueError("adder.reset must be called before adder.add_first "
                             "(called automatically if `next_timestep.last()` is "
                             "true when `add` is called).")
        self._next_observation = timestep.observation
        self._start_of_episode = True

    def add(self, action, next_timestep, extras=()):
        if self._next_observation is None:
            raise ValueError("adder.add_first must be called before adder.add.")
        self._buffer.append(Step(observation=self._next_observation, action=action,
                                 reward=next_timestep.reward, discount=next_timestep.discount,
                                 start_of_episode=self._start_of_episode, extras=extras))
        self._next_observation = next_timestep.observation
        self._start_of_episode = False
        self._write()
        if next_timestep.last():
            self._write_last()
            self.reset()

    def _emit(self, num_steps: int, steps):
        """steps: the window, or a callable building it (only priority functions read it)."""
        for table, priority in calculate_priorities(self._priority_fns, steps).items():
            self._writer.create_item(table=table, num_timesteps=num_steps, priority=priority)

    @classmethod
    def signature(cls, environment_spec: specs.EnvironmentSpec, extras_spec=()):
        return Step(observation=environment_spec.observations, action=environment_spec.actions,
                    reward=environment_spec.rewards, discount=environment_spec.discounts,
                    start_of_episode=specs.Array((), np.bool_), extras=extras_spec)

    @abc.abstractmethod
    def _write(self):
        """Called after every add."""

    @abc.abstractmethod
    def _write_last(self):
        """Called when the trajectory ends."""
