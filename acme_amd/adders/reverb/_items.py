"""N-step transition, fixed-length sequence and whole-episode adders.

Semantics (pinned by the reference's golden tables, tests/golden/adder_cases.json):
  NStepTransitionAdder  acme/adders/reverb/transition.py:119-172
      item = (o_t, a_t, R, D, o_{t+n}[, e_t]) with, over the window s_0..s_{k-1},
        R = r_0 + sum_{i>=1} (g^i prod_{j<i} d_j) r_i,  D = g^{k-1} prod_{j<k} d_j
      (the agent discount g is float32); shorter windows at episode start and end.
  SequenceAdder  acme/adders/reverb/sequence.py:30-127
      every `period` steps once `sequence_length` steps exist, an item of the last
      `sequence_length` steps; at episode end a zero-padded final step (+ padding).
  EpisodeAdder  acme/adders/reverb/episode.py:31-86
      one item per episode; raises once an episode exceeds max_sequence_length.
"""

from __future__ import annotations

import copy
from typing import Optional

import numpy as np

from acme_amd import specs
from acme_amd.adders.reverb._common import (PriorityFnMapping, ReverbAdder, Step,
                                            final_step_like, uniform_priority, zeros_like)
from acme_amd.utils import tree


# Reward / discount types whose n-step accumulation the Python path does in f32 exactly as
# the native writer does: numpy float32, and Python floats (weak scalars under NumPy >= 2:
# every operation with the adder's float32 discount stays float32).
_F32_SAFE = (np.float32, float) if int(np.__version__.split(".")[0]) >= 2 else (np.float32,)


class NStepTransitionAdder(ReverbAdder):
    """Items are formed here in Python, or, when the client is a GPU replay table's and the
    step's fields allow it, by the table's native n-step writer (csrc/replay.hip,
    acme_nstep_writer: the same items, packed in C straight into pinned staging rows).  The
    native path takes an episode whose first observation fits the table's layout, and each
    step whose reward and discount are float32 scalars (the f32 accumulation both paths then
    share; a Python float too, which NumPy >= 2 promotes weakly, so that the Python path
    computes in f32 as well), whose observation is a C-contiguous array of the table's dtype and shape, with no
    extras and the default uniform priority.  A step that does not fit falls back to the
    Python path for the rest of the episode (the window is kept in both)."""

    def __init__(self, client, n_step: int, discount: float,
                 priority_fns: Optional[PriorityFnMapping] = None, rows_per_chunk: int = 64):
        if n_step < 1:
            raise ValueError(f"n_step must be >= 1, got {n_step}")
        self._discount = np.float32(discount)
        super().__init__(client=client, buffer_size=n_step, max_sequence_length=1,
                         priority_fns=priority_fns)
        self._n_step = int(n_step)
        self._rows_per_chunk = int(rows_per_chunk)
        self._fast = None        # (writer, obs shape, obs dtype, action buffer) or False
        self._native_ep = False  # the current episode goes through the native writer

    def _fast_path(self):
        if self._fast is None:
            self._fast = self._make_fast() or False
        return self._fast

    def _make_fast(self):
        from acme_amd import replay
        if not isinstance(self._client, replay.Client) or len(self._priority_fns) != 1:
            return None
        (name, fn), = self._priority_fns.items()
        table = self._client.server.tables.get(name)
        if fn is not uniform_priority or type(table) is not replay.Table:
            return None
        f = table.fields
        if (f is None or len(f) != 5 or table.sequence_length or table.native is None
                or (f[0].shape, f[0].dtype) != (f[4].shape, f[4].dtype)
                or any(x.shape != () or x.dtype != np.float32 for x in f[2:4])):
            return None
        w = table.native.nstep_writer(self._n_step, float(self._discount), f[0].nbytes,
                                      f[1].nbytes, self._rows_per_chunk)
        table.register_writer(w)
        act = np.zeros(f[1].shape, f[1].dtype)
        return w, f[0].shape, f[0].dtype, act, act.__array_interface__["data"][0]

    def add_first(self, timestep):
        super().add_first(timestep)
        fast = self._fast_path()
        o = timestep.observation
        self._native_ep = bool(fast) and (type(o) is np.ndarray and o.dtype == fast[2]
                                          and o.shape == fast[1] and o.flags.c_contiguous)
        if self._native_ep:
            fast[0].start(o.__array_interface__["data"][0])

    def add(self, action, next_timestep, extras=()):
        if self._native_ep:
            w, shape, dtype, act, act_ptr = self._fast
            o, r, d = next_timestep.observation, next_timestep.reward, next_timestep.discount
            if (not extras and type(r) in _F32_SAFE and type(d) in _F32_SAFE
                    and type(o) is np.ndarray and o.dtype == dtype and o.shape == shape
                    and o.flags.c_contiguous and np.shape(action) == act.shape):
                self._buffer.append(Step(self._next_observation, action, r, d,
                                         self._start_of_episode, extras))
                self._next_observation = o
                self._start_of_episode = False
                act[...] = action
                last = next_timestep.last()
                w.add_raw(act_ptr, r, d, o.__array_interface__["data"][0], last)
                if last:
                    self.reset()
                return
            self._native_ep = False  # the rest of this episode takes the Python path
        super().add(action, next_timestep, extras)

    def reset(self):
        self._native_ep = False
        if self._fast:
            self._fast[0].reset()
        super().reset()

    def _transition(self):
        head = self._buffer[0]
        ret = copy.deepcopy(head.reward)
        disc = copy.deepcopy(head.discount)
        for step in list(self._buffer)[1:]:
            disc = disc * self._discount      # agent discount enters before each reward
            ret = ret + step.reward * disc
            disc = disc * step.discount
        out = (head.observation, head.action, ret, disc, self._next_observation)
        return out + (head.extras,) if head.extras else out

    def _write(self):
        item = self._transition()
        buf, nxt = list(self._buffer), self._next_observation
        self._writer.append(item)
        self._emit(1, lambda: buf + [final_step_like(buf[0], nxt)])

    def _write_last(self):
        # Drain: emit the shrinking windows that end at the final observation.
        self._buffer.popleft()
        while self._buffer:
            self._write()
            self._buffer.popleft()

    @classmethod
    def signature(cls, environment_spec: specs.EnvironmentSpec, extras_spec=()):
        sig = (environment_spec.observations, environment_spec.actions, environment_spec.rewards,
               environment_spec.discounts, environment_spec.observations)
        return sig + (extras_spec,) if extras_spec else sig


class SequenceAdder(ReverbAdder):

    def __init__(self, client, sequence_length: int, period: int, delta_encoded: bool = False,
                 chunk_length: Optional[int] = None,
                 priority_fns: Optional[PriorityFnMapping] = None,
                 pad_end_of_episode: bool = True):
        super().__init__(client=client, buffer_size=sequence_length,
                         max_sequence_length=sequence_length, delta_encoded=delta_encoded,
                         chunk_length=chunk_length, priority_fns=priority_fns)
        self._period = period
        self._pad = pad_end_of_episode
        self._count = 0

    def reset(self):
        self._count = 0
        super().reset()

    def _push(self, step):
        self._writer.append(step)
        self._count += 1

    def _write(self):
        self._push(self._buffer[-1])
        self._maybe_emit()

    def _write_last(self):
        closing = final_step_like(self._buffer[0], self._next_observation)
        self._buffer.append(closing)
        self._push(closing)
        if self._pad:
            L = self._max_sequence_length
            # Pad so that the final item is full: up to L steps if fewer were written,
            # otherwise up to the next period boundary.
            missing = L - self._count if self._count <= L else self._period - (self._count - L)
            zero = tree.map_structure(zeros_like, closing)
            for _ in range(missing):
                self._buffer.append(zero)
                self._push(zero)
        self._maybe_emit()

    def _maybe_emit(self):
        L = self._max_sequence_length
        due = self._count == L or (self._count > L and (self._count - L) % self._period == 0)
        if due:
            steps = list(self._buffer)
            self._emit(len(steps), steps)


class EpisodeAdder(ReverbAdder):

    def __init__(self, client, max_sequence_length: int, delta_encoded: bool = False,
                 chunk_length: Optional[int] = None,
                 priority_fns: Optional[PriorityFnMapping] = None):
        super().__init__(client=client, buffer_size=max_sequence_length - 1,
                         max_sequence_length=max_sequence_length, delta_encoded=delta_encoded,
                         chunk_length=chunk_length, priority_fns=priority_fns)

    def add(self, action, next_timestep, extras=()):
        if len(self._buffer) == self._buffer.maxlen:
            raise ValueError("The number of observations within the same episode exceeds "
                             "max_sequence_length")
        super().add(action, next_timestep, extras)

    def _write(self):
        self._writer.append(self._buffer[-1])

    def _write_last(self):
        closing = final_step_like(self._buffer[0], self._next_observation)
        self._writer.append(closing)
        steps = list(self._buffer) + [closing]
        self._emit(len(steps), steps)
