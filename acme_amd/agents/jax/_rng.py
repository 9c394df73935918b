"""hk.PRNGSequence stand-in: the JAX learners draw one key per network initialisation
(agents/jax/dqn/learning.py:148-151 draws two, so the target starts from its own init)."""

from __future__ import annotations

import numpy as np


class PRNGSequence:
    """Iterator of 31-bit integer seeds derived from `seed` (numpy SeedSequence)."""

    def __init__(self, seed: int):
        self._ss = np.random.SeedSequence(int(seed))

    def __iter__(self):
        return self

    def __next__(self) -> int:
        return int(self._ss.spawn(1)[0].generate_state(1)[0] & 0x7FFFFFFF)


def as_sequence(rng):
    """An int seed, a PRNGSequence or any iterator of int seeds."""
    if isinstance(rng, (int, np.integer)):
        return PRNGSequence(int(rng))
    return iter(rng)
