"""Adder interface (acme/adders/base.py:24-82)."""

import abc


class Adder(abc.ABC):
    """Receives (action, timestep) pairs from an actor and writes replay items."""

    @abc.abstractmethod
    def add_first(self, timestep):
        """Starts a trajectory with its first timestep (timestep.first() must hold)."""

    @abc.abstractmethod
    def add(self, action, next_timestep, extras=()):
        """Adds an action and the timestep it led to (plus optional extras)."""

    @abc.abstractmethod
    def reset(self):
        """Drops any partial trajectory."""
