"""Thread-safe hierarchical counter (API of acme/utils/counting.py:27-102).

Local increments are held until `time_delta` seconds have passed, then pushed to the
parent (keys prefixed `<prefix>_`); the parent's totals are cached and merged into the
counts returned locally.
"""

from __future__ import annotations

import threading
import time
from typing import Dict, Optional, Union

from acme_amd import core

Number = Union[int, float]


def _with_prefix(counts: Dict[str, Number], prefix: str) -> Dict[str, Number]:
    return {f"{prefix}_{k}": v for k, v in counts.items()} if prefix else dict(counts)


class Counter(core.Saveable):

    def __init__(self, parent: Optional["Counter"] = None, prefix: str = "",
                 time_delta: float = 1.0):
        self._parent = parent
        self._prefix = prefix
        self._time_delta = time_delta
        self._pending: Dict[str, Number] = {}
        self._parent_view: Dict[str, Number] = {}
        self._last_push = 0.0
        self._mu = threading.Lock()

    def increment(self, **deltas: Number) -> Dict[str, Number]:
        with self._mu:
            for k, v in deltas.items():
                self._pending[k] = self._pending.get(k, 0) + v
        return self.get_counts()

    def get_counts(self) -> Dict[str, Number]:
        if self._parent is not None and time.time() - self._last_push > self._time_delta:
            with self._mu:
                push = _with_prefix(self._pending, self._prefix)
                self._pending = {}
            self._parent_view = self._parent.increment(**push)
            self._last_push = time.time()
        with self._mu:
            merged = _with_prefix(self._pending, self._prefix)
        for k, v in self._parent_view.items():
            merged[k] = merged.get(k, 0) + v
        return merged

    def save(self):
        return {"counts": dict(self._pending), "cache": dict(self._parent_view)}

    def restore(self, state):
        self._pending = dict(state["counts"])
        self._parent_view = dict(state["cache"])
        self._last_push = 0.0
