"""Loggers (API of acme/utils/loggers: Logger.write(dict), TerminalLogger with a time
gate, make_default_logger).  Device scalars (torch tensors) are only fetched to the host
when a write is actually emitted, so a learner that logs every step does not
synchronise the GPU every step."""

from __future__ import annotations

import abc
import csv
import os
import sys
import time
from typing import Any, Dict, List, Mapping, Optional

LoggingData = Mapping[str, Any]


def _to_host(v):
    if hasattr(v, "detach") and hasattr(v, "cpu"):
        v = v.detach().cpu()
        return v.item() if v.numel() == 1 else v.numpy()
    return v


class Logger(abc.ABC):
    @abc.abstractmethod
    def write(self, data: LoggingData):
        """Writes `data` (a flat mapping)."""

    def close(self):
        pass


class NoOpLogger(Logger):
    def write(self, data):
        pass


class InMemoryLogger(Logger):
    def __init__(self):
        self.data: List[Dict[str, Any]] = []

    def write(self, data):
        self.data.append({k: _to_host(v) for k, v in data.items()})


class TerminalLogger(Logger):
    """Prints `[label] k = v | ...` at most once per `time_delta` seconds."""

    def __init__(self, label: str = "", time_delta: float = 0.0, print_fn=None):
        self._label = label
        self._time_delta = time_delta
        self._last = 0.0
        self._print = print_fn or (lambda s: print(s, file=sys.stderr))

    def write(self, data):
        now = time.time()
        if now - self._last < self._time_delta:
            return
        self._last = now
        parts = []
        for k, v in sorted(data.items()):
            v = _to_host(v)
            parts.append(f"{k} = {v:.4g}" if isinstance(v, float) else f"{k} = {v}")
        self._print(f"[{self._label}] " + " | ".join(parts))


class CSVLogger(Logger):
    def __init__(self, directory: str, label: str = "logs"):
        os.makedirs(directory, exist_ok=True)
        self._path = os.path.join(directory, f"{label}.csv")
        self._fields: Optional[List[str]] = None

    def write(self, data):
        row = {k: _to_host(v) for k, v in data.items()}
        new = self._fields is None
        if new:
            self._fields = sorted(row)
        with open(self._path, "a", newline="") as f:
            w = csv.DictWriter(f, fieldnames=self._fields, extrasaction="ignore")
            if new:
                w.writeheader()
            w.writerow(row)


class Dispatcher(Logger):
    def __init__(self, loggers: List[Logger]):
        self._loggers = loggers

    def write(self, data):
        for lg in self._loggers:
            lg.write(data)


def make_default_logger(label: str, save_data: bool = False, time_delta: float = 1.0) -> Logger:
    loggers: List[Logger] = [TerminalLogger(label, time_delta)]
    if save_data:
        loggers.append(CSVLogger(os.path.expanduser("~/acme_amd/logs"), label))
    return Dispatcher(loggers)
