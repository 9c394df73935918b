"""Checkpointing of Saveable objects.

Semantics of the reference (acme/tf/savers.py):
  Checkpointer            time-gated `save(force=False)` (:155-176), restore of the latest
                          checkpoint on construction (:147, :178-184);
  CheckpointingRunner     wraps a learner, alternates `step()` and `save()`, and forces a
                          save on SIGTERM (preemption, :199-221).
A Saveable's state (`save()` / `restore(state)`, acme/core.py:87-106) is a nest of dicts
whose leaves are numpy arrays or scalars.  It is written as one .npz per checkpoint: the
leaves as arrays "0", "1", ... and a JSON manifest holding each leaf's key path, so keys
may contain any character (parameter names contain '/').  Files are written atomically
(tmp + rename) and loaded with allow_pickle=False.
"""

from __future__ import annotations

import json
import logging
import os
import signal
import time
from typing import Any, Dict, List, Mapping, Tuple

import numpy as np

from acme_amd import core

_MANIFEST = "__manifest__"


def _flatten(d: Mapping, path: Tuple[str, ...] = ()) -> List[Tuple[Tuple[str, ...], Any]]:
    out = []
    for k, v in d.items():
        if not isinstance(k, str):
            raise TypeError(f"state keys must be strings, got {k!r}")
        if isinstance(v, Mapping):
            out.extend(_flatten(v, path + (k,)))
        else:
            out.append((path + (k,), v))
    return out


def _pack(state: Mapping) -> Dict[str, np.ndarray]:
    arrays, manifest = {}, []
    for i, (path, v) in enumerate(_flatten(state)):
        a = np.asarray(v)
        if a.dtype == object:
            raise TypeError(f"state leaf {'/'.join(path)} is not a numeric array")
        arrays[str(i)] = a
        manifest.append({"path": list(path), "scalar": not isinstance(v, np.ndarray) and a.ndim == 0})
    arrays[_MANIFEST] = np.array(json.dumps(manifest))
    return arrays


def _unpack(z: Mapping[str, np.ndarray]) -> Dict:
    if _MANIFEST not in z:
        # The round-1 format ('/'-joined flat keys) cannot be unflattened unambiguously:
        # parameter names contain '/' themselves.
        raise ValueError("unsupported checkpoint format: no manifest (a checkpoint.npz written "
                         "by an older acme_amd with '/'-joined flat keys); re-save it with "
                         "this version or start from a fresh directory")
    manifest = json.loads(str(z[_MANIFEST]))
    out: Dict = {}
    for i, entry in enumerate(manifest):
        node = out
        path = entry["path"]
        for k in path[:-1]:
            node = node.setdefault(k, {})
        v = z[str(i)]
        node[path[-1]] = v.item() if entry["scalar"] else v
    return out


class Checkpointer:
    """Periodic checkpointing of named Saveables (acme/tf/savers.py:52-184)."""

    def __init__(self, objects_to_save: Mapping[str, core.Saveable], directory: str = "~/acme/",
                 time_delta_minutes: float = 10.0, enable_checkpointing: bool = True,
                 subdirectory: str = "default"):
        self._objects = dict(objects_to_save)
        self._dir = os.path.join(os.path.expanduser(directory), subdirectory) \
            if subdirectory and subdirectory != "default" else os.path.expanduser(directory)
        self._delta = time_delta_minutes * 60.0
        self._last = time.time()
        self._enabled = enable_checkpointing
        self._path = os.path.join(self._dir, "checkpoint.npz")
        if enable_checkpointing and os.path.exists(self._path):
            self.restore()

    @property
    def path(self) -> str:
        return self._path

    def save(self, force: bool = False) -> bool:
        """Saves if `time_delta_minutes` have passed since the last save (or `force`)."""
        if not self._enabled or (not force and time.time() - self._last < self._delta):
            return False
        os.makedirs(self._dir, exist_ok=True)
        state = {name: obj.save() for name, obj in self._objects.items()}
        tmp = self._path + ".tmp.npz"
        np.savez(tmp, **_pack(state))
        os.replace(tmp, self._path)
        self._last = time.time()
        return True

    def restore(self) -> None:
        with np.load(self._path, allow_pickle=False) as z:
            state = _unpack({k: z[k] for k in z.files})
        for name, obj in self._objects.items():
            if name in state:
                obj.restore(state[name])


class CheckpointingRunner(core.Worker):
    """Runs a learner (or any Saveable) with periodic checkpoints and a forced save on
    SIGTERM (acme/tf/savers.py:187-233).  Attribute access falls through to the wrapped
    object."""

    def __init__(self, wrapped, *, time_delta_minutes: float = 30.0, **kwargs):
        self._wrapped = wrapped
        self._time_delta_minutes = time_delta_minutes
        self._checkpointer = Checkpointer(objects_to_save={"wrapped": wrapped},
                                          time_delta_minutes=time_delta_minutes, **kwargs)

    @property
    def checkpointer(self) -> Checkpointer:
        return self._checkpointer

    def _install_sigterm(self) -> None:
        def _handler(signum, frame):
            del signum, frame
            logging.info("Caught SIGTERM: forcing a checkpoint save.")
            self._checkpointer.save(force=True)
        try:
            signal.signal(signal.SIGTERM, _handler)
        except ValueError:  # not the main thread
            logging.warning("Not in the main thread: proceeding without "
                            "checkpointing-on-preemption.")

    def run(self, num_steps: int = None) -> None:
        """Alternates step() and save() (forever, or `num_steps` times: a bounded variant
        for tests and drivers)."""
        self._install_sigterm()
        if isinstance(self._wrapped, core.Learner):
            i = 0
            while num_steps is None or i < num_steps:
                self._wrapped.step()
                self._checkpointer.save()
                i += 1
        else:
            while True:
                self._checkpointer.save()
                time.sleep(self._time_delta_minutes * 60)

    def __dir__(self):
        return dir(self._wrapped)

    def __getattr__(self, name):
        if name.startswith("_"):
            raise AttributeError(name)
        return getattr(self._wrapped, name)
