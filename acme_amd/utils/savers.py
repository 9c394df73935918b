"""Checkpointing of Saveable objects (semantics of acme/tf/savers.py:52-167: time-gated
save, restore-on-construct; acme/jax/savers.py:44-84: arrays to an .npz).

A Saveable's state is a nest of dicts whose leaves are numpy arrays / scalars; it is
flattened to '/'-joined keys and written atomically (tmp + rename) with numpy (no
pickling; loads use allow_pickle=False)."""

from __future__ import annotations

import os
import time
from typing import Dict, Mapping

import numpy as np

from acme_amd import core


def _flatten(d: Mapping, prefix: str = "") -> Dict[str, np.ndarray]:
    out = {}
    for k, v in d.items():
        key = f"{prefix}{k}"
        if isinstance(v, Mapping):
            out.update(_flatten(v, key + "/"))
        else:
            out[key] = np.asarray(v)
    return out


def _unflatten(flat: Mapping[str, np.ndarray]) -> Dict:
    out: Dict = {}
    for key, v in flat.items():
        node = out
        parts = key.split("/")
        # Parameter names contain '/', so only split the known nesting levels: the first
        # component (object) and the state keys below it; rejoin the rest.
        head, rest = parts[0], parts[1:]
        node = out.setdefault(head, {})
        if len(rest) >= 2 and rest[0] in ("network", "target_network"):
            node.setdefault(rest[0], {})["/".join(rest[1:])] = v
        elif len(rest) >= 3 and rest[0] == "optimizer" and rest[1] in ("m", "v"):
            node.setdefault("optimizer", {}).setdefault(rest[1], {})["/".join(rest[2:])] = v
        elif len(rest) == 2 and rest[0] == "optimizer":
            node.setdefault("optimizer", {})[rest[1]] = v.item() if v.ndim == 0 else v
        else:
            node["/".join(rest)] = v.item() if v.ndim == 0 else v
    return out


class Checkpointer:

    def __init__(self, objects_to_save: Mapping[str, core.Saveable], directory: str,
                 time_delta_minutes: float = 10.0, enable_checkpointing: bool = True):
        self._objects = dict(objects_to_save)
        self._dir = directory
        self._delta = time_delta_minutes * 60.0
        self._last = time.time()
        self._enabled = enable_checkpointing
        self._path = os.path.join(directory, "checkpoint.npz")
        if enable_checkpointing and os.path.exists(self._path):
            self.restore()

    def save(self, force: bool = False) -> bool:
        if not self._enabled or (not force and time.time() - self._last < self._delta):
            return False
        os.makedirs(self._dir, exist_ok=True)
        flat = {}
        for name, obj in self._objects.items():
            flat.update(_flatten(obj.save(), name + "/"))
        tmp = self._path + ".tmp.npz"
        np.savez(tmp, **flat)
        os.replace(tmp, self._path)
        self._last = time.time()
        return True

    def restore(self) -> None:
        with np.load(self._path, allow_pickle=False) as z:
            tree = _unflatten({k: z[k] for k in z.files})
        for name, obj in self._objects.items():
            if name in tree:
                obj.restore(tree[name])
