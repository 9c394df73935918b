"""Minimal nest utilities (the subset of dm-tree the adders and datasets use).

Nests are tuples, lists, dicts (sorted keys), namedtuples and leaves.  Flattening order
matches dm-tree: dicts by sorted key, sequences in order.
"""

from __future__ import annotations

from typing import Any, Callable, List


def _is_namedtuple(x) -> bool:
    return isinstance(x, tuple) and hasattr(x, "_fields")


def is_nested(x) -> bool:
    return isinstance(x, (list, tuple, dict))


def flatten(nest) -> List[Any]:
    out: List[Any] = []

    def rec(x):
        if isinstance(x, dict):
            for k in sorted(x):
                rec(x[k])
        elif isinstance(x, (list, tuple)):
            for v in x:
                rec(v)
        else:
            out.append(x)

    rec(nest)
    return out


def unflatten_as(structure, flat):
    it = iter(flat)

    def rec(s):
        if isinstance(s, dict):
            return type(s)((k, rec(s[k])) for k in sorted(s))
        if _is_namedtuple(s):
            return type(s)(*[rec(v) for v in s])
        if isinstance(s, (list, tuple)):
            return type(s)(rec(v) for v in s)
        return next(it)

    out = rec(structure)
    rest = list(it)
    if rest:
        raise ValueError(f"{len(rest)} leaves left over when unflattening")
    return out


def map_structure(fn: Callable, *nests):
    flats = [flatten(n) for n in nests]
    if any(len(f) != len(flats[0]) for f in flats):
        raise ValueError("nests do not have the same number of leaves")
    return unflatten_as(nests[0], [fn(*xs) for xs in zip(*flats)])
