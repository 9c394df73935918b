"""Builds and binds the C replay oracle (oracle/replay_oracle.c) — test infrastructure."""

import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "oracle", "replay_oracle.c")
OUT = os.path.join(ROOT, "oracle", "build", "libreplay_oracle.so")

_L = None


def build() -> str:
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    if not os.path.exists(OUT) or os.path.getmtime(OUT) < os.path.getmtime(SRC):
        subprocess.check_call(["gcc", "-O2", "-ffp-contract=off", "-fPIC", "-shared", "-Wall",
                               "-o", OUT, SRC, "-lm"])
    return OUT


def load():
    global _L
    if _L is None:
        if not os.path.exists(OUT):
            build()
        L = ctypes.CDLL(OUT)
        vp, i64, u64, f64 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_uint64, ctypes.c_double
        L.oracle_philox4x32_10.argtypes = [vp, vp, vp]
        L.oracle_uniform.restype = f64
        L.oracle_uniform.argtypes = [u64, u64, ctypes.c_uint32]
        L.oracle_log.restype = f64
        L.oracle_log.argtypes = [f64]
        L.oracle_exp.restype = f64
        L.oracle_exp.argtypes = [f64]
        L.oracle_priority_weight.restype = f64
        L.oracle_priority_weight.argtypes = [f64, f64]
        L.oracle_table_new.restype = vp
        L.oracle_table_new.argtypes = [i64, ctypes.c_int, f64, u64]
        L.oracle_table_free.argtypes = [vp]
        L.oracle_table_insert.restype = i64
        L.oracle_table_insert.argtypes = [vp, i64, vp]
        L.oracle_table_update.argtypes = [vp, i64, vp, vp]
        L.oracle_table_sample.restype = ctypes.c_int
        L.oracle_table_sample.argtypes = [vp, i64, u64, vp, vp, vp, vp, vp]
        L.oracle_table_size.restype = i64
        L.oracle_table_size.argtypes = [vp]
        L.oracle_table_leaves.restype = ctypes.POINTER(ctypes.c_double)
        L.oracle_table_leaves.argtypes = [vp]
        L.oracle_table_total.restype = f64
        L.oracle_table_total.argtypes = [vp]
        _L = L
    return _L


def philox(ctr, key):
    L = load()
    c = np.asarray(ctr, np.uint32)
    k = np.asarray(key, np.uint32)
    o = np.zeros(4, np.uint32)
    L.oracle_philox4x32_10(c.ctypes.data, k.ctypes.data, o.ctypes.data)
    return o


class OracleTable:
    def __init__(self, capacity, prioritized, alpha, seed):
        self.L = load()
        self.capacity = capacity
        self.h = self.L.oracle_table_new(capacity, 1 if prioritized else 0, alpha, seed)

    def __del__(self):
        if getattr(self, "h", None):
            self.L.oracle_table_free(self.h)
            self.h = None

    def insert(self, priorities):
        p = np.ascontiguousarray(priorities, np.float64)
        return self.L.oracle_table_insert(self.h, len(p), p.ctypes.data)

    def update(self, keys, priorities):
        k = np.ascontiguousarray(keys, np.uint64)
        p = np.ascontiguousarray(priorities, np.float64)
        self.L.oracle_table_update(self.h, len(k), k.ctypes.data, p.ctypes.data)

    def sample(self, batch, step):
        out = dict(slots=np.empty(batch, np.int64), keys=np.empty(batch, np.uint64),
                   probabilities=np.empty(batch, np.float64),
                   table_size=np.empty(batch, np.int64), priorities=np.empty(batch, np.float64))
        rc = self.L.oracle_table_sample(self.h, batch, step, out["slots"].ctypes.data,
                                        out["keys"].ctypes.data, out["probabilities"].ctypes.data,
                                        out["table_size"].ctypes.data,
                                        out["priorities"].ctypes.data)
        if rc != 0:
            raise RuntimeError("oracle: empty table")
        return out

    def leaves(self):
        p = self.L.oracle_table_leaves(self.h)
        n = ((self.capacity + 63) // 64) * 64
        return np.ctypeslib.as_array(p, shape=(n,)).copy()

    def total(self):
        return self.L.oracle_table_total(self.h)
