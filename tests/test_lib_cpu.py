"""The C-ABI library loads without a GPU and exports every symbol include/acme_hip.h
declares (no compute calls)."""

import ctypes
import os
import re

from acme_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    text = open(os.path.join(ROOT, "include", "acme_hip.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(acme_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_and_library_exports_all():
    names = _declared()
    assert len(names) >= 25
    L = _lib.lib()
    for n in names:
        assert hasattr(L, n), f"{n} declared in include/acme_hip.h but not exported"
        assert n in _lib.EXPORTED_SYMBOLS, f"{n} has no ctypes signature in acme_amd/_lib.py"


def test_library_identity():
    L = _lib.lib()
    assert L.acme_target_arch() == b"gfx950"
    assert L.acme_version().startswith(b"acme_amd")


def test_error_status_mapping():
    L = _lib.lib()
    # Invalid config fails in argument validation before touching the GPU.
    cfg = _lib.ReplayConfig()
    cfg.capacity = 0
    h = ctypes.c_void_p()
    rc = L.acme_replay_create(ctypes.byref(cfg), ctypes.byref(h))
    assert rc == _lib.ACME_ERR_INVALID
    assert b"capacity" in L.acme_last_error()
    try:
        _lib.check(rc)
    except ValueError as e:
        assert "capacity" in str(e)
    else:  # pragma: no cover
        raise AssertionError("expected ValueError")
