import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD GPU (MI355X) and libacme_hip.so")


def pytest_collection_modifyitems(config, items):
    # GPU tests are collected everywhere but skipped (not failed) without a GPU, so
    # `-m "not gpu"` and a plain run both work on the CPU container.
    try:
        import torch
        has_gpu = torch.cuda.is_available()
    except Exception:  # pragma: no cover
        has_gpu = False
    if has_gpu:
        return
    skip = pytest.mark.skip(reason="no GPU visible")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


@pytest.fixture(scope="session")
def oracle_lib():
    """The C replay oracle (built by __graft_entry__.build / tests/_oracle.py)."""
    from tests import _oracle
    return _oracle.load()
