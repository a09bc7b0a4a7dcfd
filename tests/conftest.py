"""Shared test setup.

Markers: ``gpu`` tests need a HIP device and the in-tree ``gym_puzzles_amd/libmrp.so``; they
run on the MI355X box with ``pytest -m gpu``.  Everything else runs on CPU
(``pytest -m "not gpu"``) against the CPU oracle (``oracle/``, test infrastructure only).
"""
from __future__ import annotations

import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) and the built libmrp.so")


@pytest.fixture(scope="session")
def oracle_lib():
    from oracle import oracle
    oracle.build()
    return oracle.lib()


@pytest.fixture(scope="session")
def gpu_lib():
    """The HIP library; a GPU test fails (never falls back) when it is missing."""
    import torch
    assert torch.cuda.is_available(), "gpu test without a visible HIP device"
    from gym_puzzles_amd import _native
    return _native.load()
