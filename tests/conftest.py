"""Shared test setup.

Markers: `gpu` = needs an MI355X (run on the GPU box with `pytest -m gpu`);
everything else runs on the CPU container (`pytest -m "not gpu"`).
Parity tests compare the HIP path (through the C ABI) with the oracle
(oracle/, pinned to scipy golden vectors in tests/golden/).
"""
import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
LIB_DIR = os.path.join(ROOT, "xm-audio-utils_amd", "lib")
for p in (os.path.join(ROOT, "oracle"), os.path.join(ROOT, "xm-audio-utils_amd"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X GPU (gfx950)")


def golden(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def manifest():
    with open(os.path.join(GOLDEN, "MANIFEST.json")) as fh:
        return json.load(fh)


def bits_equal(a, b):
    a = np.ascontiguousarray(a)
    b = np.ascontiguousarray(b)
    return a.shape == b.shape and a.dtype == b.dtype and np.array_equal(a.view(np.uint8), b.view(np.uint8))


def ulp_diff(a, b):
    """Max ULP distance between two float32 arrays (ordered-int mapping)."""
    ai = np.ascontiguousarray(a, np.float32).view(np.int32).astype(np.int64)
    bi = np.ascontiguousarray(b, np.float32).view(np.int32).astype(np.int64)
    ai = np.where(ai < 0, -(ai & 0x7FFFFFFF), ai)
    bi = np.where(bi < 0, -(bi & 0x7FFFFFFF), bi)
    return int(np.max(np.abs(ai - bi))) if ai.size else 0


@pytest.fixture(scope="session")
def xm():
    import xmaudio
    return xmaudio


@pytest.fixture(scope="session")
def gpu(xm):
    n = xm.device_count()
    assert n > 0, "gpu-marked test needs a HIP device (run on the MI355X box)"
    return 0
