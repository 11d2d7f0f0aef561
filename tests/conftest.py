"""Shared test setup.

Markers: `gpu` = needs a real MI355X (run by the driver with `-m gpu` on the GPU box);
everything else runs on the CPU container (`-m "not gpu"`).
"""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "mini-opencl-raytracer_amd")
for p in (PKG, os.path.join(REPO, "oracle"), REPO):
    if p not in sys.path:
        sys.path.insert(0, p)

REFERENCE = "/root/reference"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X GPU (HIP)")


@pytest.fixture(scope="session")
def cornell():
    import clrt
    return clrt.scene.cornell()


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle
    oracle.build()
    return oracle


def reference_available() -> bool:
    return os.path.isdir(REFERENCE)
