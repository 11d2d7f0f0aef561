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


@pytest.fixture(scope="session", autouse=True)
def _torch_hip_first(request):
    """torch bundles its own HIP runtime next to the one librt_hip.so links; torch's must
    initialise first in a process (as bench.py does), or it reports no GPUs.  Only on a
    GPU session (a `-m gpu` selection); a CPU run never touches HIP."""
    markexpr = request.config.getoption("-m") or ""
    if "gpu" in markexpr and "not gpu" not in markexpr:
        import torch
        if torch.cuda.is_available():
            torch.zeros(1, device="cuda:0")
    yield
