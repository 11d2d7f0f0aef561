"""GPU: one HIP runtime per process (collected last, after every other GPU test ran here).

torch bundles its own libamdhip64.so (ROCm 7.0) under the same SONAME as the /opt/rocm one
librt_hip.so links (7.2); loading both makes the first one loaded serve the whole process.  The
product, its GPU tests and bench.py never import torch, so only /opt/rocm's runtime (and RCCL)
may be mapped.
"""
import sys

import pytest

pytestmark = pytest.mark.gpu


def test_one_hip_runtime_in_process():
    import clrt
    clrt.CLContext(0).release()
    maps = open("/proc/self/maps").read().splitlines()
    hip = {ln.split()[-1] for ln in maps if "libamdhip64" in ln}
    rccl = {ln.split()[-1] for ln in maps if "librccl" in ln}
    assert len(hip) == 1 and all(p.startswith("/opt/rocm") for p in hip), hip
    assert all(p.startswith("/opt/rocm") for p in rccl), rccl
    assert "torch" not in sys.modules
