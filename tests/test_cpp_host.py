"""GPU: the drop-in C++ host (bin/rt_render, host/rt_render.cpp) run as a fresh process.

rt_render is the reference's render loop (CLEngineBase::renderLoop + CLRaytracer::RenderFrame,
CLRaytracer.cpp:12-102) written against the reference-shaped C++ wrapper include/rt_cl_compat.hpp
(CLContext / CLKernel::SetArgument / ExecuteKernel / ReadBuffer / Finish, CLException): scene
load, 14 argument slots, one launch + read-back + finish per frame.  Its output buffer must be
byte-identical to the same frames rendered through the C ABI from Python.
"""
import os
import subprocess

import numpy as np
import pytest

from clrt import _native as N
from hip_helpers import HipRenderer

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(REPO, "mini-opencl-raytracer_amd", "bin", "rt_render")


def _run(tmp_path, *args):
    raw = tmp_path / "out.f32"
    p = subprocess.run([BIN, *args, f"raw={raw}", f"out={tmp_path / 'out.ppm'}"], capture_output=True, text=True,
                       timeout=110)
    assert p.returncode == 0, p.stderr
    assert os.path.getsize(tmp_path / "out.ppm") > 0
    return np.fromfile(raw, np.float32).reshape(-1, 4)


def _python(scene, W, H, frames, bounces, math=N.MATH_SHIPPED):
    r = HipRenderer(scene, W, H, math=math)
    for f in range(1, frames + 1):
        r.frame(f, light_bounces=bounces)
    out = r.result()
    r.close()
    return out


def test_cpp_host_default_scene_equals_c_abi_render(tmp_path, cornell):
    W, H = 320, 180
    got = _run(tmp_path, f"w={W}", f"h={H}", "frames=3", "bounces=9")
    want = _python(cornell, W, H, 3, 9)
    assert got[:, :3].tobytes() == want[:, :3].tobytes()


def test_cpp_host_obj_path_pinned(tmp_path):
    """obj= goes through the C++ OBJ/MTL loader + SAH build (CLOBJloader + CreateBVHTrees)."""
    import clrt.proxy as P
    scene = P.bunny_proxy()
    W, H = 200, 120
    got = _run(tmp_path, f"obj={os.path.join(P.GEN_DIR, 'bunny_proxy.obj')}", f"w={W}", f"h={H}", "frames=2",
               "bounces=4", "math=pinned")
    want = _python(scene, W, H, 2, 4, math=N.MATH_PINNED)
    assert got[:, :3].tobytes() == want[:, :3].tobytes()
