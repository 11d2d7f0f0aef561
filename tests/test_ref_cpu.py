"""CPU: the reference kernel itself, compiled for x86-64, against the C oracle.

oracle/_ref/libref_cpu.so is /root/reference/kernel_bvh.cl built unmodified for the host
(`make -C oracle refcpu`) with the 14 OpenCL builtins it calls supplied under the pinned
semantics (oracle/ref_cpu_host.c).  The C oracle restates that same source under those same
builtins, so the two must agree on every bit: this pins the restatement to the reference's
own code path by path (camera rays, traversal order, BRDF sampling, the three light types,
frame 0's gamma and the accumulation), beyond the live OpenCL runs on the GPU box.
"""
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "oracle"))

import refcpu  # noqa: E402

pytestmark = pytest.mark.skipif(not refcpu.available(), reason="needs oracle/_ref/libref_cpu.so or /root/reference")


def _bits(a):
    return np.ascontiguousarray(a[:, :3]).view(np.uint32)


@pytest.mark.parametrize("light_type,bounces,sky", [(0, 9, 1.0), (1, 5, 0.7), (2, 3, 1.3)])
def test_reference_cpu_equals_oracle(cornell, oracle_mod, light_type, bounces, sky):
    W, H = 123, 77  # odd sizes
    a = np.zeros((W * H, 4), np.float32)
    b = np.zeros((W * H, 4), np.float32)
    for f in range(0, 4):  # frame 0 (plain gamma), then the accumulation
        refcpu.render(cornell, W, H, frame_count=f, light_bounces=bounces, light_type=light_type, skybox=sky,
                      result=a, threads=8)
        oracle_mod.render(cornell, W, H, frame_count=f, light_bounces=bounces, light_type=light_type, skybox=sky,
                          result=b, threads=8)
        assert np.array_equal(_bits(a), _bits(b)), f"frame {f}: {(_bits(a) != _bits(b)).any(axis=1).sum()} pixels"


def test_reference_cpu_work_range_and_camera(cornell, oracle_mod):
    W, H = 96, 64
    cam = ((1.5, -22.0, 9.0), (0.1, 0.98, -0.05), (0.0, 0.0, 1.0))
    a = refcpu.render(cornell, W, H, frame_count=3, light_bounces=4, camera=cam, first=517, last=W * H - 33,
                      threads=4)
    b, _, _, _ = oracle_mod.render(cornell, W, H, frame_count=3, light_bounces=4, camera=cam, first=517,
                                   last=W * H - 33, threads=4)
    assert np.array_equal(_bits(a), _bits(b))


def test_reference_cpu_ui_camera_20_bounces(cornell, oracle_mod):
    """The reference UI's inputs: a rotated + moved camera (CLcamera.h:15-21,
    CLEngineBase.cpp:141-162), the spot light, sky 0.7 and the 20-bounce slider maximum
    (CLui.cpp:240-255), from frameCount 0."""
    from hip_helpers import reference_camera
    cam = reference_camera(1.40, 1.25, moves=("up", "up", "right"))
    W, H = 80, 60
    a = np.zeros((W * H, 4), np.float32)
    b = np.zeros((W * H, 4), np.float32)
    for f in range(0, 3):
        refcpu.render(cornell, W, H, frame_count=f, light_bounces=20, light_type=2, skybox=0.7, camera=cam,
                      result=a, threads=8)
        oracle_mod.render(cornell, W, H, frame_count=f, light_bounces=20, light_type=2, skybox=0.7, camera=cam,
                          result=b, threads=8)
        assert np.array_equal(_bits(a), _bits(b)), f"frame {f}"


def test_reference_cpu_bunny_proxy(oracle_mod):
    sys.path.insert(0, os.path.join(os.path.dirname(HERE), "mini-opencl-raytracer_amd"))
    from clrt import proxy
    sc = proxy.bunny_proxy()
    W, H = 96, 54
    a = refcpu.render(sc, W, H, frame_count=1, light_bounces=6, threads=8)
    b, _, _, _ = oracle_mod.render(sc, W, H, frame_count=1, light_bounces=6, threads=8)
    assert np.array_equal(_bits(a), _bits(b))
