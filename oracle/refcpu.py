"""ctypes binding of the reference kernel compiled for the CPU (oracle/_ref/libref_cpu.so) --
test infrastructure and bench.py's cpu_baseline only.

`make -C oracle refcpu` builds /root/reference/kernel_bvh.cl unmodified for x86-64 with the
pinned builtins of ref_cpu_host.c; the library then travels with the tree (the GPU box has
no /root/reference and only loads the prebuilt file).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_ref", "libref_cpu.so")
DEFAULT_CAMERA = ((0.0, -25.0, 8.5), (0.0, 1.0, 0.0), (0.0, 0.0, 1.0))
_lib = None


def available() -> bool:
    return os.path.exists(LIB_PATH) or os.path.isdir("/root/reference")


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            if not os.path.isdir("/root/reference"):
                raise FileNotFoundError(f"{LIB_PATH} is not built (needs /root/reference: make -C oracle refcpu)")
            subprocess.run(["make", "-s", "-C", HERE, "refcpu"], check=True)
        L = ctypes.CDLL(LIB_PATH)
        vp = ctypes.c_void_p
        L.ref_cpu_enqueue.argtypes = [vp, vp, vp, vp, ctypes.c_uint, ctypes.c_uint, ctypes.c_uint, ctypes.c_int,
                                      ctypes.c_int, ctypes.c_float, vp, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_int]
        L.ref_cpu_enqueue.restype = ctypes.c_int
        _lib = L
    return _lib


def render(scene, width: int, height: int, frame_count: int = 1, light_bounces: int = 9, light_type: int = 0,
           skybox: float = 1.0, camera=None, result: np.ndarray | None = None, first: int = 0,
           last: int | None = None, threads: int = 0) -> np.ndarray:
    """One launch of the reference KernelEntry over work-items [first, last) on the CPU;
    `result` (W*H x 4 float32) is read-modify-written in place as the reference does."""
    L = lib()
    camera = camera or DEFAULT_CAMERA
    n = width * height
    last = n if last is None else last
    if result is None:
        result = np.zeros((n, 4), np.float32)
    assert result.dtype == np.float32 and result.shape == (n, 4) and result.flags["C_CONTIGUOUS"]
    tris = np.ascontiguousarray(scene.triangles)
    nodes = np.ascontiguousarray(scene.nodes)
    mats = np.ascontiguousarray(scene.materials)
    cam = np.array([*camera[0], 0.0, *camera[1], 0.0, *camera[2], 0.0], np.float32)
    L.ref_cpu_enqueue(result.ctypes.data, tris.ctypes.data, nodes.ctypes.data, mats.ctypes.data, width, height,
                      frame_count & 0xFFFFFFFF, light_bounces, light_type, skybox, cam.ctypes.data, first, last,
                      threads or (os.cpu_count() or 1))
    return result
