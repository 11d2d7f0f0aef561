"""ctypes binding of the CPU ORACLE (oracle/liboracle.so) -- test infrastructure only.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module.
The oracle is a C restatement of /root/reference/kernel_bvh.cl under the pinned math of
include/rt_pinned_math.h (see oracle/rt_oracle.c).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")

_lib = None


class OracleArgs(ctypes.Structure):
    _fields_ = [("tris", ctypes.c_void_p), ("nodes", ctypes.c_void_p), ("mats", ctypes.c_void_p),
                ("width", ctypes.c_uint32), ("height", ctypes.c_uint32), ("frameCount", ctypes.c_uint32),
                ("lightBounces", ctypes.c_int32), ("lightType", ctypes.c_int32),
                ("skyboxIntensity", ctypes.c_float), ("cam", ctypes.c_float * 12)]


def build() -> None:
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        vp = ctypes.c_void_p
        L.oracle_render_mt.argtypes = [ctypes.POINTER(OracleArgs), vp, ctypes.c_uint32, ctypes.c_uint32,
                                       vp, vp, ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]
        L.oracle_render_mt.restype = ctypes.c_int
        for name in ("oracle_pow", "oracle_max", "oracle_min"):
            getattr(L, name).argtypes = [ctypes.c_float, ctypes.c_float]
            getattr(L, name).restype = ctypes.c_float
        for name in ("oracle_sin", "oracle_cos", "oracle_tan"):
            getattr(L, name).argtypes = [ctypes.c_float]
            getattr(L, name).restype = ctypes.c_float
        L.oracle_pixel_cost_mt.argtypes = [ctypes.POINTER(OracleArgs), ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        L.oracle_pixel_cost_mt.restype = ctypes.c_int
        L.oracle_sincos_mismatches.argtypes = [ctypes.c_void_p, ctypes.c_long]
        L.oracle_sincos_mismatches.restype = ctypes.c_long
        L.oracle_hash.argtypes = [ctypes.c_uint32]
        L.oracle_hash.restype = ctypes.c_uint32
        L.oracle_frame_hash.argtypes = [ctypes.c_uint32]
        L.oracle_frame_hash.restype = ctypes.c_uint32
        L.oracle_rand.argtypes = [ctypes.POINTER(ctypes.c_uint32)]
        L.oracle_rand.restype = ctypes.c_float
        L.oracle_ray_triangle.argtypes = [vp, vp, vp, ctypes.c_float, ctypes.POINTER(ctypes.c_float)]
        L.oracle_ray_triangle.restype = ctypes.c_int
        L.oracle_ray_bounds.argtypes = [vp, vp, vp, ctypes.c_float]
        L.oracle_ray_bounds.restype = ctypes.c_int
        _lib = L
    return _lib


def pixel_cost(scene, width: int, height: int, frame_count: int = 1, light_bounces: int = 9, threads: int = 0):
    """Per-pixel work estimate of one frame (uint32[H, W]): visits + 2 tests + 15 rays."""
    L = lib()
    camera = ((0.0, -25.0, 8.5), (0.0, 1.0, 0.0), (0.0, 0.0, 1.0))
    tris = np.ascontiguousarray(scene.triangles)
    nodes = np.ascontiguousarray(scene.nodes)
    mats = np.ascontiguousarray(scene.materials)
    cam = (ctypes.c_float * 12)(*camera[0], 0.0, *camera[1], 0.0, *camera[2], 0.0)
    a = OracleArgs(tris.ctypes.data, nodes.ctypes.data, mats.ctypes.data, width, height,
                   frame_count & 0xFFFFFFFF, light_bounces, 0, 1.0, cam)
    result = np.zeros((width * height, 4), np.float32)
    cost = np.zeros(width * height, np.uint32)
    L.oracle_pixel_cost_mt(ctypes.byref(a), result.ctypes.data, cost.ctypes.data, threads or (os.cpu_count() or 1))
    return cost.reshape(height, width)


def render(scene, width: int, height: int, frame_count: int = 1, light_bounces: int = 9,
           light_type: int = 0, skybox: float = 1.0, camera=None, result: np.ndarray | None = None,
           first: int = 0, last: int | None = None, want_hits: bool = False, threads: int = 0):
    """One KernelEntry launch over work-items [first, last) (default: all W*H).

    Returns (result[W*H,4] float32, hit_ids or None, hit_t or None, counts dict).  The
    result array is updated in place for frame accumulation (frame_count >= 1 reads it).
    """
    L = lib()
    if camera is None:
        camera = ((0.0, -25.0, 8.5), (0.0, 1.0, 0.0), (0.0, 0.0, 1.0))
    n = width * height
    last = n if last is None else last
    if result is None:
        result = np.zeros((n, 4), np.float32)
    assert result.dtype == np.float32 and result.shape == (n, 4) and result.flags["C_CONTIGUOUS"]
    tris = np.ascontiguousarray(scene.triangles)
    nodes = np.ascontiguousarray(scene.nodes)
    mats = np.ascontiguousarray(scene.materials)
    cam = (ctypes.c_float * 12)(*camera[0], 0.0, *camera[1], 0.0, *camera[2], 0.0)
    a = OracleArgs(tris.ctypes.data, nodes.ctypes.data, mats.ctypes.data, width, height,
                   frame_count & 0xFFFFFFFF, light_bounces, light_type, skybox, cam)
    ids = tvals = None
    if want_hits:
        ids = np.full(n, -1, np.int32)
        tvals = np.zeros(n, np.float32)
    counts = (ctypes.c_uint64 * 4)()
    if threads <= 0:
        threads = os.cpu_count() or 1
    L.oracle_render_mt(ctypes.byref(a), result.ctypes.data, first, last,
                       ids.ctypes.data if want_hits else None,
                       tvals.ctypes.data if want_hits else None, counts, threads)
    c = {"rays": counts[0], "node_visits": counts[1], "tri_tests": counts[2], "hits": counts[3]}
    return result, ids, tvals, c
