"""Host scene pipeline: OBJ/MTL -> triangles -> SAH BVH (librt_scene.so).

Python face of ``CLOBJloader::Load`` + ``CLBVHScene::CreateBVHTrees``
(/root/reference/CLOBJloader.cpp:10-176, CLBVHnode.cpp:7-207).  The arrays are numpy
structured arrays with the exact device byte layout (CLTriangle 256 B, CLLinearBVHNode
48 B, CLMaterial 64 B).
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass

import numpy as np

from ._native import (MATERIAL_DTYPE, NODE_DTYPE, TRIANGLE_DTYPE, RTError, check, scene_lib)


@dataclass
class Scene:
    triangles: np.ndarray  # TRIANGLE_DTYPE, BVH leaf order (after build)
    nodes: np.ndarray      # NODE_DTYPE, depth-first order (empty when not built)
    materials: np.ndarray  # MATERIAL_DTYPE
    max_prims_in_node: int = 4

    @property
    def n_triangles(self) -> int:
        return int(self.triangles.shape[0])

    def tree_stats(self) -> dict:
        """Maximum leaf depth (root = 0), leaf count, largest leaf."""
        if self.nodes.size == 0:
            raise RTError("scene has no BVH", -30)
        depth, leaves, maxp = 0, 0, 0
        stack = [(0, 0)]
        while stack:
            i, d = stack.pop()
            n = self.nodes[i]
            if n["nPrimitives"] > 0:
                leaves += 1
                depth = max(depth, d)
                maxp = max(maxp, int(n["nPrimitives"]))
            else:
                stack.append((i + 1, d + 1))
                stack.append((int(n["offset"]), d + 1))
        return {"max_depth": depth, "leaves": leaves, "max_leaf_prims": maxp}


def _copy_out(lib, handle) -> tuple:
    p = ctypes.c_void_p()
    n = ctypes.c_size_t()
    out = []
    for fn, dt in (("rtsGetTriangles", TRIANGLE_DTYPE), ("rtsGetNodes", NODE_DTYPE),
                   ("rtsGetMaterials", MATERIAL_DTYPE)):
        check(getattr(lib, fn)(handle, ctypes.byref(p), ctypes.byref(n)), fn)
        if n.value == 0:
            out.append(np.zeros(0, dt))
            continue
        buf = (ctypes.c_uint8 * (n.value * dt.itemsize)).from_address(p.value)
        out.append(np.frombuffer(bytes(buf), dtype=dt).copy())
    return tuple(out)


def load_obj(path: str, max_prims_in_node: int = 4, build: bool = True) -> Scene:
    """CLOBJloader::Load(path, maxPrimitivesInNode) then CreateBVHTrees (CLEngineBase.cpp:173-179)."""
    lib = scene_lib()
    h = ctypes.c_void_p()
    if build:
        rc = lib.rtsLoadOBJ(path.encode(), int(max_prims_in_node), ctypes.byref(h))
    else:
        rc = lib.rtsLoadOBJUnbuilt(path.encode(), ctypes.byref(h))
    check(rc, f"Failed to load scene file {path}")
    try:
        tris, nodes, mats = _copy_out(lib, h)
    finally:
        lib.rtsRelease(h)
    return Scene(tris, nodes, mats, max_prims_in_node)


def build_bvh(triangles: np.ndarray, materials: np.ndarray, max_prims_in_node: int = 4) -> Scene:
    """CLBVHScene::CreateBVHTrees over caller-supplied triangles (file order)."""
    lib = scene_lib()
    tris = np.ascontiguousarray(triangles, dtype=TRIANGLE_DTYPE)
    mats = np.ascontiguousarray(materials, dtype=MATERIAL_DTYPE)
    h = ctypes.c_void_p()
    check(lib.rtsBuildFromTriangles(tris.ctypes.data, tris.shape[0], mats.ctypes.data, mats.shape[0],
                                    int(max_prims_in_node), ctypes.byref(h)), "CreateBVHTrees")
    try:
        t, n, m = _copy_out(lib, h)
    finally:
        lib.rtsRelease(h)
    return Scene(t, n, m, max_prims_in_node)


def build_bvh_device(triangles: np.ndarray, materials: np.ndarray, max_prims_in_node: int = 4,
                     device: int = 0, method: str = "ploc") -> Scene:
    """Device-side BVH build (rtBuildBVHEx): same array contract as build_bvh,
    a PLOC ("ploc") or linear ("lbvh") BVH instead of the reference's SAH tree.  Needs a GPU."""
    from . import _native as N
    from .device import CLContext
    tris = np.ascontiguousarray(triangles, dtype=TRIANGLE_DTYPE)
    n = tris.shape[0]
    ctx = CLContext(device)
    try:
        tb = ctx.create_buffer(N.MEM_READ_WRITE | N.MEM_COPY_HOST_PTR, tris.nbytes, tris)
        nb = ctx.create_buffer(N.MEM_READ_WRITE, max(1, 2 * n - 1) * NODE_DTYPE.itemsize)
        count = ctx.BuildBVH(tb, n, max_prims_in_node, nb, {"lbvh": N.BVH_LBVH, "ploc": N.BVH_PLOC}[method])
        out_t = np.empty_like(tris)
        out_n = np.empty(count, NODE_DTYPE)
        ctx.ReadBuffer(tb, out_t, blocking=True)
        ctx.ReadBuffer(nb, out_n, out_n.nbytes, blocking=True)
        tb.release()
        nb.release()
    finally:
        ctx.release()
    return Scene(out_t, out_n, np.ascontiguousarray(materials, dtype=MATERIAL_DTYPE), max_prims_in_node)


def save_scene(scene: Scene, path: str) -> None:
    """Binary scene cache (rtsSaveScene): the three arrays exactly as built."""
    lib = scene_lib()
    t = np.ascontiguousarray(scene.triangles, dtype=TRIANGLE_DTYPE)
    n = np.ascontiguousarray(scene.nodes, dtype=NODE_DTYPE)
    m = np.ascontiguousarray(scene.materials, dtype=MATERIAL_DTYPE)
    h = ctypes.c_void_p()
    check(lib.rtsFromArrays(t.ctypes.data, t.shape[0], n.ctypes.data, n.shape[0], m.ctypes.data, m.shape[0],
                            int(scene.max_prims_in_node), ctypes.byref(h)), "rtsFromArrays")
    try:
        check(lib.rtsSaveScene(h, path.encode()), f"Failed to write scene cache {path}")
    finally:
        lib.rtsRelease(h)


def load_scene(path: str, max_prims_in_node: int = 4) -> Scene:
    """Read a binary scene cache written by save_scene / rtsSaveScene."""
    lib = scene_lib()
    h = ctypes.c_void_p()
    check(lib.rtsLoadScene(path.encode(), ctypes.byref(h)), f"Failed to load scene cache {path}")
    try:
        tris, nodes, mats = _copy_out(lib, h)
    finally:
        lib.rtsRelease(h)
    return Scene(tris, nodes, mats, max_prims_in_node)


_REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CORNELL_NPZ = os.path.join(_REPO, "scenes", "cornell_scene.npz")


def cornell(max_prims_in_node: int = 4) -> Scene:
    """The benchmark scene: /root/reference/cornell.obj as parsed by load_obj (stored in
    scenes/cornell_scene.npz so it is available where the reference is not), built with
    maxPrimitivesInNode = 4 as CLEngineBase::renderLoop does (CLEngineBase.cpp:175-179)."""
    z = np.load(CORNELL_NPZ, allow_pickle=False)
    tris = z["triangles"].view(TRIANGLE_DTYPE)
    mats = z["materials"].view(MATERIAL_DTYPE)
    return build_bvh(tris, mats, max_prims_in_node)
