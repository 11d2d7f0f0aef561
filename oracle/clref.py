"""ctypes binding of oracle/_ref/libclref.so -- the REFERENCE kernel run through OpenCL.

Test infrastructure only.  oracle/_ref/kernel_bvh_{strict,shipped}.co are the unmodified
/root/reference/kernel_bvh.cl compiled by the image's OpenCL compiler for gfx950
(`make -C oracle ref`, in the container that has the reference); libclref.so drives them
through the system OpenCL runtime on the GPU box.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF_DIR = os.path.join(HERE, "_ref")
LIB = os.path.join(REF_DIR, "libclref.so")
VARIANTS = {
    "strict": os.path.join(REF_DIR, "kernel_bvh_strict.co"),
    "shipped": os.path.join(REF_DIR, "kernel_bvh_shipped.co"),
    # built by the OpenCL runtime itself from source, as the reference host does
    # (oracle/offline_build.c: clBuildProgram(" -I . ") for an offline gfx950 device)
    "runtime": os.path.join(REF_DIR, "kernel_bvh_runtime.co"),
}


class _Scene(ctypes.Structure):
    _fields_ = [("tris", ctypes.c_void_p), ("tris_bytes", ctypes.c_size_t),
                ("nodes", ctypes.c_void_p), ("nodes_bytes", ctypes.c_size_t),
                ("mats", ctypes.c_void_p), ("mats_bytes", ctypes.c_size_t),
                ("width", ctypes.c_uint32), ("height", ctypes.c_uint32),
                ("lightBounces", ctypes.c_int32), ("lightType", ctypes.c_int32),
                ("skyboxIntensity", ctypes.c_float), ("cam", ctypes.c_float * 12)]


def available() -> tuple[bool, str]:
    for p in [LIB] + list(VARIANTS.values()):
        if not os.path.exists(p):
            return False, f"{p} not built (needs /root/reference at build time)"
    return True, ""


class ReferenceKernel:
    """The reference KernelEntry (and the PrimaryHitEntry harness) on the OpenCL GPU device."""

    def __init__(self, variant: str = "strict"):
        L = ctypes.CDLL(LIB)
        L.clref_open.restype = ctypes.c_void_p
        L.clref_open.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_int)]
        L.clref_close.argtypes = [ctypes.c_void_p]
        L.clref_device_name.restype = ctypes.c_char_p
        L.clref_device_name.argtypes = [ctypes.c_void_p]
        L.clref_render.argtypes = [ctypes.c_void_p, ctypes.POINTER(_Scene), ctypes.c_uint32, ctypes.c_uint32,
                                   ctypes.c_void_p]
        L.clref_primary_hits.argtypes = [ctypes.c_void_p, ctypes.POINTER(_Scene), ctypes.c_uint32,
                                         ctypes.c_void_p, ctypes.c_void_p]
        self.L = L
        err = ctypes.c_int(0)
        self.h = L.clref_open(VARIANTS[variant].encode(), ctypes.byref(err))
        if not self.h:
            raise RuntimeError(f"clref_open({variant}) failed: cl error {err.value}")
        self.device_name = L.clref_device_name(self.h).decode(errors="replace")

    def _scene(self, scene, W, H, lb, lt, sky, camera):
        self._keep = [np.ascontiguousarray(a) for a in (scene.triangles, scene.nodes, scene.materials)]
        t, n, m = self._keep
        cam = (ctypes.c_float * 12)(*camera[0], 0.0, *camera[1], 0.0, *camera[2], 0.0)
        return _Scene(t.ctypes.data, t.nbytes, n.ctypes.data, n.nbytes, m.ctypes.data, m.nbytes,
                      W, H, lb, lt, sky, cam)

    def render(self, scene, W, H, frames=(1,), light_bounces=9, light_type=0, skybox=1.0,
               camera=((0.0, -25.0, 8.5), (0.0, 1.0, 0.0), (0.0, 0.0, 1.0)), result=None):
        """KernelEntry for frames min(frames)..max(frames) into one buffer.  `result` (W*H x 4
        float32) is the buffer's starting content (default zeros), as after earlier frames of
        an interactive session; a new array is returned."""
        s = self._scene(scene, W, H, light_bounces, light_type, skybox, camera)
        out = np.zeros((W * H, 4), np.float32) if result is None else np.array(result, np.float32, copy=True)
        assert out.shape == (W * H, 4)
        f0, f1 = min(frames), max(frames)
        rc = self.L.clref_render(self.h, ctypes.byref(s), f0, f1, out.ctypes.data)
        if rc != 0:
            raise RuntimeError(f"clref_render: cl error {rc}")
        return out

    def primary_hits(self, scene, W, H, frame=1,
                     camera=((0.0, -25.0, 8.5), (0.0, 1.0, 0.0), (0.0, 0.0, 1.0))):
        s = self._scene(scene, W, H, 1, 0, 1.0, camera)
        ids = np.zeros(W * H, np.int32)
        t = np.zeros(W * H, np.float32)
        rc = self.L.clref_primary_hits(self.h, ctypes.byref(s), frame, ids.ctypes.data, t.ctypes.data)
        if rc != 0:
            raise RuntimeError(f"clref_primary_hits: cl error {rc}")
        return ids, t

    def close(self):
        if self.h:
            self.L.clref_close(self.h)
            self.h = None
