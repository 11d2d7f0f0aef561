"""Output/format step (include/rt_image.h via librt_scene.so): accumulation buffer -> image.

Replaces the reference's GL texture display (CLRaytracer.cpp:25-26, :64-67): 8-bit RGB,
clamp to [0, 1] (NaN -> 0), rows flipped (row 0 of the kernel's buffer is the bottom).
"""
from __future__ import annotations

import ctypes

import numpy as np

from ._native import check, scene_lib

IMAGE_EXPORTS = ("rtiToRGB8", "rtiWritePPM", "rtiWritePNG", "rtiSaveAccum", "rtiLoadAccum")  # include/rt_image.h


def _px(pixels: np.ndarray, W: int, H: int) -> np.ndarray:
    a = np.ascontiguousarray(pixels, dtype=np.float32).reshape(-1)
    if a.size != W * H * 4:
        raise ValueError(f"expected {W}x{H} float4 pixels, got {a.size} floats")
    return a


def _protos(lib):
    if getattr(lib, "_rti_ready", False):
        return lib
    fp = ctypes.POINTER(ctypes.c_float)
    lib.rtiToRGB8.argtypes = [fp, ctypes.c_uint, ctypes.c_uint, ctypes.POINTER(ctypes.c_ubyte)]
    lib.rtiWritePPM.argtypes = [ctypes.c_char_p, fp, ctypes.c_uint, ctypes.c_uint]
    lib.rtiWritePNG.argtypes = [ctypes.c_char_p, fp, ctypes.c_uint, ctypes.c_uint]
    u = ctypes.POINTER(ctypes.c_uint)
    lib.rtiSaveAccum.argtypes = [ctypes.c_char_p, fp, ctypes.c_uint, ctypes.c_uint, ctypes.c_uint]
    lib.rtiLoadAccum.argtypes = [ctypes.c_char_p, fp, u, u, u]
    for f in (lib.rtiToRGB8, lib.rtiWritePPM, lib.rtiWritePNG, lib.rtiSaveAccum, lib.rtiLoadAccum):
        f.restype = ctypes.c_int
    lib._rti_ready = True
    return lib


def to_rgb8(pixels: np.ndarray, W: int, H: int) -> np.ndarray:
    """(H, W, 3) uint8, top row first."""
    lib = _protos(scene_lib())
    a = _px(pixels, W, H)
    out = np.empty((H, W, 3), np.uint8)
    check(lib.rtiToRGB8(a.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), W, H,
                        out.ctypes.data_as(ctypes.POINTER(ctypes.c_ubyte))), "rtiToRGB8")
    return out


def write_ppm(path: str, pixels: np.ndarray, W: int, H: int) -> None:
    lib = _protos(scene_lib())
    a = _px(pixels, W, H)
    check(lib.rtiWritePPM(path.encode(), a.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), W, H), "rtiWritePPM")


def write_png(path: str, pixels: np.ndarray, W: int, H: int) -> None:
    lib = _protos(scene_lib())
    a = _px(pixels, W, H)
    check(lib.rtiWritePNG(path.encode(), a.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), W, H), "rtiWritePNG")


def save_accum(path: str, pixels: np.ndarray, W: int, H: int, next_frame: int) -> None:
    """rtiSaveAccum: the accumulation buffer + the frame count the next render uses."""
    lib = _protos(scene_lib())
    a = _px(pixels, W, H)
    check(lib.rtiSaveAccum(path.encode(), a.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), W, H, int(next_frame)),
          "rtiSaveAccum")


def load_accum(path: str) -> tuple[np.ndarray, int]:
    """rtiLoadAccum: (W*H x 4 float32 pixels, next frame count)."""
    lib = _protos(scene_lib())
    W, H, f = ctypes.c_uint(), ctypes.c_uint(), ctypes.c_uint()
    check(lib.rtiLoadAccum(path.encode(), None, ctypes.byref(W), ctypes.byref(H), ctypes.byref(f)), "rtiLoadAccum")
    px = np.empty((W.value * H.value, 4), np.float32)
    check(lib.rtiLoadAccum(path.encode(), px.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), ctypes.byref(W),
                           ctypes.byref(H), ctypes.byref(f)), "rtiLoadAccum")
    return px, int(f.value)

