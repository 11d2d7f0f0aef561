"""ctypes bindings of the two product libraries (include/rt_hip.h, include/rt_scene.h).

The libraries are built in-tree by ``make -C mini-opencl-raytracer_amd`` (or
``__graft_entry__.build()``).  Nothing here falls back to a CPU path: if
``librt_hip.so`` is missing or no GPU is visible, the calls fail with ``RTError``.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

_PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_DIR = os.path.join(_PKG_ROOT, "lib")
HIP_LIB_PATH = os.environ.get("RT_HIP_LIB") or os.path.join(LIB_DIR, "librt_hip.so")
SCENE_LIB_PATH = os.path.join(LIB_DIR, "librt_scene.so")

# ---- status codes (include/rt_status.h == cl_int codes, CLutils.h:31-105) -------------
RT_SUCCESS = 0
_ERROR_NAMES = {
    0: "CL_SUCCESS", -1: "CL_DEVICE_NOT_FOUND", -4: "CL_MEM_OBJECT_ALLOCATION_FAILURE",
    -5: "CL_OUT_OF_RESOURCES", -6: "CL_OUT_OF_HOST_MEMORY", -30: "CL_INVALID_VALUE",
    -33: "CL_INVALID_DEVICE", -34: "CL_INVALID_CONTEXT", -36: "CL_INVALID_COMMAND_QUEUE",
    -37: "CL_INVALID_HOST_PTR", -38: "CL_INVALID_MEM_OBJECT", -46: "CL_INVALID_KERNEL_NAME",
    -48: "CL_INVALID_KERNEL", -49: "CL_INVALID_ARG_INDEX", -50: "CL_INVALID_ARG_VALUE",
    -51: "CL_INVALID_ARG_SIZE", -52: "CL_INVALID_KERNEL_ARGS", -59: "CL_INVALID_OPERATION",
    -61: "CL_INVALID_BUFFER_SIZE", -63: "CL_INVALID_GLOBAL_WORK_SIZE",
    -1001: "RT_FILE_NOT_FOUND", -1002: "RT_PARSE_ERROR",
}


def error_string(code: int) -> str:
    """GetClErrorString (CLutils.h:31-105)."""
    return _ERROR_NAMES.get(int(code), "Unknown OpenCL error")


class RTError(RuntimeError):
    """CLException (CLutils.h:107-114): ``message (CL_NAME)`` plus the numeric code."""

    def __init__(self, message: str, code: int):
        super().__init__(f"{message} ({error_string(code)})")
        self.code = int(code)


def check(code: int, message: str) -> None:
    if code != RT_SUCCESS:
        raise RTError(message, code)


# ---- rt_cl_types.h as numpy dtypes ------------------------------------------------------
FLOAT3 = np.dtype((np.float32, 4))  # OpenCL float3: 16-byte slot
VERTEX_DTYPE = np.dtype([("position", FLOAT3), ("uv", FLOAT3), ("normal", FLOAT3),
                         ("tangent_s", FLOAT3), ("tangent_t", FLOAT3)])
TRIANGLE_DTYPE = np.dtype([("v1", VERTEX_DTYPE), ("v2", VERTEX_DTYPE), ("v3", VERTEX_DTYPE),
                           ("mtlIndex", np.uint32), ("padding", np.uint32, (3,))])
NODE_DTYPE = np.dtype([("bmin", FLOAT3), ("bmax", FLOAT3), ("offset", np.uint32),
                       ("nPrimitives", np.uint16), ("axis", np.uint8), ("pad", np.uint8, (9,))])
MATERIAL_DTYPE = np.dtype([("diffuse", FLOAT3), ("specular", FLOAT3), ("emission", FLOAT3),
                           ("type", np.uint32), ("roughness", np.float32), ("ior", np.float32),
                           ("padding", np.int32)])
assert VERTEX_DTYPE.itemsize == 80 and TRIANGLE_DTYPE.itemsize == 256
assert NODE_DTYPE.itemsize == 48 and MATERIAL_DTYPE.itemsize == 64

# RenderKernelArgument_t (CLutils.h:11-27)
BUFFER_OUT, BUFFER_SCENE, BUFFER_NODE, BUFFER_MATERIAL = 0, 1, 2, 3
WIDTH, HEIGHT, FRAME_COUNT, FRAME_SEED = 4, 5, 6, 7
LIGHT_BOUNCES, LIGHT_TYPE, SKYBOX_INTENSITY = 8, 9, 10
CAMERA_POS, CAMERA_FRONT, CAMERA_UP = 11, 12, 13

MEM_READ_WRITE, MEM_WRITE_ONLY, MEM_READ_ONLY, MEM_COPY_HOST_PTR = 1, 2, 4, 32
MATH_PINNED, MATH_DEVICELIB, MATH_SHIPPED = 0, 1, 2
SCHED_TILES, SCHED_STEP, SCHED_WAVEFRONT = 0, 2, 4  # (1, 3: retired schedules)
BVH_LBVH, BVH_PLOC = 0, 1  # rtBuildBVHEx
# rt_tuning (rt_hip.h): scheduling parameters, results unchanged
TUNING = {"refill_min": 0, "shade_min": 1, "refill_min_global": 2, "shade_min_global": 3,
          "step_weight_node": 4, "step_weight_leaf": 5, "chunk_pixels": 6, "tail_chunk": 7,
          "bulk_percent": 8, "top_nodes": 9,
          "tile_major": 13, "perframe_sky": 14, "wf_refill_min": 15, "wf_streams_per_cu": 16,
          "wf_top_nodes": 17, "global_oct": 18, "perframe_defer": 19, "max_blocks": 20,
          "perframe_defer_min": 21, "perframe_batch": 23, "step_weight_node_global": 24,
          "step_weight_leaf_global": 25}


class Stats(ctypes.Structure):
    _fields_ = [("rays", ctypes.c_uint64), ("node_visits", ctypes.c_uint64),
                ("tri_tests", ctypes.c_uint64), ("hits", ctypes.c_uint64),
                ("launches", ctypes.c_uint64), ("kernel_ms", ctypes.c_double),
                ("cycles_refill", ctypes.c_uint64), ("cycles_traverse", ctypes.c_uint64),
                ("cycles_shade", ctypes.c_uint64), ("cycles_total", ctypes.c_uint64),
                ("sched", ctypes.c_uint64 * 12), ("accum_ms", ctypes.c_double),
                ("render_period_ms", ctypes.c_double)]


class Rect(ctypes.Structure):
    """rt_rect (rt_hip.h): one 2-D copy of the band gather's pack plan."""
    _fields_ = [("img_offset", ctypes.c_uint64), ("img_pitch", ctypes.c_uint64), ("width", ctypes.c_uint64),
                ("rows", ctypes.c_uint64), ("stage_offset", ctypes.c_uint64)]


COMM_ID_BYTES = 128
COMM_SUM, COMM_MAX = 0, 1
COMM_TRANSPORT_COPY_ENGINES, COMM_TRANSPORT_RCCL, COMM_TRANSPORT_COPY_ENGINES_IPC = 0, 1, 2
COMM_TRANSPORT_NAMES = {-1: "none", COMM_TRANSPORT_COPY_ENGINES: "copy engines",
                        COMM_TRANSPORT_RCCL: "RCCL", COMM_TRANSPORT_COPY_ENGINES_IPC: "copy engines (IPC links)"}
# rt_comm_status.fallback_reason
COMM_FALLBACK_NAMES = {0: None, 1: "no peer access", 2: "IPC handle export/map failed",
                       3: "link trial round failed"}
COMM_OPT_FAIL_LINKS = 1  # test hook (rtCommSetOption)
COMM_OPT_REPLAN_PERIOD = 2  # gathers per plan before a collective re-plan (rtCommSetOption)
COMM_OPT_SYSTEM_ACQUIRE = 3  # force the root's system-scope acquire after a gather (rtCommSetOption)


class CommStatus(ctypes.Structure):
    """rt_comm_status (rt_hip.h)."""
    _fields_ = [("rank", ctypes.c_int), ("nranks", ctypes.c_int), ("transport", ctypes.c_int),
                ("active", ctypes.c_int), ("fallback", ctypes.c_int), ("fallback_reason", ctypes.c_int),
                ("copies_per_gather", ctypes.c_uint), ("bytes_per_gather", ctypes.c_ulonglong),
                ("gathers", ctypes.c_ulonglong), ("last_xfer_ms", ctypes.c_double)]

_vp = ctypes.c_void_p
_HIP_PROTOS = {
    "rtCreateContext": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(_vp)]),
    "rtReleaseContext": (ctypes.c_int, [_vp]),
    "rtCreateBuffer": (ctypes.c_int, [_vp, ctypes.c_uint64, ctypes.c_size_t, _vp, ctypes.POINTER(_vp)]),
    "rtReleaseBuffer": (ctypes.c_int, [_vp]),
    "rtCreateKernel": (ctypes.c_int, [_vp, ctypes.c_char_p, ctypes.POINTER(_vp)]),
    "rtReleaseKernel": (ctypes.c_int, [_vp]),
    "rtSetKernelArg": (ctypes.c_int, [_vp, ctypes.c_uint, ctypes.c_size_t, _vp]),
    "rtEnqueueKernel": (ctypes.c_int, [_vp, _vp, ctypes.c_size_t]),
    "rtEnqueueKernelFrames": (ctypes.c_int, [_vp, _vp, ctypes.c_size_t, ctypes.c_uint]),
    "rtEnqueueReadBuffer": (ctypes.c_int, [_vp, _vp, ctypes.c_int, ctypes.c_size_t, ctypes.c_size_t, _vp]),
    "rtEnqueueWriteBuffer": (ctypes.c_int, [_vp, _vp, ctypes.c_int, ctypes.c_size_t, ctypes.c_size_t, _vp]),
    "rtFinish": (ctypes.c_int, [_vp]),
    "rtEnqueueCopyBufferToPointer": (ctypes.c_int, [_vp, _vp, ctypes.c_size_t, ctypes.c_size_t, _vp]),
    "rtKernelSetMathMode": (ctypes.c_int, [_vp, ctypes.c_int]),
    "rtKernelSetWorkRange": (ctypes.c_int, [_vp, ctypes.c_uint64, ctypes.c_uint64]),
    "rtKernelSetSchedule": (ctypes.c_int, [_vp, ctypes.c_int]),
    "rtKernelSetRowInterleave": (ctypes.c_int, [_vp, ctypes.c_uint, ctypes.c_uint]),
    "rtEnqueueCopyBufferRectToPointer": (ctypes.c_int, [_vp, _vp, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_size_t,
                                                        ctypes.c_size_t, _vp, ctypes.c_size_t]),
    "rtEnqueueCopyPointerRectToBuffer": (ctypes.c_int, [_vp, _vp, ctypes.c_size_t, _vp, ctypes.c_size_t,
                                                        ctypes.c_size_t, ctypes.c_size_t, ctypes.c_size_t]),
    "rtKernelSetHitBuffers": (ctypes.c_int, [_vp, _vp, _vp]),
    "rtKernelSetStats": (ctypes.c_int, [_vp, ctypes.c_int]),
    "rtKernelSetTiming": (ctypes.c_int, [_vp, ctypes.c_int]),
    "rtKernelGetStats": (ctypes.c_int, [_vp, ctypes.POINTER(Stats)]),
    "rtKernelResetStats": (ctypes.c_int, [_vp]),
    "rtKernelGetSceneInLDS": (ctypes.c_int, [_vp, ctypes.POINTER(ctypes.c_int)]),
    "rtKernelForceGlobalScene": (ctypes.c_int, [_vp, ctypes.c_int]),
    "rtBuildBVH": (ctypes.c_int, [_vp, _vp, ctypes.c_size_t, ctypes.c_uint, _vp, ctypes.POINTER(ctypes.c_size_t)]),
    "rtBuildBVHEx": (ctypes.c_int, [_vp, _vp, ctypes.c_size_t, ctypes.c_uint, ctypes.c_int, _vp,
                                    ctypes.POINTER(ctypes.c_size_t)]),
    "rtBufferGetDevicePointer": (ctypes.c_int, [_vp, ctypes.POINTER(_vp)]),
    "rtBufferGetSize": (ctypes.c_int, [_vp, ctypes.POINTER(ctypes.c_size_t)]),
    "rtContextGetStream": (ctypes.c_int, [_vp, ctypes.POINTER(_vp)]),
    "rtContextSetReadbackOnAccumStream": (ctypes.c_int, [_vp, ctypes.c_int]),
    "rtContextGetAccumStream": (ctypes.c_int, [_vp, ctypes.POINTER(_vp)]),
    "rtContextGetDevice": (ctypes.c_int, [_vp, ctypes.POINTER(ctypes.c_int)]),
    "rtValidateBVH": (ctypes.c_int, [_vp, ctypes.c_size_t, ctypes.c_size_t, ctypes.POINTER(ctypes.c_int)]),
    "rtKernelSetTuning": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int]),
    "rtKernelGetTuning": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.POINTER(ctypes.c_int)]),
    "rtContextSetAccumOverlap": (ctypes.c_int, [_vp, ctypes.c_int]),
    "rtCommGetUniqueId": (ctypes.c_int, [_vp]),
    "rtCommInitRank": (ctypes.c_int, [_vp, ctypes.c_int, _vp, ctypes.c_int, ctypes.POINTER(_vp)]),
    "rtCommInitAll": (ctypes.c_int, [ctypes.POINTER(_vp), ctypes.c_int, ctypes.POINTER(_vp)]),
    "rtCommInitLoopback": (ctypes.c_int, [ctypes.POINTER(_vp), ctypes.c_int, ctypes.POINTER(_vp)]),
    "rtCommInitShared": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int, ctypes.c_char_p, ctypes.POINTER(_vp)]),
    "rtCommDestroy": (ctypes.c_int, [_vp]),
    "rtCommGetRank": (ctypes.c_int, [_vp, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]),
    "rtCommShardKernel": (ctypes.c_int, [_vp, _vp]),
    "rtCommSetTransport": (ctypes.c_int, [_vp, ctypes.c_int]),
    "rtCommGetTransport": (ctypes.c_int, [_vp, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]),
    "rtCommGetStatus": (ctypes.c_int, [_vp, ctypes.POINTER(CommStatus)]),
    "rtCommSetOption": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int]),
    "rtCommEnqueueGatherBands": (ctypes.c_int, [ctypes.POINTER(_vp), ctypes.POINTER(_vp), ctypes.c_int, ctypes.c_uint,
                                                ctypes.c_uint, ctypes.c_int, _vp]),
    "rtCommAllReduceF64": (ctypes.c_int, [ctypes.POINTER(_vp), ctypes.c_int, ctypes.POINTER(ctypes.c_double),
                                          ctypes.c_int, ctypes.c_int]),
    "rtCommBarrier": (ctypes.c_int, [ctypes.POINTER(_vp), ctypes.c_int]),
    "rtBandPackPlan": (ctypes.c_int, [ctypes.c_uint, ctypes.c_uint, ctypes.c_uint, ctypes.c_uint, ctypes.POINTER(Rect),
                                      ctypes.c_int, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_size_t)]),
    "rtGetBuildInfo": (ctypes.c_char_p, []),
    "rtDiagPinnedMath": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, _vp, _vp, _vp, ctypes.c_size_t]),
}
HIP_EXPORTS = tuple(_HIP_PROTOS)

_SCENE_PROTOS = {
    "rtsLoadOBJ": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_uint, ctypes.POINTER(_vp)]),
    "rtsLoadOBJUnbuilt": (ctypes.c_int, [ctypes.c_char_p, ctypes.POINTER(_vp)]),
    "rtsBuildFromTriangles": (ctypes.c_int, [_vp, ctypes.c_size_t, _vp, ctypes.c_size_t, ctypes.c_uint,
                                             ctypes.POINTER(_vp)]),
    "rtsGetTriangles": (ctypes.c_int, [_vp, ctypes.POINTER(_vp), ctypes.POINTER(ctypes.c_size_t)]),
    "rtsGetNodes": (ctypes.c_int, [_vp, ctypes.POINTER(_vp), ctypes.POINTER(ctypes.c_size_t)]),
    "rtsGetMaterials": (ctypes.c_int, [_vp, ctypes.POINTER(_vp), ctypes.POINTER(ctypes.c_size_t)]),
    "rtsGetTreeStats": (ctypes.c_int, [_vp, ctypes.POINTER(ctypes.c_uint), ctypes.POINTER(ctypes.c_uint),
                                       ctypes.POINTER(ctypes.c_uint)]),
    "rtsFromArrays": (ctypes.c_int, [_vp, ctypes.c_size_t, _vp, ctypes.c_size_t, _vp, ctypes.c_size_t,
                                     ctypes.c_uint, ctypes.POINTER(_vp)]),
    "rtsSaveScene": (ctypes.c_int, [_vp, ctypes.c_char_p]),
    "rtsLoadScene": (ctypes.c_int, [ctypes.c_char_p, ctypes.POINTER(_vp)]),
    "rtsRelease": (None, [_vp]),
}
SCENE_EXPORTS = tuple(_SCENE_PROTOS)

_libs: dict = {}


def _load(path: str, protos: dict) -> ctypes.CDLL:
    if path in _libs:
        return _libs[path]
    if not os.path.exists(path):
        raise RTError(f"{os.path.basename(path)} is not built (run __graft_entry__.build())", -59)
    lib = ctypes.CDLL(path)
    for name, (res, args) in protos.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _libs[path] = lib
    return lib


def validate_bvh(nodes: np.ndarray, n_tris: int) -> int:
    """rtValidateBVH (host-only): the BVH depth, or RTError(CL_INVALID_MEM_OBJECT)."""
    nodes = np.ascontiguousarray(nodes)
    d = ctypes.c_int()
    check(hip_lib().rtValidateBVH(nodes.ctypes.data, len(nodes), int(n_tris), ctypes.byref(d)), "Invalid BVH")
    return d.value


def hip_lib() -> ctypes.CDLL:
    """librt_hip.so -- the HIP hot path.  Loading it does not touch the GPU."""
    return _load(HIP_LIB_PATH, _HIP_PROTOS)


def scene_lib() -> ctypes.CDLL:
    """librt_scene.so -- the host scene pipeline."""
    return _load(SCENE_LIB_PATH, _SCENE_PROTOS)


PINNED_OPS = {"rcp": 0, "div": 1, "sqrt": 2, "rsqrt": 3, "pow": 4, "sin": 5, "cos": 6}


def pinned_math(op: str, a, b=None, device: int = 0) -> np.ndarray:
    """rtDiagPinnedMath: the pinned policy's device builtins, element-wise (tests)."""
    a = np.ascontiguousarray(a, dtype=np.float32)
    bb = None if b is None else np.ascontiguousarray(np.broadcast_to(np.float32(b) if np.isscalar(b) else b, a.shape),
                                                     dtype=np.float32)
    out = np.empty_like(a)
    check(hip_lib().rtDiagPinnedMath(int(device), PINNED_OPS[op], a.ctypes.data,
                                     None if bb is None else bb.ctypes.data, out.ctypes.data, a.size),
          f"pinned math {op}")
    return out
