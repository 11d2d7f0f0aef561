"""Python mirror of the reference's device wrapper over librt_hip.so.

``CLContext`` / ``CLKernel`` / ``Buffer`` keep the method names and argument meaning of
/root/reference/CLutils.h:116-145 (ReadBuffer, ExecuteKernel, Finish, SetArgument) and
raise ``RTError`` (the reference's CLException) on any non-zero status.
"""
from __future__ import annotations

import ctypes
import struct

import numpy as np

from . import _native as N
from ._native import RTError, check, hip_lib


class CLContext:
    """CLContext(platform) (CLutils.cpp:9-35): GPU `device` + one in-order HIP stream."""

    def __init__(self, device: int = 0):
        self._lib = hip_lib()
        h = ctypes.c_void_p()
        check(self._lib.rtCreateContext(int(device), ctypes.byref(h)), "Failed to create context")
        self.handle = h
        self.device = int(device)

    def create_buffer(self, flags: int, size: int, host: np.ndarray | None = None) -> "Buffer":
        return Buffer(self, flags, size, host)

    def ReadBuffer(self, buffer: "Buffer", out: np.ndarray, size: int | None = None,
                   blocking: bool = False) -> None:
        """enqueueReadBuffer(buffer, blocking=false, 0, size, ptr) (CLutils.cpp:37-42)."""
        size = out.nbytes if size is None else int(size)
        if not out.flags["C_CONTIGUOUS"] or size > out.nbytes:
            raise RTError("Failed to read buffer", -30)
        check(self._lib.rtEnqueueReadBuffer(self.handle, buffer.handle, int(blocking), 0, size,
                                            out.ctypes.data), "Failed to read buffer")

    def WriteBuffer(self, buffer: "Buffer", data: np.ndarray, blocking: bool = True) -> None:
        data = np.ascontiguousarray(data)
        check(self._lib.rtEnqueueWriteBuffer(self.handle, buffer.handle, int(blocking), 0, data.nbytes,
                                             data.ctypes.data), "Failed to write buffer")

    def BuildBVH(self, tris: "Buffer", n_tris: int, max_prims_in_node: int, nodes: "Buffer",
                 method: int = N.BVH_PLOC) -> int:
        """rtBuildBVHEx: device-side BVH (PLOC, or the linear BVH) over `tris` (permuted in place);
        returns the node count written to `nodes`."""
        n = ctypes.c_size_t()
        check(self._lib.rtBuildBVHEx(self.handle, tris.handle, int(n_tris), int(max_prims_in_node), int(method),
                                     nodes.handle, ctypes.byref(n)), "Failed to build BVH")
        return int(n.value)

    def CopyToDevicePointer(self, buffer: "Buffer", offset: int, size: int, dst: int) -> None:
        """Device-to-device copy into foreign device memory (e.g. a torch tensor)."""
        check(self._lib.rtEnqueueCopyBufferToPointer(self.handle, buffer.handle, int(offset), int(size),
                                                     ctypes.c_void_p(int(dst))), "Failed to copy buffer")

    def CopyRectToDevicePointer(self, buffer: "Buffer", src_offset: int, src_pitch: int, width: int,
                                rows: int, dst: int, dst_pitch: int) -> None:
        check(self._lib.rtEnqueueCopyBufferRectToPointer(self.handle, buffer.handle, int(src_offset), int(src_pitch),
                                                         int(width), int(rows), ctypes.c_void_p(int(dst)),
                                                         int(dst_pitch)), "Failed to copy rect")

    def CopyRectFromDevicePointer(self, src: int, src_pitch: int, buffer: "Buffer", dst_offset: int,
                                  dst_pitch: int, width: int, rows: int) -> None:
        check(self._lib.rtEnqueueCopyPointerRectToBuffer(self.handle, ctypes.c_void_p(int(src)), int(src_pitch),
                                                         buffer.handle, int(dst_offset), int(dst_pitch), int(width),
                                                         int(rows)), "Failed to copy rect")

    def ExecuteKernel(self, kernel: "CLKernel", work_size: int) -> None:
        """enqueueNDRangeKernel(kernel, NullRange, NDRange(workSize)) (CLutils.cpp:44-50)."""
        check(self._lib.rtEnqueueKernel(self.handle, kernel.handle, int(work_size)),
              "Failed to enqueue kernel")

    def ExecuteKernelFrames(self, kernel: "CLKernel", work_size: int, n_frames: int) -> None:
        """Extension: frames FRAME_COUNT .. FRAME_COUNT + n_frames - 1 (rtEnqueueKernelFrames),
        bit-identical to n_frames ExecuteKernel calls with those frame counts."""
        check(self._lib.rtEnqueueKernelFrames(self.handle, kernel.handle, int(work_size), int(n_frames)),
              "Failed to enqueue kernel frames")

    def Finish(self) -> None:
        check(self._lib.rtFinish(self.handle), "Failed to finish queue")

    def stream(self) -> int:
        s = ctypes.c_void_p()
        check(self._lib.rtContextGetStream(self.handle, ctypes.byref(s)), "stream")
        return int(s.value or 0)

    def accum_stream(self) -> int:
        """The fused-frame accumulation stream (rtContextGetAccumStream)."""
        s = ctypes.c_void_p()
        check(self._lib.rtContextGetAccumStream(self.handle, ctypes.byref(s)), "accumulation stream")
        return int(s.value or 0)

    def set_accum_overlap(self, enable: bool) -> None:
        """rtContextSetAccumOverlap: fused frames' accumulation beside the next render (default)."""
        check(self._lib.rtContextSetAccumOverlap(self.handle, int(bool(enable))), "accumulation overlap")

    def set_readback_on_accum_stream(self, enable: bool) -> None:
        check(self._lib.rtContextSetReadbackOnAccumStream(self.handle, int(bool(enable))), "readback stream")

    def release(self) -> None:
        if self.handle:
            self._lib.rtReleaseContext(self.handle)
            self.handle = None


class Buffer:
    """cl::Buffer(context, flags, size, host_ptr) (CLBVHnode.cpp:215-236)."""

    def __init__(self, ctx: CLContext, flags: int, size: int, host: np.ndarray | None = None):
        self._lib = ctx._lib
        self.ctx = ctx
        h = ctypes.c_void_p()
        ptr = None
        if host is not None:
            host = np.ascontiguousarray(host)
            if host.nbytes < size:
                raise RTError("Failed to create buffer", -37)
            ptr = host.ctypes.data
        check(self._lib.rtCreateBuffer(ctx.handle, int(flags), int(size), ptr, ctypes.byref(h)),
              "Failed to create buffer")
        self.handle = h
        self.size = int(size)

    def device_pointer(self) -> int:
        p = ctypes.c_void_p()
        check(self._lib.rtBufferGetDevicePointer(self.handle, ctypes.byref(p)), "device pointer")
        return int(p.value)

    def release(self) -> None:
        if self.handle:
            self._lib.rtReleaseBuffer(self.handle)
            self.handle = None


class CLKernel:
    """CLKernel(file, devices) (CLutils.cpp:52-66).  The kernel is precompiled; only the
    name "KernelEntry" exists."""

    def __init__(self, ctx: CLContext, name: str = "KernelEntry"):
        self._lib = ctx._lib
        self.ctx = ctx
        h = ctypes.c_void_p()
        check(self._lib.rtCreateKernel(ctx.handle, name.encode(), ctypes.byref(h)),
              "Failed to create kernel")
        self.handle = h
        self._keep = {}

    def SetArgument(self, index: int, data: bytes) -> bool:
        """SetArgument(argIndex, data, size) (CLutils.cpp:68-77): raw bytes of the value."""
        buf = ctypes.create_string_buffer(bytes(data), len(data))
        check(self._lib.rtSetKernelArg(self.handle, int(index), len(data), buf),
              "Failed to set kernel argument")
        return True

    # typed helpers = CLRaytracer::SetUniform<T> instantiations (CLRaytracer.cpp:139-148)
    def set_buffer(self, index: int, buf: Buffer) -> bool:
        self._keep[index] = buf
        return self.SetArgument(index, struct.pack("P", buf.handle.value))

    def set_uint(self, index: int, v: int) -> bool:
        return self.SetArgument(index, struct.pack("<I", int(v) & 0xFFFFFFFF))

    def set_int(self, index: int, v: int) -> bool:
        return self.SetArgument(index, struct.pack("<i", int(v)))

    def set_float(self, index: int, v: float) -> bool:
        return self.SetArgument(index, struct.pack("<f", float(v)))

    def set_float3(self, index: int, v) -> bool:
        x, y, z = (float(c) for c in v)
        return self.SetArgument(index, struct.pack("<4f", x, y, z, 0.0))

    # extensions
    def set_math_mode(self, mode: int) -> None:
        check(self._lib.rtKernelSetMathMode(self.handle, int(mode)), "math mode")

    def set_schedule(self, sched: int) -> None:
        check(self._lib.rtKernelSetSchedule(self.handle, int(sched)), "schedule")

    def set_tuning(self, name: str, value: int) -> None:
        """rtKernelSetTuning: a scheduling parameter by name (N.TUNING); results are unchanged."""
        check(self._lib.rtKernelSetTuning(self.handle, N.TUNING[name], int(value)), f"tuning {name}")

    def get_tuning(self, name: str) -> int:
        v = ctypes.c_int()
        check(self._lib.rtKernelGetTuning(self.handle, N.TUNING[name], ctypes.byref(v)), f"tuning {name}")
        return int(v.value)

    def set_row_interleave(self, period: int, phase: int) -> None:
        check(self._lib.rtKernelSetRowInterleave(self.handle, int(period), int(phase)), "row interleave")

    def set_work_range(self, first: int, last: int) -> None:
        check(self._lib.rtKernelSetWorkRange(self.handle, int(first), int(last)), "work range")

    def set_hit_buffers(self, ids: Buffer | None, t: Buffer | None) -> None:
        check(self._lib.rtKernelSetHitBuffers(self.handle, ids.handle if ids else None,
                                              t.handle if t else None), "hit buffers")
        self._keep["hits"] = (ids, t)

    def set_stats(self, enable: bool) -> None:
        check(self._lib.rtKernelSetStats(self.handle, int(bool(enable))), "stats")

    def set_timing(self, enable: bool) -> None:
        check(self._lib.rtKernelSetTiming(self.handle, int(bool(enable))), "timing")

    def force_global_scene(self, force: bool) -> None:
        check(self._lib.rtKernelForceGlobalScene(self.handle, int(bool(force))), "force global")

    def scene_in_lds(self) -> bool:
        v = ctypes.c_int()
        check(self._lib.rtKernelGetSceneInLDS(self.handle, ctypes.byref(v)), "scene in lds")
        return bool(v.value)

    def stats(self) -> dict:
        s = N.Stats()
        check(self._lib.rtKernelGetStats(self.handle, ctypes.byref(s)), "stats")
        return {"rays": s.rays, "node_visits": s.node_visits, "tri_tests": s.tri_tests,
                "hits": s.hits, "launches": s.launches, "kernel_ms": s.kernel_ms, "accum_ms": s.accum_ms,
                "render_period_ms": s.render_period_ms,
                "cycles": {"refill": s.cycles_refill, "traverse": s.cycles_traverse,
                           "shade": s.cycles_shade, "total": s.cycles_total},
                "sched": dict(zip(("node_steps", "node_lanes", "tri_steps", "tri_lanes", "shade_rounds",
                                   "shade_lanes", "refill_rounds", "refill_lanes", "other_lanes",
                                   "shade_wait", "free_wait", "reserved"), list(s.sched)))}

    def reset_stats(self) -> None:
        check(self._lib.rtKernelResetStats(self.handle), "reset stats")

    def release(self) -> None:
        if self.handle:
            self._lib.rtReleaseKernel(self.handle)
            self.handle = None
