"""Image-space sharding of a frame across GPUs (one process per GPU).

The reference renders on one OpenCL device (CLRaytracer.cpp:104-120); pixels are
independent (the seed depends only on the global work-item id and frameCount,
kernel_bvh.cl:445), so a frame shards by pixel rows with no exchange until the image is
needed.  Rows are dealt in interleaved 8-row *bands* (band b goes to rank b % N): Cornell's
cost varies with height (contiguous row tiles measured max/mean 1.23 at N = 8 on the
oracle's counters, interleaved bands 1.08).  Every rank renders its bands into a full-size
output buffer at their global positions; to assemble the image the bands are packed
(one strided 2-D device copy), gathered to rank 0 over torch.distributed ("nccl" = RCCL over
xGMI on the GPU box: grouped send/recv, so the root receives on all its links at once), and
unpacked on the root with the inverse 2-D copy.

The product path is the library's RCCL communicator (``Comm`` below over rtComm* in
include/rt_hip.h, csrc/rt_comm.cpp): pack on the context's accumulation stream, grouped
send/recv to the root on the communicator's stream, unpack on a third stream -- no torch
and no second HIP runtime in the process.  The plans below are pure index math, the same
as the library's rtBandPackPlan (tests compare them), and drive the numpy path the CPU tests
use over torch.distributed/gloo.
"""
from __future__ import annotations

import ctypes
import os
import time
from dataclasses import dataclass

import numpy as np

from . import _native as N
from ._native import check

BAND_ROWS = 8          # = the 8x8 tile height of the regen/step schedules
PIXEL_BYTES = 16       # one float3 slot of the output buffer


@dataclass(frozen=True)
class Rect:
    """`rows` rows of `width` bytes: image bytes [img_offset + i*img_pitch, +width) <->
    staging bytes [stage_offset + i*width, +width)."""
    img_offset: int
    img_pitch: int
    width: int
    rows: int
    stage_offset: int


def rank_bands(height: int, period: int, phase: int) -> list[int]:
    nb = (height + BAND_ROWS - 1) // BAND_ROWS
    return list(range(phase, nb, period))


def staging_bytes(width: int, height: int, period: int) -> int:
    """Bytes of one rank's staging buffer (the largest rank's share; equal for all ranks
    so the gather moves equal-size tensors)."""
    nb = (height + BAND_ROWS - 1) // BAND_ROWS
    per_rank = (nb + period - 1) // period
    return per_rank * BAND_ROWS * width * PIXEL_BYTES


def pack_plan(width: int, height: int, period: int, phase: int) -> list[Rect]:
    """Copies moving this rank's bands out of the full image into its staging buffer."""
    bands = rank_bands(height, period, phase)
    band_bytes = BAND_ROWS * width * PIXEL_BYTES
    full = [b for b in bands if (b + 1) * BAND_ROWS <= height]
    rects = []
    if full:
        rects.append(Rect(full[0] * band_bytes, period * band_bytes, band_bytes, len(full), 0))
    tail = [b for b in bands if (b + 1) * BAND_ROWS > height]
    for b in tail:  # at most one short band (the image's last rows)
        rows = height - b * BAND_ROWS
        rects.append(Rect(b * band_bytes, band_bytes, rows * width * PIXEL_BYTES, 1, len(full) * band_bytes))
    return rects


def pack_numpy(image: np.ndarray, plan: list[Rect], staging: np.ndarray) -> None:
    src = image.view(np.uint8).reshape(-1)
    dst = staging.view(np.uint8).reshape(-1)
    for r in plan:
        for i in range(r.rows):
            s = r.img_offset + i * r.img_pitch
            d = r.stage_offset + i * r.width
            dst[d:d + r.width] = src[s:s + r.width]


def unpack_numpy(staging: np.ndarray, plan: list[Rect], image: np.ndarray) -> None:
    src = staging.view(np.uint8).reshape(-1)
    dst = image.view(np.uint8).reshape(-1)
    for r in plan:
        for i in range(r.rows):
            s = r.stage_offset + i * r.width
            d = r.img_offset + i * r.img_pitch
            dst[d:d + r.width] = src[s:s + r.width]


def pack_device(ctx, out_buffer, plan: list[Rect], staging_ptr: int) -> None:
    """Device version of pack_numpy: one 2-D copy per rect on the context's stream."""
    for r in plan:
        ctx.CopyRectToDevicePointer(out_buffer, r.img_offset, r.img_pitch, r.width, r.rows,
                                    staging_ptr + r.stage_offset, r.width)


def unpack_device(ctx, staging_ptr: int, plan: list[Rect], out_buffer) -> None:
    for r in plan:
        ctx.CopyRectFromDevicePointer(staging_ptr + r.stage_offset, r.width, out_buffer, r.img_offset,
                                      r.img_pitch, r.width, r.rows)


def gather_to_root(dist, tensor, rank: int, world: int):
    """Gather equal-size staging tensors to rank 0 (list on the root, None elsewhere)."""
    import torch
    out = [torch.empty_like(tensor) for _ in range(world)] if rank == 0 else None
    dist.gather(tensor, out, dst=0)
    return out


def native_pack_plan(width: int, height: int, period: int, phase: int) -> tuple[list[Rect], int]:
    """rtBandPackPlan: the library's plan (host-only, loads librt_hip.so without a GPU)."""
    lib = N.hip_lib()
    rects = (N.Rect * 2)()
    n = ctypes.c_int()
    sb = ctypes.c_size_t()
    check(lib.rtBandPackPlan(width, height, period, phase, rects, 2, ctypes.byref(n), ctypes.byref(sb)), "band plan")
    return [Rect(r.img_offset, r.img_pitch, r.width, r.rows, r.stage_offset) for r in rects[:n.value]], sb.value


class Comm:
    """One rank's RCCL communicator (rt_comm): band sharding + the pipelined band gather."""

    def __init__(self, handle: int, ctx):
        self._lib = N.hip_lib()
        self.handle = handle
        self.ctx = ctx
        r, n = ctypes.c_int(), ctypes.c_int()
        check(self._lib.rtCommGetRank(handle, ctypes.byref(r), ctypes.byref(n)), "comm rank")
        self.rank, self.nranks = r.value, n.value

    @staticmethod
    def unique_id() -> bytes:
        buf = ctypes.create_string_buffer(N.COMM_ID_BYTES)
        check(N.hip_lib().rtCommGetUniqueId(buf), "comm unique id")
        return buf.raw

    @classmethod
    def init_rank(cls, ctx, nranks: int, uid: bytes, rank: int) -> "Comm":
        """One process per GPU (ncclCommInitRank)."""
        assert len(uid) == N.COMM_ID_BYTES
        h = ctypes.c_void_p()
        check(N.hip_lib().rtCommInitRank(ctx.handle, nranks, uid, rank, ctypes.byref(h)), "comm init rank")
        return cls(h.value, ctx)

    @classmethod
    def init_all(cls, ctxs) -> list["Comm"]:
        """One process driving len(ctxs) GPUs (ncclCommInitAll)."""
        n = len(ctxs)
        hs = (ctypes.c_void_p * n)(*[c.handle for c in ctxs])
        out = (ctypes.c_void_p * n)()
        check(N.hip_lib().rtCommInitAll(hs, n, out), "comm init all")
        return [cls(out[i], ctxs[i]) for i in range(n)]

    @classmethod
    def init_loopback(cls, ctxs) -> list["Comm"]:
        """A world of len(ctxs) ranks in this process without RCCL (rtCommInitLoopback): the
        transfer is a device copy, the rest of the gather is the RCCL flow; the contexts may
        share one GPU."""
        n = len(ctxs)
        hs = (ctypes.c_void_p * n)(*[c.handle for c in ctxs])
        out = (ctypes.c_void_p * n)()
        check(N.hip_lib().rtCommInitLoopback(hs, n, out), "comm init loopback")
        return [cls(out[i], ctxs[i]) for i in range(n)]

    @classmethod
    def init_shared(cls, ctx, nranks: int, rank: int, directory: str) -> "Comm":
        """A world of processes on one node without RCCL (rtCommInitShared): setup and reductions
        through files in `directory`, gathers on the copy engines over IPC mappings -- several
        ranks may share one GPU."""
        h = ctypes.c_void_p()
        check(N.hip_lib().rtCommInitShared(ctx.handle, nranks, rank, directory.encode(), ctypes.byref(h)),
              "comm init shared")
        return cls(h.value, ctx)

    def set_transport(self, transport: int) -> None:
        """rtCommSetTransport: N.COMM_TRANSPORT_COPY_ENGINES (default) or N.COMM_TRANSPORT_RCCL."""
        check(self._lib.rtCommSetTransport(self.handle, transport), "comm transport")

    def transport(self) -> tuple[int, int]:
        """(requested, active) transport; active -1 before the first gather."""
        t, a = ctypes.c_int(), ctypes.c_int()
        check(self._lib.rtCommGetTransport(self.handle, ctypes.byref(t), ctypes.byref(a)), "comm transport")
        return t.value, a.value

    def status(self) -> dict:
        """rtCommGetStatus: what the current plan does -- the effective transport, whether the
        copy-engine links fell back to RCCL (and why), the bytes and copy commands this rank
        moves per gather, the last gather's transfer time on this rank."""
        st = N.CommStatus()
        check(self._lib.rtCommGetStatus(self.handle, ctypes.byref(st)), "comm status")
        return {"rank": st.rank, "nranks": st.nranks, "transport": N.COMM_TRANSPORT_NAMES[st.transport],
                "active": N.COMM_TRANSPORT_NAMES[st.active], "active_code": st.active,
                "fallback": bool(st.fallback), "fallback_reason": N.COMM_FALLBACK_NAMES.get(st.fallback_reason),
                "copies_per_gather": st.copies_per_gather, "bytes_per_gather": st.bytes_per_gather,
                "gathers": st.gathers, "last_xfer_ms": None if st.last_xfer_ms < 0 else st.last_xfer_ms}

    def set_option(self, option: int, value: int) -> None:
        """rtCommSetOption (N.COMM_OPT_FAIL_LINKS, N.COMM_OPT_REPLAN_PERIOD, N.COMM_OPT_SYSTEM_ACQUIRE)."""
        check(self._lib.rtCommSetOption(self.handle, option, value), "comm option")

    def shard(self, kernel) -> None:
        """The kernel renders this rank's interleaved bands (rtCommShardKernel)."""
        check(self._lib.rtCommShardKernel(self.handle, kernel.handle), "shard kernel")

    @staticmethod
    def gather_bands(comms, outs, width: int, height: int, root: int = 0, dst=None) -> None:
        """rtCommEnqueueGatherBands over the communicators this thread drives."""
        n = len(comms)
        hc = (ctypes.c_void_p * n)(*[c.handle for c in comms])
        ho = (ctypes.c_void_p * n)(*[o.handle for o in outs])
        check(comms[0]._lib.rtCommEnqueueGatherBands(hc, ho, n, width, height, root, dst.handle if dst else None),
              "gather bands")

    @staticmethod
    def allreduce(comms, values, op: int = N.COMM_SUM) -> np.ndarray:
        """Blocking reduction of float64 values (n_local x count)."""
        v = np.ascontiguousarray(np.asarray(values, np.float64).reshape(len(comms), -1))
        hc = (ctypes.c_void_p * len(comms))(*[c.handle for c in comms])
        check(comms[0]._lib.rtCommAllReduceF64(hc, len(comms), v.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                                               v.shape[1], op), "allreduce")
        return v

    @staticmethod
    def barrier(comms) -> None:
        hc = (ctypes.c_void_p * len(comms))(*[c.handle for c in comms])
        check(comms[0]._lib.rtCommBarrier(hc, len(comms)), "barrier")

    def destroy(self) -> None:
        if self.handle:
            self._lib.rtCommDestroy(self.handle)
            self.handle = None


def _rendezvous_path() -> str:
    """Keyed by the launcher's pid (every rank of a torch.distributed.run job has the same
    parent), MASTER_PORT, and the elastic run id + restart count: a restarted attempt (same
    agent pid and port under --max-restarts) gets a fresh path, so no rank can read an id a
    failed attempt left behind.  RT_COMM_ID_FILE overrides it."""
    if os.environ.get("RT_COMM_ID_FILE"):
        return os.environ["RT_COMM_ID_FILE"]
    run = "".join(ch if ch.isalnum() else "_" for ch in os.environ.get("TORCHELASTIC_RUN_ID", "none"))[:64]
    attempt = os.environ.get("TORCHELASTIC_RESTART_COUNT", "0")
    return os.path.join("/tmp", f"rt_comm_{os.environ.get('MASTER_PORT', '0')}_{os.getppid()}_{run}_{attempt}.id")


def file_rendezvous(rank: int, world: int, make_id, timeout: float = 300.0) -> bytes:
    """Hand rank 0's communicator id to the other ranks of ONE node through a file (no torch,
    no sockets), at _rendezvous_path()."""
    path = _rendezvous_path()
    if rank == 0:
        uid = make_id()
        tmp = f"{path}.{os.getpid()}.tmp"
        with open(tmp, "wb") as f:
            f.write(uid)
        os.replace(tmp, path)
        return uid
    t0 = time.monotonic()
    while True:
        try:
            with open(path, "rb") as f:
                uid = f.read()
            if len(uid) == N.COMM_ID_BYTES:
                return uid
        except FileNotFoundError:
            pass
        if time.monotonic() - t0 > timeout:
            raise TimeoutError(f"rank {rank}: no communicator id at {path} after {timeout:.0f} s")
        time.sleep(0.05)


def rendezvous_cleanup() -> None:
    path = _rendezvous_path()
    try:
        os.unlink(path)
    except FileNotFoundError:
        pass
