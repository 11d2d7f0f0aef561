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

The plans below are pure index math, shared by the device path (clrt.CLContext 2-D copies)
and the numpy path the CPU tests use.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

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
