#!/usr/bin/env python3
"""Round-6 experiment (library variant built with -DRT_TILE_ORDER=1, RT_HIP_LIB): hand a launch's tiles
out costliest first -- longest-processing-time-first, so that the launch ends on cheap (sky) tiles and
its drain shortens.  The cost of a tile = its pixels that are not primary misses, from one render's
primary hit ids.  Results cannot change (seeds follow the pixel).  Prints ms per step for raster order
vs the cost order, for one GPU (N = 1) and an emulated N = 8 rank (its interleaved bands), fused frames.
env: RT_EXP_SCENE=cornell|bunny, RT_EXP_STEPS."""
import ctypes
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(REPO, "mini-opencl-raytracer_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import clrt  # noqa: E402
from clrt import _native as N  # noqa: E402
from hip_helpers import HipRenderer  # noqa: E402

W, H, F = 3840, 2160, 8
steps = int(os.environ.get("RT_EXP_STEPS", "10"))
if os.environ.get("RT_EXP_SCENE") == "bunny":
    from clrt import proxy
    sc = proxy.bunny_proxy()
else:
    sc = clrt.scene.cornell()
lib = N.hip_lib()
lib.rtDiagSetTileOrder.restype = ctypes.c_int
lib.rtDiagSetTileOrder.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]

# primary hits of the whole frame (frame 1): cost per 8x8 block = pixels that hit something
r0 = HipRenderer(sc, W, H, math=N.MATH_SHIPPED, hits=True)
r0.frame(1, light_bounces=9)
ids = r0.hits()[0].reshape(H, W)
r0.close()
bx, by = (W + 7) // 8, (H + 7) // 8
pad = np.full((by * 8, bx * 8), -1, np.int32)
pad[:H, :W] = ids
cost = (pad.reshape(by, 8, bx, 8) >= 0).sum(axis=(1, 3))  # [block row, block col]


def order_for(n, rank):
    rows = np.arange(rank, by, n)  # this rank's 8-row bands (tile rows)
    c = cost[rows].reshape(-1)     # tile t = ty * bx + tx over the rank's tile rows
    return np.argsort(-c, kind="stable").astype(np.uint32)


def step_ms(n, rank, ordered):
    r = HipRenderer(sc, W, H, math=N.MATH_SHIPPED)
    if n > 1:
        r.k.set_row_interleave(n, rank)
    if ordered:
        o = order_for(n, rank)
        assert lib.rtDiagSetTileOrder(r.k.handle, o.ctypes.data, o.size) == 0
    r.frame(1, light_bounces=9, n_frames=F)
    r.ctx.Finish()
    t0 = time.perf_counter()
    for _ in range(steps):
        r.frame(1, light_bounces=9, n_frames=F)
    r.ctx.Finish()
    el = (time.perf_counter() - t0) / steps * 1e3
    out = r.result()
    r.close()
    return el, out


for n, ranks in ((1, [0]), (8, [0, 3, 7])):
    for rank in ranks:
        a, ra = step_ms(n, rank, False)
        b, rb = step_ms(n, rank, True)
        a2, _ = step_ms(n, rank, False)
        b2, _ = step_ms(n, rank, True)
        same = ra.tobytes() == rb.tobytes()
        print(f"N={n} rank {rank}: raster {a:.3f} {a2:.3f} ms/step | cost order {b:.3f} {b2:.3f} ms/step | same bits {same}",
              flush=True)
