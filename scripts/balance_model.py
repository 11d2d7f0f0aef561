#!/usr/bin/env python3
"""Load-balance model for the multi-GPU split: per-pixel work of one 4K 9-bounce
Cornell frame from the oracle, summed per rank for candidate pixel-to-rank assignments.
Prints max/mean rank work (1.00 = perfect) for N = 2, 4, 8."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mini-opencl-raytracer_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import clrt  # noqa: E402
import oracle  # noqa: E402

W, H = (int(x) for x in (sys.argv[1:3] or (3840, 2160)))
oracle.build()
cost = oracle.pixel_cost(clrt.scene.cornell(), W, H).astype(np.float64)
tiles = cost.reshape(H // 8, 8, W // 8, 8).sum(axis=(1, 3))  # [ty, tx] 8x8-tile work
ty, tx = np.indices(tiles.shape)
schemes = {
    "contiguous rows": lambda n: (ty * n) // tiles.shape[0],
    "8-row bands b%N (current)": lambda n: ty % n,
    "tile columns tx%N": lambda n: tx % n,
    "tile diagonal (tx+ty)%N": lambda n: (tx + ty) % n,
    "tile (tx+3ty)%N": lambda n: (tx + 3 * ty) % n,
    "tile (tx+(ty%N)*N/2... ) skew": lambda n: (tx + ty * max(1, n // 2 + 1)) % n,
}
print(f"{W}x{H}, 9 bounces: total work {cost.sum():.3g}, tiles {tiles.shape}")
for name, f in schemes.items():
    row = []
    for n in (2, 4, 8):
        r = f(n)
        w = np.array([tiles[r == k].sum() for k in range(n)])
        row.append(f"N={n} {w.max() / w.mean():.4f}")
    print(f"{name:32s} " + "  ".join(row))
