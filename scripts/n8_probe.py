#!/usr/bin/env python3
"""Where does an emulated N = 8 rank's step go?  For rank 0 and N-1 of N (interleaved 8-row
bands of the 4K 8-spp Cornell step, fused): isolated latency of one step (Finish after each),
back-to-back period (the bench's loop), host time spent inside the enqueue calls, the same loop
with the accumulation on the main stream (no render-stream overlap), and the render kernel's own
event time.  usage: n8_probe.py [N ...]  (env RT_EMU_SCENE=cornell|bunny, RT_EMU_TUNE=name=v,..,
RT_EMU_BOUNCES, RT_EMU_ISO=1: isolated steps only)"""
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mini-opencl-raytracer_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import clrt  # noqa: E402
from clrt import _native as N  # noqa: E402
from hip_helpers import HipRenderer  # noqa: E402

if os.environ.get("RT_EMU_SCENE", "cornell") == "bunny":
    from clrt import proxy
    sc = proxy.bunny_proxy()
else:
    sc = clrt.scene.cornell()
tunes = [t.split("=") for t in os.environ.get("RT_EMU_TUNE", "").split(",") if t]
W, H, F, STEPS = 3840, 2160, 8, 20
B = int(os.environ.get("RT_EMU_BOUNCES", "9"))
ONLY_ISO = os.environ.get("RT_EMU_ISO", "0") == "1"
for n in [int(x) for x in sys.argv[1:]] or [1, 8]:
    for rank in sorted({0, n - 1}):
        res = {}
        for overlap in ((True,) if ONLY_ISO else (True, False)):
            r = HipRenderer(sc, W, H, math=N.MATH_SHIPPED)
            r.k.set_row_interleave(n, rank)
            for name, v in tunes:
                r.k.set_tuning(name, int(v))
            r.ctx.set_accum_overlap(overlap)
            r.frame(1, light_bounces=B, n_frames=F)
            r.ctx.Finish()
            if overlap:
                iso = []
                for _ in range(10):
                    t0 = time.perf_counter()
                    r.frame(1, light_bounces=B, n_frames=F)
                    r.ctx.Finish()
                    iso.append((time.perf_counter() - t0) * 1e3)
                res["isolated"] = statistics.median(iso)
                r.k.set_timing(True)
                r.k.reset_stats()
                for _ in range(5):
                    r.frame(1, light_bounces=B, n_frames=F)
                    r.ctx.Finish()
                res["isolated_kernel"] = r.k.stats()["kernel_ms"] / 5
                if ONLY_ISO:
                    r.close()
                    continue
            r.k.set_timing(True)
            r.k.reset_stats()
            host = 0.0
            t0 = time.perf_counter()
            for _ in range(STEPS):
                h0 = time.perf_counter()
                r.frame(1, light_bounces=B, n_frames=F)
                host += time.perf_counter() - h0
            r.ctx.Finish()
            el = (time.perf_counter() - t0) / STEPS * 1e3
            ks = r.k.stats()
            key = "overlap" if overlap else "in_order"
            res[key] = el
            res[key + "_kernel"] = ks["kernel_ms"] / STEPS
            res[key + "_host"] = host / STEPS * 1e3
            r.close()
        print(f"N={n} rank={rank}: " + ", ".join(f"{k} {v:.3f}" for k, v in res.items()), flush=True)
