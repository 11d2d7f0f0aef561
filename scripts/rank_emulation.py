#!/usr/bin/env python3
"""Emulate the per-rank work of an N-GPU run on one GPU: rank r of N renders the interleaved
8-row bands b % N == r of the 4K 8-spp frame (exactly what bench.py --gpus N gives it), one rank
after another.  Prints per-rank ms per 8-frame step and the strong-scaling efficiency of the
render alone (T1 / (N * max_r T_r)); the RCCL gather is not included.
usage: rank_emulation.py [N ...]   (env: RT_EMU_MATH, RT_EMU_SCENE=cornell|bunny, RT_EMU_STEPS,
       RT_EMU_FUSED=1: the 8 frames as one rtEnqueueKernelFrames call, RT_EMU_TUNE=name=v,name=v:
       library tunings; RT_EMU_STEPS defaults to bench.py's 20 timed steps)"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mini-opencl-raytracer_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import clrt  # noqa: E402
from clrt import _native as N  # noqa: E402
from hip_helpers import HipRenderer  # noqa: E402

math = {"pinned": N.MATH_PINNED, "devicelib": N.MATH_DEVICELIB, "shipped": N.MATH_SHIPPED}[
    os.environ.get("RT_EMU_MATH", "shipped")]
if os.environ.get("RT_EMU_SCENE", "cornell") == "bunny":
    from clrt import proxy
    sc = proxy.bunny_proxy()
else:
    sc = clrt.scene.cornell()
steps = int(os.environ.get("RT_EMU_STEPS", "20"))
tunes = [t.split("=") for t in os.environ.get("RT_EMU_TUNE", "").split(",") if t]
W, H, F = 3840, 2160, 8
t1 = None
for n in [int(x) for x in sys.argv[1:]] or [1, 2, 4, 8]:
    per = []
    for rank in range(n):
        r = HipRenderer(sc, W, H, math=math)
        r.k.set_row_interleave(n, rank)
        for name, v in tunes:
            r.k.set_tuning(name, int(v))

        def step():
            if os.environ.get("RT_EMU_FUSED", "0") == "1":
                r.frame(1, light_bounces=9, n_frames=F)
                return
            for f in range(1, F + 1):
                r.frame(f, light_bounces=9)
        step()
        r.ctx.Finish()
        r.k.set_timing(True)
        r.k.reset_stats()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        r.ctx.Finish()
        el = (time.perf_counter() - t0) / steps * 1e3
        ks = r.k.stats()
        kern = ks["kernel_ms"] / steps
        per.append((el, kern))
        r.close()
    tmax = max(p[0] for p in per)
    if n == 1:
        t1 = tmax
    eff = t1 / (n * tmax) if t1 else float("nan")
    print(f"N={n} ms/step per rank: " + " ".join(f"{p[0]:.3f}" for p in per) +
          f" | KernelEntry ms/step: " + " ".join(f"{p[1]:.3f}" for p in per) +
          f" | max {tmax:.3f} | render-only strong-scaling efficiency {eff:.3f}", flush=True)
