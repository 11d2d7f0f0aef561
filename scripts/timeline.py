#!/usr/bin/env python3
"""Diagnostic (needs a build with -DRT_TIMELINE=1, scripts/build_variant.sh, via RT_HIP_LIB):
launch span vs mean wave end of the instrumented step launch -- how much of a launch is the
drain (waves finished, GPU waiting for the last ones).  usage: timeline.py [N ...]
env: RT_TL_W, RT_TL_H (3840x2160), RT_TL_LB (9 bounces), RT_TL_FRAMES (8: per-frame launch, then F fused
frames; 1: per-frame only), RT_TL_DIV (the build's RT_TIMELINE_DIV: histogram bins that many times finer)"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mini-opencl-raytracer_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import clrt  # noqa: E402
from clrt import _native as N  # noqa: E402
from hip_helpers import HipRenderer  # noqa: E402

sc = clrt.scene.cornell()
W, H = int(os.environ.get("RT_TL_W", "3840")), int(os.environ.get("RT_TL_H", "2160"))
LB, NF = int(os.environ.get("RT_TL_LB", "9")), int(os.environ.get("RT_TL_FRAMES", "8"))
DIV = float(os.environ.get("RT_TL_DIV", "1"))
for n in [int(x) for x in sys.argv[1:]] or [1, 8]:
    for fused in ((False, True) if NF > 1 else (False,)):
        r = HipRenderer(sc, W, H, math=N.MATH_SHIPPED, stats=True)
        r.k.set_row_interleave(n, 0)
        npx = W * H
        hb = (r.ctx.create_buffer(N.MEM_READ_WRITE, (npx + 192) * 4), r.ctx.create_buffer(N.MEM_READ_WRITE, (npx + 192) * 4))
        r.k.set_hit_buffers(*hb)
        r.k.reset_stats()
        if fused:
            r.frame(1, light_bounces=LB, n_frames=NF)
        else:
            r.frame(1, light_bounces=LB)
        r.ctx.Finish()
        s = r.k.stats()["sched"]
        t0 = (~s["other_lanes"]) & 0xffffffffffffffff
        t1, tsum, waves = s["shade_wait"], s["free_wait"], s["reserved"]
        last_start = (s["refill_lanes"] - t0) / 100.0
        span = (t1 - t0) / 100.0
        mean_end = (tsum / max(1, waves) - t0) / 100.0
        print(f"{W}x{H} lb={LB} N={n} {f'fused x{NF}' if fused else 'one frame'}: waves {waves}, span {span:.1f} us, "
              f"last wave start {last_start:.1f} us, mean wave end {mean_end:.1f} us, drain {span - mean_end:.1f} us ({(span - mean_end) / span:.1%})",
              flush=True)
        import numpy as np
        h = np.zeros(npx + 192, np.int32)
        r.ctx.ReadBuffer(hb[0], h, blocking=True)
        for name, off, us in (("wave lifetime", 0, 40 / DIV), ("counter dry after", 64, 40 / DIV),
                              ("wave end - dry", 128, 10 / DIV)):
            hist = h[npx + off:npx + off + 64]
            nz = np.nonzero(hist)[0]
            print(f"   {name} histogram ({us} us bins, bins {nz[0]}..{nz[-1]}): " +
                  " ".join(str(int(x)) for x in hist[nz[0]:nz[-1] + 1]), flush=True)
        r.k.set_hit_buffers(None, None)
        for x in hb:
            x.release()
        r.close()
