#!/usr/bin/env python3
"""Diagnostic: per-phase wave-cycle shares of the step schedule (stats variant, s_memtime)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mini-opencl-raytracer_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import clrt  # noqa: E402
from clrt import _native as N  # noqa: E402
from hip_helpers import HipRenderer  # noqa: E402

sc = clrt.scene.cornell()
for math in (N.MATH_DEVICELIB, N.MATH_PINNED):
    for lb in (1, 9):
        r = HipRenderer(sc, 3840, 2160, math=math, stats=True, sched=N.SCHED_STEP)
        r.frame(1, light_bounces=lb)
        r.ctx.Finish()
        s = r.k.stats()
        c = s["cycles"]
        tot = c["total"] or 1
        print(f"math={math} lb={lb} rays={s['rays']} visits={s['node_visits']} tests={s['tri_tests']} "
              f"| refill {c['refill']/tot:.3f} traverse {c['traverse']/tot:.3f} shade {c['shade']/tot:.3f} "
              f"| cycles/ray {tot/ s['rays'] * 1.0:.0f} (sum over waves)")
        r.close()
