#!/usr/bin/env python3
"""Diagnostic: per-phase wave-cycle shares of the step schedule (stats variant, s_memtime).
Usage: phase_profile.py [step]   (env: RT_PHASE_SCENE=bunny, RT_PHASE_MATH, RT_PHASE_LB, RT_PHASE_FRAMES,
RT_PHASE_TUNE=name=value,..., RT_PHASE_W, RT_PHASE_H)"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mini-opencl-raytracer_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import clrt  # noqa: E402
from clrt import _native as N  # noqa: E402
from hip_helpers import HipRenderer  # noqa: E402

if os.environ.get("RT_PHASE_SCENE") == "bunny":
    from clrt import proxy
    sc = proxy.bunny_proxy()
else:
    sc = clrt.scene.cornell()
scheds = sys.argv[1:] or ["step"]
for name in scheds:
  sched = {"step": N.SCHED_STEP}[name]
  maths = [{"pinned": N.MATH_PINNED, "devicelib": N.MATH_DEVICELIB, "shipped": N.MATH_SHIPPED}[m]
           for m in os.environ.get("RT_PHASE_MATH", "shipped,devicelib,pinned").split(",")]
  lbs = [int(x) for x in os.environ.get("RT_PHASE_LB", "1,9").split(",")]
  for math in maths:
    for lb in lbs:
        r = HipRenderer(sc, int(os.environ.get("RT_PHASE_W", "3840")), int(os.environ.get("RT_PHASE_H", "2160")),
                        math=math, stats=True, sched=sched)
        for t in filter(None, os.environ.get("RT_PHASE_TUNE", "").split(",")):  # name=value,...
            r.k.set_tuning(t.split("=")[0], int(t.split("=")[1]))
        nf = int(os.environ.get("RT_PHASE_FRAMES", "8"))
        r.frame(1, light_bounces=lb, n_frames=nf if nf > 1 else None)
        r.ctx.Finish()
        s = r.k.stats()
        c = s["cycles"]
        tot = c["total"] or 1
        u = s["sched"]
        print(f"{name} math={math} lb={lb} rays={s['rays']} visits={s['node_visits']} tests={s['tri_tests']} "
              f"| refill {c['refill']/tot:.3f} traverse {c['traverse']/tot:.3f} shade {c['shade']/tot:.3f} "
              f"| lanes/step node {u['node_lanes']/max(1,u['node_steps']):.1f} ({u['node_steps']}) "
              f"tri {u['tri_lanes']/max(1,u['tri_steps']):.1f} ({u['tri_steps']}) "
              f"shade {u['shade_lanes']/max(1,u['shade_rounds']):.1f} ({u['shade_rounds']}) "
              f"refill {u['refill_lanes']/max(1,u['refill_rounds']):.1f} ({u['refill_rounds']}) "
              f"| per step: other {u['other_lanes']/max(1,u['node_steps']+u['tri_steps']):.1f} "
              f"shade-wait {u['shade_wait']/max(1,u['node_steps']+u['tri_steps']):.1f} "
              f"free {u['free_wait']/max(1,u['node_steps']+u['tri_steps']):.1f}")
        r.close()
