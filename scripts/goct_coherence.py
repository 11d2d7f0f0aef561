#!/usr/bin/env python3
"""Diagnostic: coherence of the HBM/L2 octant walk's loads (bunny proxy 4K, fused frames, 9 bounces), from a
build with -DRT_LDS_CONFLICTS=1 (lib/diag/librt_hip_lds_conflicts.so, selected with RT_HIP_LIB): per node step
and per triangle step, the active lanes, the distinct records they read, the distinct 128-B lines, and the
steps whose active lanes all read one record (a scalar load could serve those without the address unit).
Usage: RT_HIP_LIB=... python scripts/goct_coherence.py [frames]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mini-opencl-raytracer_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import clrt  # noqa: E402
from clrt import _native as N  # noqa: E402
from clrt import proxy  # noqa: E402
from hip_helpers import HipRenderer  # noqa: E402

frames = int(sys.argv[1]) if len(sys.argv) > 1 else 2
r = HipRenderer(proxy.bunny_proxy(), 3840, 2160, math=N.MATH_SHIPPED, stats=True)
r.frame(1, light_bounces=9, n_frames=frames if frames > 1 else None)
r.ctx.Finish()
s = r.k.stats()
r.close()
u = s["sched"]
raw = [u[k] for k in ("node_steps", "node_lanes", "tri_steps", "tri_lanes", "shade_rounds", "shade_lanes",
                      "refill_rounds", "refill_lanes", "other_lanes", "shade_wait", "free_wait", "reserved")]
print(f"bunny 4K, {frames} fused frames, 9 bounces: node visits {s['node_visits']}, triangle tests {s['tri_tests']}")
for name, o, steps in (("node steps", 0, raw[8]), ("triangle steps", 4, raw[9])):
    lanes, rec, lines, uni = raw[o:o + 4]
    print(f"{name:15s} {steps:12d}: lanes/step {lanes / max(1, steps):5.1f}, distinct records/step "
          f"{rec / max(1, steps):5.1f}, distinct 128-B lines/step {lines / max(1, steps):5.1f}, "
          f"one-record steps {uni / max(1, steps):.3f}")
print(f"node steps with <= 2 records {raw[10] / max(1, raw[8]):.3f}, <= 4 records {raw[11] / max(1, raw[8]):.3f}")
