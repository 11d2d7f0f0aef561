#!/usr/bin/env python3
"""Diagnostic: modelled LDS bank-conflict cycles per read site of the step schedule's LDS walk
(4K Cornell, 8 fused frames, 9 bounces), from a build with -DRT_LDS_CONFLICTS=1
(scripts/build_variant.sh lds_conflicts "-DRT_LDS_CONFLICTS=1"; run with RT_HIP_LIB pointing at it).

Every node visit's A read (its B read is the same addresses + a constant offset: the same cycles)
and every triangle test's reads are modelled with the banking rules of MI355X_MICROARCH.md (LDS):
cycles per read = sum over lane groups of the largest number of distinct addresses sharing a
bank; ideal = one cycle per group with an active lane.  Alternatives are modelled on the same lane
populations: the octant planes at other strides, and the triangle's 4-byte e2.z read from a dense
float array.  Usage: RT_HIP_LIB=... python scripts/lds_conflicts.py [frames]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mini-opencl-raytracer_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import clrt  # noqa: E402
from clrt import _native as N  # noqa: E402
from hip_helpers import HipRenderer  # noqa: E402

frames = int(sys.argv[1]) if len(sys.argv) > 1 else 8
W, H = 3840, 2160
r = HipRenderer(clrt.scene.cornell(), W, H, math=N.MATH_SHIPPED, stats=True)
r.frame(1, light_bounces=9, n_frames=frames if frames > 1 else None)
r.ctx.Finish()
s = r.k.stats()
r.close()
u = s["sched"]
raw = [u[k] for k in ("node_steps", "node_lanes", "tri_steps", "tri_lanes", "shade_rounds", "shade_lanes",
                      "refill_rounds", "refill_lanes", "other_lanes", "shade_wait", "free_wait", "reserved")]
sites = [("node A read (octant planes, stride %d: current)" % 41, 0, 2),
         ("node A read, stride 43", 2, 2), ("node A read, stride 48", 4, 2),
         ("triangle 16-B reads (each of two)", 6, 2), ("triangle 4-B e2.z read (16-B stride: current)", 8, 2),
         ("triangle e2.z from a dense float array", 10, 2)]
print(f"4K Cornell, {frames} fused frames, 9 bounces: node visits {s['node_visits']}, triangle tests {s['tri_tests']}")
for name, i, _ in sites:
    ideal, cyc = raw[i], raw[i + 1]
    print(f"{name:52s} ideal {ideal:14d}  modelled {cyc:14d}  conflict cycles {cyc - ideal:14d}  "
          f"({(cyc - ideal) / max(1, cyc):.3f} of its cycles)")
node = 2 * (raw[1] - raw[0])
tri = 2 * (raw[7] - raw[6]) + (raw[9] - raw[8])
tot_c = 2 * raw[1] + 2 * raw[7] + raw[9]
print(f"walk total: modelled cycles {tot_c}, conflict cycles {node + tri} "
      f"(node reads {node}, triangle reads {tri}); ratio {(node + tri) / max(1, tot_c):.3f}")
