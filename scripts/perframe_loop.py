#!/usr/bin/env python3
"""The reference's RenderFrame loop on the C ABI: per frame one rtEnqueueKernel, a read-back of the
image (CLRaytracer.cpp:35-47: ExecuteKernel, ReadBuffer, Finish) -- or, with --no-readback, just
rtFinish.  Prints ms per frame.  usage: perframe_loop.py [--scene S] [--w W --h H] [--bounces B]
[--frames F] [--tune NAME=V ...] [--no-readback]"""
import argparse
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mini-opencl-raytracer_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import clrt  # noqa: E402
from clrt import _native as N  # noqa: E402
from hip_helpers import HipRenderer  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--scene", default="cornell")
p.add_argument("--w", type=int, default=3840)
p.add_argument("--h", type=int, default=2160)
p.add_argument("--bounces", type=int, default=9)
p.add_argument("--frames", type=int, default=16)
p.add_argument("--tune", action="append", default=[])
p.add_argument("--no-readback", action="store_true")
a = p.parse_args()
if a.scene == "bunny":
    from clrt import proxy
    sc = proxy.bunny_proxy()
else:
    sc = clrt.scene.cornell()
r = HipRenderer(sc, a.w, a.h, math=N.MATH_SHIPPED)
for t in a.tune:
    k, v = t.split("=")
    r.k.set_tuning(k, int(v))
host = np.zeros((a.w * a.h, 4), np.float32)


def frame(f):
    r.frame(f, light_bounces=a.bounces)
    if a.no_readback:
        r.ctx.Finish()
    else:
        r.ctx.ReadBuffer(r.out, host, blocking=True)


frame(1)
t0 = time.perf_counter()
for f in range(2, a.frames + 2):
    frame(f)
dt = (time.perf_counter() - t0) / a.frames * 1e3
print(f"{a.scene} {a.w}x{a.h} lb={a.bounces} {' '.join(a.tune) or 'default'} "
      f"{'finish' if a.no_readback else 'readback'}: {dt:.3f} ms/frame")
r.close()
