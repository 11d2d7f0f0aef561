#!/usr/bin/env python3
"""Emulate the per-rank work of an N-GPU run on one GPU: rank r of N renders the interleaved
8-row bands b % N == r of the 4K 8-spp frame (exactly what bench.py --gpus N gives it), one rank
after another.  Prints per-rank ms per 8-frame step and the strong-scaling efficiency
T1 / (N * max_r T_r).

RT_EMU_GATHER=1 adds the gather bench.py runs every step (rtCommEnqueueGatherBands): rank r's
context joins a loopback world of N contexts on this GPU (rtCommInitLoopback: pack on the
accumulation stream, two staging slots, copy-engine transfer into the root's receive slots,
unpack on the root's stream) in which only rank r renders; every step all N ranks pack and copy
and root 0 unpacks every other rank's bands into its own output, pipelined with the next step as
in bench.py.  All N ranks' copies then share THIS GPU's copy engines (N x 16.6 MB per 4K step at
N = 8, ~2.2 ms at 61 GB/s), where each real rank copies only its own share on its own engines:
with the copy-engine transport this measures one GPU's engines, not a rank's step -- a loose
upper bound (profiles/r04/rank_emulation_r04.txt).

usage: rank_emulation.py [N ...]   (env: RT_EMU_MATH, RT_EMU_SCENE=cornell|bunny, RT_EMU_STEPS,
       RT_EMU_FUSED=1: the 8 frames as one rtEnqueueKernelFrames call (default 1),
       RT_EMU_GATHER=1: include the gather, RT_EMU_TUNE=name=v,name=v: library tunings;
       RT_EMU_STEPS defaults to bench.py's 20 timed steps)"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mini-opencl-raytracer_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import clrt  # noqa: E402
from clrt import _native as N  # noqa: E402
from clrt import multigpu as mg  # noqa: E402
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
fused = os.environ.get("RT_EMU_FUSED", "1") == "1"
GATHER = os.environ.get("RT_EMU_GATHER", "0") == "1"
W, H, F = 3840, 2160, 8


def rank_step_ms(n, rank):
    """ms per step of rank `rank` of `n` (and its KernelEntry ms per step).  N = 1 never gathers:
    bench.py's one-GPU run has no communicator, so T1 is the plain render."""
    gather = GATHER and n > 1
    rs = [HipRenderer(sc, W, H, math=math) for _ in range(n if gather else 1)]
    me = rs[rank] if gather else rs[0]
    comms = mg.Comm.init_loopback([r.ctx for r in rs]) if gather else None
    if gather:
        for c, r in zip(comms, rs):
            c.shard(r.k)
    else:
        me.k.set_row_interleave(n, rank)
    for name, v in tunes:
        me.k.set_tuning(name, int(v))

    def step():
        if fused:
            me.frame(1, light_bounces=9, n_frames=F)
        else:
            for f in range(1, F + 1):
                me.frame(f, light_bounces=9)
        if gather:
            mg.Comm.gather_bands(comms, [r.out for r in rs], W, H, root=0)

    def finish():
        for r in rs:
            r.ctx.Finish()

    step()
    finish()
    me.k.set_timing(True)
    me.k.reset_stats()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    finish()
    el = (time.perf_counter() - t0) / steps * 1e3
    kern = me.k.stats()["kernel_ms"] / steps
    if gather:
        for c in comms:
            c.destroy()
    for r in rs:
        r.close()
    return el, kern


t1 = None
for n in [int(x) for x in sys.argv[1:]] or [1, 2, 4, 8]:
    per = [rank_step_ms(n, rank) for rank in range(n)]
    tmax = max(p[0] for p in per)
    if n == 1:
        t1 = tmax
    eff = t1 / (n * tmax) if t1 else float("nan")
    what = "render + gather" if GATHER and n > 1 else "render-only"
    print(f"N={n} ms/step per rank: " + " ".join(f"{p[0]:.3f}" for p in per) +
          " | KernelEntry ms/step: " + " ".join(f"{p[1]:.3f}" for p in per) +
          f" | max {tmax:.3f} | {what} strong-scaling efficiency {eff:.3f}", flush=True)
