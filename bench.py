#!/usr/bin/env python3
"""Benchmark: Mrays/s + ms/frame, 3840x2160 Cornell box, 8 spp path trace (BASELINE.json).

One *step* = one full 8-spp render of the workload: KernelEntry for frames 1..8 (9 light
bounces, the reference defaults) accumulated into one output buffer, then -- for N > 1 --
every rank's interleaved 8-row bands gathered to rank 0 over RCCL by the library
(rtCommEnqueueGatherBands, csrc/rt_comm.cpp).  Scene and output stay resident in HBM; nothing
is read back to the host inside the timed region.  The process never imports torch: the only
HIP runtime in it is the one librt_hip.so links (/opt/rocm).

  python bench.py [--gpus N --steps K --warmup W]
  (N > 1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...; the
  launcher only starts the processes -- ranks meet through the library's RCCL communicator)

Rays are counted as the reference's Intersect() calls over all bounces and frames
(SURVEY.md 8(d)); the count comes from an instrumented pass before the timed region and is
deterministic (the HIP path is bit-exact with the reference, tests/).

Roofline of the dominant kernel (KernelEntry's render launch), per launch:
  * bound "valu": the kernel is VALU-issue bound (the Cornell scene lives in LDS; HBM sees the
    output only).  achieved = VALU wave-instructions per launch (rocprofv3 SQ_INSTS_VALU of the
    same command and build, profiles/pmc.json) / the launch's time measured live here with HIP
    events on the kernel's streams (launch_ms: consecutive fused renders overlap, so the interval
    between their ends, period_ms; kernel_ms is each launch's own event span); peak = 1,024
    SIMDs x 2.4 GHz / 2 cycles per wave64 VALU instruction (MI355X_MICROARCH.md).
    frac = achieved / peak.
  * lane_util = SQ_THREAD_CYCLES_VALU / (64 x SQ_INSTS_VALU): active lanes per issued VALU op.
  * traffic / hbm_frac: measured HBM bytes per launch ((2 FETCH_SIZE + WRITE_SIZE) KiB, the
    guide's gfx950 correction) and their rate against 8 TB/s.
  * alg_bytes_per_launch / alg_gbs: SURVEY 8(d)'s algorithmic bytes (48 B per node visit and
    triangle test, 164 B per closest hit, 32 B output RMW per pixel) -- a plain number: most of
    those bytes are LDS reads, not HBM traffic.
cpu_baseline: the reference kernel itself (kernel_bvh.cl compiled unmodified for x86-64,
oracle/_ref/libref_cpu.so) over all 8 frames of the same render on the host cores, rank 0,
N = 1 only.
"""
import argparse
import glob
import hashlib
import json
import os
import sys
import shutil
import tempfile
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "mini-opencl-raytracer_amd"))

import clrt  # noqa: E402
from clrt import _native as N  # noqa: E402
from clrt import multigpu as mg  # noqa: E402

HBM_PEAK_GBS = 8000.0
SIMDS = 256 * 4                    # MI355X: 256 CUs x 4 SIMD-32
VALU_PEAK = SIMDS * 2.4e9 / 2.0    # wave64 VALU instructions per second (2 cycles each)
CAMERA = ((0.0, -25.0, 8.5), (0.0, 1.0, 0.0), (0.0, 0.0, 1.0))
PMC_PATH = os.path.join(REPO, "profiles", "pmc.json")


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--width", type=int, default=3840)
    p.add_argument("--height", type=int, default=2160)
    p.add_argument("--frames", type=int, default=8)
    p.add_argument("--bounces", type=int, default=9)
    p.add_argument("--math", choices=["pinned", "devicelib", "shipped"], default="shipped",
                   help="shipped (default): bit-exact with the reference as clBuildProgram builds it; "
                        "devicelib: ... with -ffp-contract=off -cl-fp32-correctly-rounded-divide-sqrt; "
                        "pinned: bit-exact with the CPU oracle")
    p.add_argument("--bvh", choices=["host", "device", "device-lbvh"], default="host",
                   help="host: the reference's SAH build (default); device: rtBuildBVH (PLOC); "
                        "device-lbvh: rtBuildBVHEx linear BVH")
    p.add_argument("--scene", choices=["cornell", "bunny"], default="cornell",
                   help="bunny = the deterministic ~70k-triangle proxy (config 5)")
    p.add_argument("--sched", choices=["tiles", "step", "wavefront"], default="step",
                   help="step (default): per-wave state machine in one persistent launch; wavefront: "
                        "extend + shade launches per bounce over HBM ray queues (SURVEY 8(f.3))")
    p.add_argument("--launch", choices=["fused", "per-frame"], default="fused",
                   help="fused: the F frames of a step as one rtEnqueueKernelFrames call (one step launch "
                        "over (frame, pixel) work items + the per-pixel accumulation); per-frame: one "
                        "rtEnqueueKernel per frame, as the reference's RenderFrame loop. Same bits.")
    p.add_argument("--tune", action="append", default=[], metavar="NAME=VALUE",
                   help="rtKernelSetTuning parameter (clrt._native.TUNING names); results unchanged")
    p.add_argument("--no-accum-overlap", action="store_true",
                   help="fused frames: accumulate on the main stream (rtContextSetAccumOverlap 0)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-drop-in", action="store_true",
                   help="skip the extra per-frame (drop-in RenderFrame loop) measurement reported beside "
                        "the fused headline at N = 1")
    p.add_argument("--no-configs", action="store_true",
                   help="skip the other BASELINE configs timed after the headline at N = 1 (the `configs` key)")
    p.add_argument("--cpu-threads", type=int, default=16)
    p.add_argument("--gather-sync", action="store_true",
                   help="N>1: wait for each step's gather before queueing the next step (no pipelining)")
    p.add_argument("--force-dist", action="store_true",
                   help="run the N>1 flow (RCCL communicator + gather) even at WORLD_SIZE 1")
    p.add_argument("--transport", choices=["copy", "rccl", "copy-ipc"], default="copy",
                   help="N>1: how the gather moves the bands (rtCommSetTransport): copy engines over xGMI "
                        "(default), RCCL send/recv kernels, or copy engines linked by IPC handles even at "
                        "world size 1 (the multi-process path)")
    p.add_argument("--shared-world", action="store_true",
                   help="N>1 with every rank on GPU 0 and no RCCL (rtCommInitShared: setup through files, "
                        "gathers over IPC mappings on the copy engines) -- the N>1 orchestration on a one-GPU box; "
                        "not a scaling measurement (the ranks share one GPU)")
    p.add_argument("--check-gather", action="store_true",
                   help="after timing, rank 0 renders the whole frame unsharded and checks the gathered "
                        "image against it byte for byte")
    p.add_argument("--fail-links", action="store_true",
                   help="test hook (rtCommSetOption RT_COMM_OPT_FAIL_LINKS): this rank reports its copy-engine "
                        "links as broken, so the world takes the RCCL fallback -- which the line then reports")
    return p.parse_args(argv)


class Rank:
    """One GPU's share of the image: the interleaved 8-row bands b % world == rank, rendered
    at their global positions (global seeds)."""

    def __init__(self, scene, args, device, comm=None):
        self.args = args
        W, H = args.width, args.height
        self.W, self.H = W, H
        self.ctx = comm.ctx if comm is not None else clrt.CLContext(device)
        world, rank = (comm.nranks, comm.rank) if comm is not None else (1, 0)
        self.bands = mg.rank_bands(H, world, rank)
        self.pixels = sum(min(H, (b + 1) * mg.BAND_ROWS) - b * mg.BAND_ROWS for b in self.bands) * W
        flags = N.MEM_READ_ONLY | N.MEM_COPY_HOST_PTR
        self.bufs = [self.ctx.create_buffer(flags, a.nbytes, a)
                     for a in (scene.triangles, scene.nodes, scene.materials)]
        self.out = self.ctx.create_buffer(N.MEM_READ_WRITE, W * H * 16)
        self.k = make_kernel(self.ctx, self.bufs, self.out, args)
        if comm is not None:
            comm.shard(self.k)
        if args.no_accum_overlap:
            self.ctx.set_accum_overlap(False)

    def render(self, k=None):
        """frames 1..F accumulated (RenderFrame's m_FrameCount sequence): one launch per frame,
        or (--launch fused, default) one rtEnqueueKernelFrames call -- the same bits."""
        k = k or self.k
        if self.args.launch == "fused":
            k.set_uint(N.FRAME_COUNT, 1)
            self.ctx.ExecuteKernelFrames(k, self.W * self.H, self.args.frames)
            return
        for f in range(1, self.args.frames + 1):
            k.set_uint(N.FRAME_COUNT, f)
            self.ctx.ExecuteKernel(k, self.W * self.H)

    def finish(self):
        self.ctx.Finish()

    def release(self):
        self.finish()
        self.k.release()
        for b in self.bufs + [self.out]:
            b.release()
        self.ctx.release()


def make_kernel(ctx, bufs, out, args):
    k = clrt.CLKernel(ctx, "KernelEntry")
    k.set_buffer(N.BUFFER_OUT, out)
    k.set_buffer(N.BUFFER_SCENE, bufs[0])
    k.set_buffer(N.BUFFER_NODE, bufs[1])
    k.set_buffer(N.BUFFER_MATERIAL, bufs[2])
    k.set_int(N.WIDTH, args.width)
    k.set_int(N.HEIGHT, args.height)
    k.set_uint(N.FRAME_SEED, 0)
    k.set_int(N.LIGHT_BOUNCES, args.bounces)
    k.set_int(N.LIGHT_TYPE, 0)
    k.set_float(N.SKYBOX_INTENSITY, 1.0)
    k.set_float3(N.CAMERA_POS, CAMERA[0])
    k.set_float3(N.CAMERA_FRONT, CAMERA[1])
    k.set_float3(N.CAMERA_UP, CAMERA[2])
    k.set_math_mode({"pinned": N.MATH_PINNED, "devicelib": N.MATH_DEVICELIB, "shipped": N.MATH_SHIPPED}[args.math])
    k.set_schedule({"tiles": N.SCHED_TILES, "step": N.SCHED_STEP, "wavefront": N.SCHED_WAVEFRONT}[args.sched])
    for t in args.tune:
        name, value = t.split("=", 1)
        k.set_tuning(name, int(value))
    return k


def load_scene(args, device=0):
    if args.scene == "bunny":
        from clrt import proxy as clrt_proxy
        scene = clrt_proxy.bunny_proxy()
    else:
        scene = clrt.scene.cornell()
    if args.bvh.startswith("device"):  # BVH built on the GPU (rtBuildBVHEx)
        if args.scene == "bunny":
            raw = clrt.scene.load_obj(os.path.join(clrt_proxy.GEN_DIR, "bunny_proxy.obj"), build=False)
            ft, fm = raw.triangles, raw.materials
        else:
            z = np.load(clrt.scene.CORNELL_NPZ, allow_pickle=False)
            ft, fm = z["triangles"].view(N.TRIANGLE_DTYPE), z["materials"].view(N.MATERIAL_DTYPE)
        scene = clrt.scene.build_bvh_device(ft, fm, 4, device=device,
                                            method="lbvh" if args.bvh == "device-lbvh" else "ploc")
    return scene


# The other BASELINE configs, timed in the same N = 1 run after the headline (rank 0 only): each
# on its own context with its own count pass, warm-up and timed loop, priced by its own PMC key.
# `value` stays the headline's (config 3).  Config 1 is the reference's CPU-only plumbing case
# and config 4 the 8-GPU run (the driver's scaling bench).
EXTRA_CONFIGS = (
    ("cfg5_bunny", {"scene": "bunny"}, 10,
     "BASELINE config 5 on one GPU: the bunny-class proxy (69,692 triangles, 48k-node BVH in HBM/L2), "
     "3840x2160, 8 spp, 9 bounces"),
    ("cfg2_1080p", {"width": 1920, "height": 1080, "bounces": 2, "frames": 1}, 40,
     "BASELINE config 2: 1920x1080 Cornell, 1 spp, 2 bounces (primary + one secondary ray per pixel: "
     "the reference has no shadow rays, SURVEY.md 7 hard part 6)"),
    ("cfg3_pinned", {"math": "pinned"}, 10,
     "BASELINE config 3 in the CPU-parity math (pinned: bit-exact with the reference kernel built for the "
     "CPU, tests/test_ref_cpu.py, tests/test_gpu_parity.py)"),
)


def time_config(over, steps, device):
    """One extra config: its own context, count pass, 2 warm-up steps and `steps` timed steps."""
    a = parse([])
    a.__dict__.update(over)
    r = Rank(load_scene(a, device), a, device)
    st = count_pass(r)
    local_counts = np.array([st["rays"], st["node_visits"], st["tri_tests"], st["hits"]], np.float64)
    for _ in range(2):
        r.render()
    r.k.set_timing(True)
    r.k.reset_stats()
    r.finish()
    t0 = time.perf_counter()
    for _ in range(steps):
        r.render()
    r.finish()
    dt = time.perf_counter() - t0
    ks = r.k.stats()
    r.k.set_timing(False)
    launches = max(1, ks["launches"])
    fpl = a.frames if a.launch == "fused" else 1
    period = ks["render_period_ms"] if fpl > 1 else 0.0
    rl = roofline(a, 1, fpl, ks["kernel_ms"] / launches, period, local_counts, r.pixels)
    r.release()
    ms_step = dt * 1e3 / steps
    return {"workload": f"{a.scene} {a.width}x{a.height} {a.frames}spp {a.bounces}-bounce path trace",
            "math": a.math, "steps": steps, "ms_per_step": round(ms_step, 4),
            "ms_per_frame": round(ms_step / a.frames, 4),
            "value": round(local_counts[0] * steps / dt / 1e6, 3), "unit": "Mrays/s",
            "rays_per_step": int(local_counts[0]), "roofline": rl}


def extra_configs(device):
    out = {}
    for name, over, steps, desc in EXTRA_CONFIGS:
        t0 = time.perf_counter()
        out[name] = {"config": desc, **time_config(over, steps, device),
                     "wall_s": None}
        out[name]["wall_s"] = round(time.perf_counter() - t0, 2)
    return out


def count_pass(r):
    r.k.set_stats(True)
    r.k.reset_stats()
    r.render()
    r.finish()
    s = r.k.stats()
    r.k.set_stats(False)
    r.k.reset_stats()
    return s


def kernel_source_hash() -> str:
    """Hash of everything that shapes the render kernel's instruction stream: the PMC numbers in
    profiles/pmc.json are only valid for the build they were measured on."""
    h = hashlib.sha1()
    files = sorted(glob.glob(os.path.join(REPO, "mini-opencl-raytracer_amd", "csrc", "rt_kernels*"))
                   + [os.path.join(REPO, "mini-opencl-raytracer_amd", "csrc", "rt_math.hpp"),
                      os.path.join(REPO, "mini-opencl-raytracer_amd", "csrc", "rt_capi.cpp"),  # launch parameters
                      os.path.join(REPO, "include", "rt_pinned_math.h"),
                      os.path.join(REPO, "include", "rt_cl_types.h"),
                      os.path.join(REPO, "mini-opencl-raytracer_amd", "Makefile")])
    for f in files:
        with open(f, "rb") as fh:
            h.update(os.path.basename(f).encode() + b"\0" + fh.read())
    return h.hexdigest()[:16]


def workload_key(args, world, frames_per_launch):
    return (f"{args.scene}_{args.width}x{args.height}_f{args.frames}_b{args.bounces}_{args.math}_{args.sched}_n{world}"
            + ("_fused" if frames_per_launch > 1 else ""))


def pinned_rays(r, args):
    """Intersect() calls of the step under the pinned builtins -- exactly the CPU reference
    build's count (HIP pinned == C oracle == kernel_bvh.cl on the CPU, bit for bit and counter
    for counter: tests/test_gpu_parity.py, tests/test_ref_cpu.py)."""
    k = make_kernel(r.ctx, r.bufs, r.out, args)
    k.set_math_mode(N.MATH_PINNED)
    k.set_stats(True)
    r.render(k)
    r.finish()
    rays = k.stats()["rays"]
    k.release()
    return rays


def cpu_baseline(scene, args, rays_per_step):
    """The reference kernel (kernel_bvh.cl, compiled for x86-64) over all frames of the step;
    rays_per_step: the pinned-math count of the same render."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import refcpu
    W, H = args.width, args.height
    threads = max(1, min(args.cpu_threads, len(os.sched_getaffinity(0))))
    res = np.zeros((W * H, 4), np.float32)
    t0 = time.perf_counter()
    for f in range(1, args.frames + 1):
        refcpu.render(scene, W, H, frame_count=f, light_bounces=args.bounces, result=res, threads=threads)
    dt = time.perf_counter() - t0
    return {"value": rays_per_step / dt / 1e6, "unit": "Mrays/s", "cores": threads, "kind": "reference",
            "sample": f"the whole step: frames 1-{args.frames} of the {W}x{H} {args.bounces}-bounce render, "
                      f"/root/reference/kernel_bvh.cl compiled unmodified for x86-64 (pinned builtins), "
                      f"{threads} threads ({int(rays_per_step)} rays, {dt:.2f} s wall)",
            "ms_per_frame": dt * 1e3 / args.frames}


def drop_in(r, args, rays_per_step, steps=3):
    """The drop-in path beside the fused headline: the same step as the reference's RenderFrame
    loop issues it -- one rtEnqueueKernel (ExecuteKernel) per frame -- (a) queued back to back for
    `steps` steps (the library coalesces queued frames into fused launches, RT_TUNE_PERFRAME_BATCH),
    (b) with RenderFrame's per-frame ReadBuffer of the W*H*16-B image + Finish (CLRaytracer.cpp:
    57-59; PCIe read-back inside, so never the headline), one step."""
    k = make_kernel(r.ctx, r.bufs, r.out, args)
    W, H, F = args.width, args.height, args.frames

    def frames(readback, host):
        for f in range(1, F + 1):
            k.set_uint(N.FRAME_COUNT, f)
            r.ctx.ExecuteKernel(k, W * H)
            if readback:
                r.ctx.ReadBuffer(r.out, host, blocking=True)
    host = np.ones((W * H, 4), np.float32)  # resident pages, as the reference's long-lived image vector
    frames(False, host)
    r.ctx.ReadBuffer(r.out, host, blocking=True)  # (first read-back into these pages, untimed)
    r.finish()
    out = {"launch": "per frame (rtEnqueueKernel, the reference's RenderFrame loop)"}
    for name, rb, n in (("queued", False, steps), ("with_readback", True, 1)):
        t0 = time.perf_counter()
        for _ in range(n):
            frames(rb, host)
        r.finish()
        dt = (time.perf_counter() - t0) / n
        out[name] = {"ms_per_frame": round(dt * 1e3 / F, 4), "value": round(rays_per_step / dt / 1e6, 1),
                     "unit": "Mrays/s"}
    out["with_readback"]["note"] = f"ReadBuffer of {W * H * 16 / 1e6:.1f} MB + Finish after every frame, as RenderFrame does"
    k.release()
    return out


def roofline(args, world, frames_per_launch, kernel_ms, period_ms, local_counts, tile_px):
    alg_bytes = ((48 * local_counts[1] + 48 * local_counts[2] + 164 * local_counts[3]) / args.frames
                 + 32 * tile_px) * frames_per_launch
    # per-launch time: back-to-back fused renders overlap (one stream per radiance set, each
    # starts on the CUs the previous one's draining waves free), so a launch's own event span
    # (kernel_ms) also holds its wait for the previous launch; the interval between the ends of
    # consecutive launches (period_ms, HIP events on the render streams) is the time each launch
    # costs -- the denominator here.  Per-frame / unfused launches: the span itself.
    launch_ms = period_ms if period_ms > 0 else kernel_ms
    rl = {"bound": "valu", "achieved": None, "peak": VALU_PEAK, "unit": "VALU wave-instructions/s",
          "frac": None, "traffic": None, "kernel": "KernelEntry", "launch_ms": round(launch_ms, 4),
          "kernel_ms": round(kernel_ms, 4), "period_ms": round(period_ms, 4) if period_ms > 0 else None,
          "frames_per_launch": frames_per_launch, "lane_util": None, "hbm_frac": None,
          "alg_bytes_per_launch": int(alg_bytes),
          "alg_note": "SURVEY 8(d) byte model (48 B per node visit and triangle test, 164 B per closest hit, "
                      "32 B per pixel): mostly LDS reads, not HBM traffic -- not a bound; HBM is `traffic`",
          "alg_gbs": round(alg_bytes / (launch_ms * 1e-3) / 1e9, 2) if launch_ms > 0 else None,
          "pmc": None}
    kernel_ms = launch_ms
    key = workload_key(args, world, frames_per_launch)
    db = json.load(open(PMC_PATH)) if os.path.exists(PMC_PATH) else {}
    e = db.get(key)
    if e is None or kernel_ms <= 0:
        rl["pmc"] = f"no PMC pass for {key} in profiles/pmc.json"
        return rl
    src = kernel_source_hash()
    insts = e["SQ_INSTS_VALU"]
    achieved = insts / (kernel_ms * 1e-3)
    rl["achieved"] = round(achieved, 1)
    rl["frac"] = round(achieved / VALU_PEAK, 4)
    rl["lane_util"] = round(e["SQ_THREAD_CYCLES_VALU"] / (64.0 * insts), 4) if "SQ_THREAD_CYCLES_VALU" in e else None
    if "hbm_bytes_per_launch" in e:
        rl["traffic"] = int(e["hbm_bytes_per_launch"])
        rl["hbm_frac"] = round(e["hbm_bytes_per_launch"] / (kernel_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 5)
    if "TA_TA_BUSY_sum" in e and e.get("GRBM_GUI_ACTIVE"):
        # vector-memory address unit (TA) busy share of the launch: TA cycles summed over the 256
        # CUs against the busy cycles summed over the 8 XCDs -- the HBM/L2 octant walk's binding
        # resource (VALU issue is not: DESIGN.md section 5)
        rl["ta_busy"] = round(e["TA_TA_BUSY_sum"] / 256.0 / (e["GRBM_GUI_ACTIVE"] / 8.0), 4)
    acc = e.get("accum")
    if acc and "SQ_INSTS_VALU" in acc:
        # the fused launch's accumulation (accum_frames, one per render launch) issues on the same
        # SIMDs while the next render runs: its VALU, and both kernels' VALU over the render period
        ai = acc["SQ_INSTS_VALU"]
        rl["accum_valu_insts_per_launch"] = int(ai)
        rl["accum_lane_util"] = (round(acc["SQ_THREAD_CYCLES_VALU"] / (64.0 * ai), 4)
                                 if "SQ_THREAD_CYCLES_VALU" in acc and ai else None)
        rl["frac_with_accum"] = round((insts + ai) / (kernel_ms * 1e-3) / VALU_PEAK, 4)
    else:
        rl["accum_valu_insts_per_launch"] = None
        rl["frac_with_accum"] = None
    rl["pmc"] = {"file": "profiles/pmc.json", "key": key, "valu_insts_per_launch": int(insts),
                 "kernel_ms_in_pmc_pass": e.get("kernel_ms"), "source_hash": e.get("source_hash"),
                 "stale": e.get("source_hash") != src}
    return rl


def comm_report(comm, ks, args):
    """What the N > 1 flow actually ran, rank by rank, gathered to every rank (collective): the
    communicator's world size, each rank's effective transport (a world whose copy-engine links
    fail falls back to RCCL -- reported here, never hidden), its render launch time and its last
    gather's transfer time."""
    fields = 7
    launches = max(1, ks["launches"])
    st = comm.status()
    mine = [float(st["active_code"]), float(st["fallback"]),
            float([k for k, v in N.COMM_FALLBACK_NAMES.items() if v == st["fallback_reason"]][0]),
            ks["render_period_ms"] if ks["render_period_ms"] > 0 else ks["kernel_ms"] / launches,
            -1.0 if st["last_xfer_ms"] is None else st["last_xfer_ms"],
            float(st["bytes_per_gather"]), float(st["copies_per_gather"])]
    vec = np.zeros(comm.nranks * fields)
    vec[comm.rank * fields:(comm.rank + 1) * fields] = mine
    for i in range(0, len(vec), 64):  # (rtCommAllReduceF64 takes up to 64 values per call)
        vec[i:i + 64] = mg.Comm.allreduce([comm], [vec[i:i + 64]], N.COMM_SUM)[0]
    per = vec.reshape(comm.nranks, fields)
    ranks = [{"rank": q, "transport": N.COMM_TRANSPORT_NAMES[int(p[0])],
              "fallback": N.COMM_FALLBACK_NAMES[int(p[2])] if p[1] else None,
              "render_ms": round(p[3], 4), "last_gather_ms": None if p[4] < 0 else round(p[4], 4),
              "bytes_per_gather": int(p[5]), "copies_per_gather": int(p[6])} for q, p in enumerate(per)]
    kinds = sorted({r["transport"] for r in ranks})
    return {"nranks": comm.nranks, "requested": N.COMM_TRANSPORT_NAMES[comm.transport()[0]],
            "effective": kinds[0] if len(kinds) == 1 else "mixed: " + ", ".join(kinds),
            "fallback": any(r["fallback"] for r in ranks), "per_rank": ranks}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))

    scene = load_scene(args, local)

    comm = None
    shared_dir = None
    if world > 1 or args.force_dist:
        # one rank per GPU: rank 0's RCCL id reaches the others through a file on this node
        if args.shared_world:
            # every rank on GPU 0; rank 0 makes the world's exchange directory and hands its name to
            # the others through the same per-launch file as the RCCL id
            ctx = clrt.CLContext(0)
            tok = mg.file_rendezvous(rank, world, lambda: tempfile.mkdtemp(prefix="rt_shared_").encode().ljust(
                N.COMM_ID_BYTES, b"\0"))
            shared_dir = tok.rstrip(b"\0").decode()
            comm = mg.Comm.init_shared(ctx, world, rank, shared_dir)
        else:
            ctx = clrt.CLContext(local)
            uid = mg.file_rendezvous(rank, world, mg.Comm.unique_id)
            comm = mg.Comm.init_rank(ctx, world, uid, rank)
        mg.Comm.barrier([comm])
        if rank == 0:
            mg.rendezvous_cleanup()
    r = Rank(scene, args, local, comm)
    # the root assembles the image in a buffer of its own (an application's display image): the
    # gather then moves every rank's bands, the root's own included, so a world of one runs the
    # whole data path (pack, transfer, unpack)
    img = None
    if comm is not None:
        comm.set_transport({"rccl": N.COMM_TRANSPORT_RCCL, "copy": N.COMM_TRANSPORT_COPY_ENGINES,
                            "copy-ipc": N.COMM_TRANSPORT_COPY_ENGINES_IPC}[args.transport])
        if args.fail_links:
            comm.set_option(N.COMM_OPT_FAIL_LINKS, 1)
        if rank == 0:
            img = r.ctx.create_buffer(N.MEM_READ_WRITE, r.W * r.H * 16)

    # instrumented pass: ray / node / triangle / hit counts of one step on this rank
    st = count_pass(r)
    local_counts = np.array([st["rays"], st["node_visits"], st["tri_tests"], st["hits"]], np.float64)
    counts = local_counts
    if comm is not None:
        counts = mg.Comm.allreduce([comm], local_counts, N.COMM_SUM)[0]

    def step():
        r.render()  # steps are queued back to back (sync only around the timed region)
        if comm is not None:
            mg.Comm.gather_bands([comm], [r.out], r.W, r.H, root=0, dst=img)
            if args.gather_sync:
                r.finish()

    def sync_all():
        r.finish()
        if comm is not None:
            mg.Comm.barrier([comm])

    for _ in range(args.warmup):
        step()
    r.k.set_timing(True)
    r.k.reset_stats()
    sync_all()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    sync_all()
    elapsed = time.perf_counter() - t0
    ks = r.k.stats()
    r.k.set_timing(False)
    comm_line = None
    if comm is not None:
        elapsed = float(mg.Comm.allreduce([comm], [elapsed], N.COMM_MAX)[0][0])
        comm_line = comm_report(comm, ks, args)

    check = None
    if args.check_gather and comm is not None and rank == 0:
        # the gathered image (every rank's bands, through RCCL) against an unsharded render
        a = np.empty((r.H * r.W, 4), np.float32)
        r.ctx.ReadBuffer(img, a, blocking=True)
        ref_out = r.ctx.create_buffer(N.MEM_READ_WRITE, r.W * r.H * 16)
        kf = make_kernel(r.ctx, r.bufs, ref_out, args)
        r.render(kf)
        b = np.empty_like(a)
        r.ctx.ReadBuffer(ref_out, b, blocking=True)
        same = a.view(np.uint32)[:, :3] == b.view(np.uint32)[:, :3]
        if not same.all():
            raise SystemExit(f"check-gather: {int((~same).any(axis=1).sum())} pixels of the gathered image differ")
        check = f"gathered {r.W}x{r.H} image byte-identical to an unsharded render ({world} ranks)"
        print(f"check-gather: {check}", file=sys.stderr)
        kf.release()
        ref_out.release()
    if comm is not None:
        mg.Comm.barrier([comm])

    rays_per_step, visits, tests, hits = counts
    ms_step = elapsed * 1e3 / args.steps
    value = rays_per_step * args.steps / elapsed / 1e6
    launches = max(1, ks["launches"])
    kernel_ms = ks["kernel_ms"] / launches
    frames_per_launch = args.frames if (args.launch == "fused" and args.sched in ("step", "wavefront")) else 1
    period_ms = ks["render_period_ms"] if frames_per_launch > 1 and not args.no_accum_overlap else 0.0
    rl = roofline(args, world, frames_per_launch, kernel_ms, period_ms, local_counts, r.pixels)
    rl["accum_overlapped"] = frames_per_launch > 1 and not args.no_accum_overlap
    if not rl["accum_overlapped"] and frames_per_launch > 1:
        rl["accum_ms_per_launch"] = round(ks["accum_ms"] / launches, 4)
    if rank != 0:
        comm.destroy()
        if shared_dir:  # tell rank 0 this rank is done with the exchange files
            open(os.path.join(shared_dir, f"done_{rank}"), "w").close()
        return
    if shared_dir:  # the directory goes once every other rank has left it
        t0 = time.monotonic()
        while (time.monotonic() - t0 < 30 and
               not all(os.path.exists(os.path.join(shared_dir, f"done_{q}")) for q in range(1, world))):
            time.sleep(0.01)
        shutil.rmtree(shared_dir, ignore_errors=True)
    scene_name = "Cornell box" if args.scene == "cornell" else "bunny-class proxy, 69,692 triangles"
    line = {
        "metric": f"Mrays/s ({args.width}x{args.height} {scene_name}, {args.frames} spp, {args.bounces} bounces)",
        "value": round(value, 3),
        "unit": "Mrays/s",
        "n_gpus": comm.nranks if comm is not None else world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_step, 4),
        "ms_per_frame": round(ms_step / args.frames, 4),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "data": ("reference scene cornell.obj (scenes/cornell_scene.npz)" if args.scene == "cornell" else
                 "generated bunny-class proxy OBJ (clrt/proxy.py)") + "; rays generated in-kernel",
        "config": {"workload": f"{args.scene} {args.width}x{args.height} {args.frames}spp {args.bounces}-bounce path trace",
                   "width": args.width, "height": args.height, "frames": args.frames, "bounces": args.bounces,
                   "math": args.math, "schedule": args.sched, "launch": args.launch, "bvh": args.bvh,
                   "parallelism": f"interleaved 8-row bands x{comm.nranks if comm is not None else world}" + (
                       (" (shared world: every rank on GPU 0, no RCCL)" if args.shared_world else "") +
                       f" + gather to rank 0 over {comm_line['effective']}"
                       " (librt_hip rtCommEnqueueGatherBands"
                       + (", host-synchronised)" if args.gather_sync else ", pipelined with the next step)")
                       if comm is not None else ""),
                   "rays_per_step": int(rays_per_step), "samples_per_step": args.width * args.height * args.frames,
                   "tuning": args.tune or None},
        "roofline": rl,
    }
    if comm_line is not None:
        line["comm"] = comm_line
    if check:
        line["check_gather"] = check
    if world == 1 and comm is None and args.launch == "fused" and not args.no_drop_in:
        line["drop_in"] = drop_in(r, args, rays_per_step, steps=args.steps)
    if world == 1 and comm is None and not args.no_configs:
        line["configs"] = extra_configs(local)
    if world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(scene, args, pinned_rays(r, args))
    print(json.dumps(line))
    if comm is not None:
        comm.destroy()


if __name__ == "__main__":
    main()
