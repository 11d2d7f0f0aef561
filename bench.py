#!/usr/bin/env python3
"""Benchmark: Mrays/s + ms/frame, 3840x2160 Cornell box, 8 spp path trace (BASELINE.json).

One *step* = one full 8-spp render of the workload: KernelEntry launched for frames
1..8 (9 light bounces, the reference defaults) into one accumulation buffer, then -- for
N > 1 -- the per-rank row tiles gathered to rank 0 over RCCL (torch.distributed "nccl").
Scene and output stay resident in HBM; nothing is read back to the host inside the
timed region.

  python bench.py [--gpus N --steps K --warmup W]
  (N > 1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...)

Rays are counted as the reference's Intersect() calls over all bounces and frames
(SURVEY.md 8(d)); the count comes from an instrumented pass before the timed region and
is deterministic (the HIP path is bit-exact with the oracle, tests/test_gpu_parity.py).

Roofline: the dominant kernel is KernelEntry.  achieved = algorithmic bytes per launch
(48*node_visits + 48*tri_tests + 164*hits + 32*W*H) / average launch
duration from HIP events recorded on the kernel's own stream during the timed region;
peak = 8000 GB/s (MI355X HBM3E).  traffic = HBM bytes per launch from rocprofv3 PMC
counters (profiles/traffic.json, written by scripts/profile.sh) when present.
cpu_baseline: the CPU oracle (a C restatement of kernel_bvh.cl) on the host cores, rank 0,
N = 1 only, on a bounded sample (frames 1-2 of the same 4K render).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "mini-opencl-raytracer_amd"))

import clrt  # noqa: E402
from clrt import _native as N  # noqa: E402
from clrt import multigpu as mg  # noqa: E402

HBM_PEAK_GBS = 8000.0
SIMDS = 256 * 4  # MI355X: 256 CUs x 4 SIMD-32
CAMERA = ((0.0, -25.0, 8.5), (0.0, 1.0, 0.0), (0.0, 0.0, 1.0))


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--pack-stream", choices=["accum", "main"], default="accum",
                   help="pipelined RCCL gather: pack each step's bands on the accumulation stream "
                        "(the next render does not wait for the accumulation) or on the main stream")
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--width", type=int, default=3840)
    p.add_argument("--height", type=int, default=2160)
    p.add_argument("--frames", type=int, default=8)
    p.add_argument("--bounces", type=int, default=9)
    p.add_argument("--math", choices=["pinned", "devicelib", "shipped"], default="shipped",
                   help="shipped (default): bit-exact with the reference as clBuildProgram builds it; "
                        "devicelib: ... with -ffp-contract=off -cl-fp32-correctly-rounded-divide-sqrt; "
                        "pinned: bit-exact with the CPU oracle")
    p.add_argument("--bvh", choices=["host", "device"], default="host",
                   help="host: the reference's SAH build (default); device: rtBuildBVH linear BVH")
    p.add_argument("--scene", choices=["cornell", "bunny"], default="cornell",
                   help="bunny = the deterministic ~70k-triangle proxy (config 5)")
    p.add_argument("--sched", choices=["regen", "tiles", "step", "pool"], default="step")
    p.add_argument("--launch", choices=["fused", "per-frame"], default="fused",
                   help="fused: the F frames of a step as one rtEnqueueKernelFrames call (one step launch "
                        "over (frame, pixel) work items + the per-pixel accumulation); per-frame: one "
                        "rtEnqueueKernel per frame, as the reference's RenderFrame loop. Same bits.")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-threads", type=int, default=16)
    p.add_argument("--no-overlap", action="store_true",
                   help="N>1 nccl: gather after each step with a host sync instead of pipelining it")
    p.add_argument("--force-dist", action="store_true",
                   help="run the N>1 flow even at WORLD_SIZE 1 (exercises the RCCL path on one GPU)")
    p.add_argument("--check-gather", action="store_true",
                   help="after timing, check rank 0's bands in the gathered image (pipelined nccl)")
    p.add_argument("--dist-backend", choices=["nccl", "gloo"], default="nccl",
                   help="gloo = dry run of the N>1 flow (host-staged gather; ranks may share a GPU)")
    return p.parse_args()


class Rank:
    """One GPU's share of the image: the interleaved 8-row bands b % world == rank
    (clrt.multigpu), rendered at their global positions (global seeds)."""

    def __init__(self, scene, args, device, rank, world):
        self.args = args
        W, H = args.width, args.height
        self.W, self.H = W, H
        self.rank, self.world = rank, world
        self.bands = mg.rank_bands(H, world, rank)
        self.pixels = sum(min(H, (b + 1) * mg.BAND_ROWS) - b * mg.BAND_ROWS for b in self.bands) * W
        self.ctx = clrt.CLContext(device)
        self.k = clrt.CLKernel(self.ctx, "KernelEntry")
        flags = N.MEM_READ_ONLY | N.MEM_COPY_HOST_PTR
        self.bufs = [self.ctx.create_buffer(flags, a.nbytes, a)
                     for a in (scene.triangles, scene.nodes, scene.materials)]
        self.out = self.ctx.create_buffer(N.MEM_READ_WRITE, W * H * 16)
        k = self.k
        k.set_buffer(N.BUFFER_OUT, self.out)
        k.set_buffer(N.BUFFER_SCENE, self.bufs[0])
        k.set_buffer(N.BUFFER_NODE, self.bufs[1])
        k.set_buffer(N.BUFFER_MATERIAL, self.bufs[2])
        k.set_int(N.WIDTH, W)
        k.set_int(N.HEIGHT, H)
        k.set_uint(N.FRAME_SEED, 0)
        k.set_int(N.LIGHT_BOUNCES, args.bounces)
        k.set_int(N.LIGHT_TYPE, 0)
        k.set_float(N.SKYBOX_INTENSITY, 1.0)
        k.set_float3(N.CAMERA_POS, CAMERA[0])
        k.set_float3(N.CAMERA_FRONT, CAMERA[1])
        k.set_float3(N.CAMERA_UP, CAMERA[2])
        k.set_math_mode({"pinned": N.MATH_PINNED, "devicelib": N.MATH_DEVICELIB, "shipped": N.MATH_SHIPPED}[args.math])
        k.set_schedule({"tiles": N.SCHED_TILES, "regen": N.SCHED_REGEN, "step": N.SCHED_STEP,
                        "pool": N.SCHED_POOL}[args.sched])
        k.set_row_interleave(world, rank)

    def render(self):
        """frames 1..F accumulated (RenderFrame's m_FrameCount sequence): one launch per frame,
        or (--launch fused, default) one rtEnqueueKernelFrames call -- the same bits."""
        if self.args.launch == "fused":
            self.k.set_uint(N.FRAME_COUNT, 1)
            self.ctx.ExecuteKernelFrames(self.k, self.W * self.H, self.args.frames)
            return
        for f in range(1, self.args.frames + 1):
            self.k.set_uint(N.FRAME_COUNT, f)
            self.ctx.ExecuteKernel(self.k, self.W * self.H)

    def finish(self):
        self.ctx.Finish()


def count_pass(r):
    r.k.set_stats(True)
    r.k.reset_stats()
    r.render()
    r.finish()
    s = r.k.stats()
    r.k.set_stats(False)
    r.k.reset_stats()
    return s


def cpu_baseline(scene, args):
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle
    W, H = args.width, args.height
    threads = max(1, min(args.cpu_threads, len(os.sched_getaffinity(0))))
    res = np.zeros((W * H, 4), np.float32)
    rays = 0
    t0 = time.perf_counter()
    sample_frames = 2
    for f in range(1, sample_frames + 1):
        res, _, _, c = oracle.render(scene, W, H, frame_count=f, light_bounces=args.bounces, result=res,
                                     threads=threads)
        rays += c["rays"]
    dt = time.perf_counter() - t0
    return {"value": rays / dt / 1e6, "unit": "Mrays/s", "cores": threads, "kind": "port",
            "sample": f"frames 1-{sample_frames} of the same {W}x{H} {args.bounces}-bounce render, all pixels "
                      f"({rays} rays, {dt:.2f} s wall)"}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    device = local
    if world > 1 or args.force_dist:
        import torch
        import torch.distributed as dist_mod
        if args.dist_backend == "nccl":
            torch.cuda.set_device(local)
            dist_mod.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            device = local % max(1, torch.cuda.device_count())
            torch.cuda.set_device(device)
            dist_mod.init_process_group("gloo")
        dist = dist_mod

    if args.scene == "bunny":
        from clrt import proxy as clrt_proxy
        scene = clrt_proxy.bunny_proxy()
    else:
        scene = clrt.scene.cornell()
    if args.bvh == "device":  # linear BVH built on the GPU (rtBuildBVH)
        if args.scene == "bunny":
            raw = clrt.scene.load_obj(os.path.join(clrt_proxy.GEN_DIR, "bunny_proxy.obj"), build=False)
            ft, fm = raw.triangles, raw.materials
        else:
            z = np.load(clrt.scene.CORNELL_NPZ, allow_pickle=False)
            ft, fm = z["triangles"].view(N.TRIANGLE_DTYPE), z["materials"].view(N.MATERIAL_DTYPE)
        scene = clrt.scene.build_bvh_device(ft, fm, 4, device=device)
    r = Rank(scene, args, device, rank, world)

    # instrumented pass: ray / node / triangle / hit counts of one step on this rank
    st = count_pass(r)
    counts = np.array([st["rays"], st["node_visits"], st["tri_tests"], st["hits"]], np.float64)

    gather = land_all = None
    final = None
    if dist is not None:
        import torch
        nbytes = mg.staging_bytes(r.W, r.H, world)
        plans = [mg.pack_plan(r.W, r.H, world, q) for q in range(world)]
        if args.dist_backend == "nccl" and not args.no_overlap:
            # Pipelined: step k's staging buffer is gathered on RCCL's stream while step k+1
            # renders on the kernel's stream; rank 0 unpacks step k into the final image on a
            # side stream, so its render stream never carries the unpack copies (at N = 8 that
            # is 7 x 16.6 MB per step that would otherwise make rank 0 the slowest).  Two
            # staging slots; every hand-off is a stream-side event wait (no host sync), and
            # the timed region ends with the last gather landed.
            # The pack of step k runs on the context's accumulation stream right after step k's
            # accumulation (rtContextSetReadbackOnAccumStream), so the kernel stream goes straight
            # on to step k+1's render and the accumulation keeps overlapping it at N > 1 too; the
            # gather is issued from its own stream after the pack.
            dev = torch.device("cuda", device)
            r.ctx.set_readback_on_accum_stream(args.pack_stream == "accum")
            acc = torch.cuda.ExternalStream(r.ctx.accum_stream(), device=dev)
            issue = torch.cuda.Stream(device=dev)
            side = torch.cuda.Stream(device=dev)
            stages = [torch.empty(nbytes // 4, dtype=torch.float32, device=dev) for _ in range(2)]
            parts = [[torch.empty_like(stages[0]) for _ in range(world)] if rank == 0 else None for _ in range(2)]
            final = torch.zeros(r.W * r.H * 4, dtype=torch.float32, device=dev) if rank == 0 else None
            pending = [None, None]
            landed = [None, None]  # event on `side`: slot's gather (and unpack) done
            slot = [0]

            def unpack(part, plan):
                # mg.unpack_device as strided tensor copies (float32 elements: every offset and
                # pitch is a multiple of 16 B)
                for rc in plan:
                    dst = final.as_strided((rc.rows, rc.width // 4), (rc.img_pitch // 4, 1), rc.img_offset // 4)
                    src = part[rc.stage_offset // 4: rc.stage_offset // 4 + rc.rows * rc.width // 4]
                    dst.copy_(src.view(rc.rows, rc.width // 4))

            def land(s):
                if pending[s] is None:
                    return
                with torch.cuda.stream(side):
                    pending[s].wait()
                    if rank == 0:
                        for q in range(world):
                            unpack(parts[s][q], plans[q])
                    landed[s] = torch.cuda.Event()
                    landed[s].record(side)
                pending[s] = None

            def gather():
                s = slot[0]
                slot[0] ^= 1
                land(s ^ 1)
                if landed[s] is not None:  # slot s's previous gather/unpack (a step ago) is done
                    acc.wait_event(landed[s])
                mg.pack_device(r.ctx, r.out, plans[rank], stages[s].data_ptr())  # on `acc`
                issue.wait_stream(acc)
                with torch.cuda.stream(issue):
                    pending[s] = dist.gather(stages[s], parts[s], dst=0, async_op=True)

            def land_all():
                land(0)
                land(1)
        else:
            stage = torch.empty(nbytes // 4, dtype=torch.float32, device=f"cuda:{device}")
            host_staged = args.dist_backend == "gloo"

            def gather():
                # pack this rank's bands (2-D device copy on the kernel's stream), gather the
                # staging buffers to rank 0, unpack them into rank 0's image
                mg.pack_device(r.ctx, r.out, plans[rank], stage.data_ptr())
                r.finish()
                parts = mg.gather_to_root(dist, stage.cpu() if host_staged else stage, rank, world)
                if rank == 0:
                    if host_staged:
                        parts = [p.to(stage.device) for p in parts]
                    torch.cuda.current_stream().synchronize()
                    for q in range(1, world):
                        mg.unpack_device(r.ctx, parts[q].data_ptr(), plans[q], r.out)
                    r.finish()

        small_dev = f"cuda:{device}" if args.dist_backend == "nccl" else "cpu"
        tot = torch.tensor(counts, dtype=torch.float64, device=small_dev)
        dist.all_reduce(tot)
        counts = tot.cpu().numpy()

    def step():
        r.render()  # N = 1: steps are queued back to back (sync only around the timed region)
        if gather is not None:
            gather()

    def steps(n):
        for _ in range(n):
            step()
        if land_all is not None:
            land_all()

    steps(args.warmup)

    def sync_all():
        r.finish()
        if dist is not None:
            import torch
            torch.cuda.synchronize()
            dist.barrier()

    r.k.set_timing(True)
    r.k.reset_stats()
    sync_all()
    t0 = time.perf_counter()
    steps(args.steps)
    sync_all()
    elapsed = time.perf_counter() - t0
    ks = r.k.stats()
    r.k.set_timing(False)
    if dist is not None:
        import torch
        e = torch.tensor([elapsed], dtype=torch.float64, device=f"cuda:{device}" if args.dist_backend == "nccl" else "cpu")
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())

    rays_per_step, visits, tests, hits = counts
    ms_step = elapsed * 1e3 / args.steps
    value = rays_per_step * args.steps / elapsed / 1e6
    # roofline of KernelEntry on rank 0: algorithmic bytes of one launch (one frame of this
    # rank's tile) / its mean duration
    launches = max(1, ks["launches"])
    kernel_ms = ks["kernel_ms"] / launches
    accum_ms = ks["accum_ms"] / launches
    frames_per_launch = args.frames if (args.launch == "fused" and args.sched == "step") else 1
    # fused launches accumulate on a second stream that overlaps the next render (rt_capi.cpp,
    # RT_ACCUM_OVERLAP): its event span then includes the wait for the render, so it is not a
    # kernel duration -- the rocprofv3 kernel trace under profiles/ carries that
    accum_overlapped = frames_per_launch > 1 and os.environ.get("RT_ACCUM_OVERLAP", "1") != "0"
    local_counts = np.array([st["rays"], st["node_visits"], st["tri_tests"], st["hits"]], np.float64)
    tile_px = r.pixels
    alg_bytes = ((48 * local_counts[1] + 48 * local_counts[2] + 164 * local_counts[3]) / args.frames
                 + 32 * tile_px) * frames_per_launch
    achieved = alg_bytes / (kernel_ms * 1e-3) / 1e9 if kernel_ms > 0 else 0.0
    traffic = None
    valu = None
    tpath = os.path.join(REPO, "profiles", "traffic.json")
    if os.path.exists(tpath):
        try:
            tj = json.load(open(tpath))
            key = (f"{args.scene}_{args.width}x{args.height}_f{args.frames}_b{args.bounces}_{args.math}_n{world}"
                   + ("_fused" if frames_per_launch > 1 else ""))
            if key in tj:
                traffic = tj[key]["hbm_bytes_per_launch"]
                insts = tj[key].get("valu_insts_per_launch")
                if insts and kernel_ms > 0:
                    # VALU issue: one wave64 VALU instruction holds a SIMD-32 for 2 cycles; 4 SIMDs
                    # per CU at the 2.4 GHz clock (MI355X_MICROARCH.md).  The binding resource of
                    # this LDS-resident traversal, next to the HBM roofline the contract asks for.
                    cap = SIMDS * 2.4e9 * kernel_ms * 1e-3 / 2.0
                    valu = {"insts_per_launch": int(insts), "issue_frac": round(insts / cap, 4),
                            "peak_insts_per_s": SIMDS * 2.4e9 / 2.0}
        except (ValueError, KeyError):
            traffic = None

    if args.check_gather and final is not None:
        # rank 0's own bands must have travelled out through RCCL and back into the final image
        a = np.empty((r.H * r.W, 4), np.float32)
        b = np.empty_like(a)
        r.ctx.ReadBuffer(r.out, a)
        torch.cuda.synchronize()
        b[:] = final.cpu().numpy().reshape(b.shape)  # the pipelined flow's final image (a tensor)
        rows = np.concatenate([np.arange(bb * mg.BAND_ROWS, min(r.H, (bb + 1) * mg.BAND_ROWS)) for bb in r.bands])
        a, b = a.reshape(r.H, r.W, 4)[rows], b.reshape(r.H, r.W, 4)[rows]
        if not (a.view(np.uint32) == b.view(np.uint32)).all():
            raise SystemExit("gathered image differs from the rendered bands")
        print(f"check-gather: {rows.size} rows identical", file=sys.stderr)
    if rank != 0:
        if dist is not None:
            dist.destroy_process_group()
        return
    scene_name = "Cornell box" if args.scene == "cornell" else "bunny-class proxy, 69,692 triangles"
    line = {
        "metric": f"Mrays/s ({args.width}x{args.height} {scene_name}, {args.frames} spp, {args.bounces} bounces)",
        "value": round(value, 3),
        "unit": "Mrays/s",
        "n_gpus": world,
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
                   "math": args.math, "schedule": args.sched, "launch": args.launch, "bvh": args.bvh, "parallelism": f"interleaved 8-row bands x{world}" + (
                       (" + gloo gather to rank 0 (host-staged)" if args.dist_backend == "gloo" else
                        " + RCCL gather to rank 0" + ("" if args.no_overlap else ", pipelined with the next step"))
                       if dist is not None else ""),
                   "rays_per_step": int(rays_per_step), "samples_per_step": args.width * args.height * args.frames},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "kernel": "KernelEntry", "kernel_ms": round(kernel_ms, 4),
                     "frames_per_launch": frames_per_launch, "accum_ms_per_launch": None if accum_overlapped else round(accum_ms, 4),
                     "accum_overlapped": accum_overlapped,
                     "alg_bytes_per_launch": int(alg_bytes), "valu": valu},
    }
    if world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(scene, args)
    print(json.dumps(line))
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
