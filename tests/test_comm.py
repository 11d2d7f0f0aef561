"""The multi-GPU component of the library (rtComm*, csrc/rt_comm.cpp).

CPU: the library's band pack plan equals the Python plan the gloo tests use, for every rank
of many image sizes, and covers every row exactly once.
GPU (one MI355X, so a world of one rank -- the root's own bands still travel the whole RCCL
path: pack on the accumulation stream, a send/receive to itself, unpack): the gathered image
is byte-identical to the rendered one, through ncclCommInitRank and ncclCommInitAll, gathered
into a separate buffer or into the output itself, pipelined over back-to-back steps, after
per-frame launches; and bench.py's own N > 1 flow (--force-dist --check-gather) in a fresh
process.  Worlds of 2..8 ranks need more GPUs than the test box has: the driver's 8-GPU bench
runs them; the band arithmetic for them is the CPU part here and tests/test_multigpu_gloo.py.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

from clrt import _native as N
from clrt import multigpu as mg

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("w,h,n", [(3840, 2160, 8), (3840, 2160, 2), (3840, 2160, 4), (1920, 1080, 3),
                                   (37, 45, 2), (5, 7, 4), (16, 64, 8), (3, 5, 9), (640, 8, 1)])
def test_native_plan_equals_python_plan(w, h, n):
    hit = np.zeros(h, np.int32)
    row_bytes = w * mg.PIXEL_BYTES
    for rank in range(n):
        plan, sb = mg.native_pack_plan(w, h, n, rank)
        assert plan == mg.pack_plan(w, h, n, rank)
        assert sb == mg.staging_bytes(w, h, n)
        for r in plan:
            assert r.stage_offset + r.rows * r.width <= sb
            for i in range(r.rows):
                start = (r.img_offset + i * r.img_pitch) // row_bytes
                hit[start:start + r.width // row_bytes] += 1
    assert (hit == 1).all()


def test_native_plan_rejects_bad_arguments():
    import clrt
    for args in [(0, 8, 1, 0), (8, 0, 1, 0), (8, 8, 0, 0), (8, 8, 2, 2)]:
        with pytest.raises(clrt.RTError):
            mg.native_pack_plan(*args)


# ---- GPU -----------------------------------------------------------------------------------
def _setup(ctx, scene, W, H):
    import clrt
    flags = N.MEM_READ_ONLY | N.MEM_COPY_HOST_PTR
    bufs = [ctx.create_buffer(flags, a.nbytes, a) for a in (scene.triangles, scene.nodes, scene.materials)]
    out = ctx.create_buffer(N.MEM_READ_WRITE, W * H * 16)
    k = clrt.CLKernel(ctx)
    for slot, b in zip((N.BUFFER_OUT, N.BUFFER_SCENE, N.BUFFER_NODE, N.BUFFER_MATERIAL), [out] + bufs):
        k.set_buffer(slot, b)
    k.set_int(N.WIDTH, W)
    k.set_int(N.HEIGHT, H)
    k.set_uint(N.FRAME_SEED, 0)
    k.set_int(N.LIGHT_BOUNCES, 9)
    k.set_int(N.LIGHT_TYPE, 0)
    k.set_float(N.SKYBOX_INTENSITY, 1.0)
    k.set_float3(N.CAMERA_POS, (0.0, -25.0, 8.5))
    k.set_float3(N.CAMERA_FRONT, (0.0, 1.0, 0.0))
    k.set_float3(N.CAMERA_UP, (0.0, 0.0, 1.0))
    return bufs, out, k


def _read(ctx, buf, n):
    a = np.zeros((n, 4), np.float32)
    ctx.ReadBuffer(buf, a, blocking=True)
    return a


@pytest.mark.gpu
@pytest.mark.parametrize("init,into_out", [("rank", False), ("rank", True), ("all", False)])
def test_gather_world_of_one(cornell, init, into_out):
    import clrt
    W, H = 640, 360
    ctx = clrt.CLContext(0)
    if init == "rank":
        comm = mg.Comm.init_rank(ctx, 1, mg.Comm.unique_id(), 0)
    else:
        (comm,) = mg.Comm.init_all([ctx])
    assert (comm.rank, comm.nranks) == (0, 1)
    bufs, out, k = _setup(ctx, cornell, W, H)
    comm.shard(k)
    dst = None if into_out else ctx.create_buffer(N.MEM_READ_WRITE, W * H * 16)
    images = []
    for step in range(3):  # pipelined: gathers queued behind back-to-back fused renders
        k.set_uint(N.FRAME_COUNT, 1 + 8 * step)
        ctx.ExecuteKernelFrames(k, W * H, 8)
        mg.Comm.gather_bands([comm], [out], W, H, root=0, dst=dst)
        if step == 0:
            images.append(_read(ctx, dst or out, W * H))
    ctx.Finish()
    gathered = _read(ctx, dst or out, W * H)
    rendered = _read(ctx, out, W * H)
    assert gathered.tobytes() == rendered.tobytes()
    # the same frames without any gather
    bufs2, out2, k2 = _setup(ctx, cornell, W, H)
    k2.set_uint(N.FRAME_COUNT, 1)
    ctx.ExecuteKernelFrames(k2, W * H, 8)
    assert images[0].tobytes() == _read(ctx, out2, W * H).tobytes()
    comm.destroy()
    for b in bufs + bufs2 + [out, out2] + ([dst] if dst else []):
        b.release()
    k.release()
    k2.release()
    ctx.release()


@pytest.mark.gpu
def test_gather_after_per_frame_launches(cornell):
    """Per-frame launches write the output on the main stream; the gather's pack waits for them."""
    import clrt
    W, H = 512, 288
    ctx = clrt.CLContext(0)
    comm = mg.Comm.init_rank(ctx, 1, mg.Comm.unique_id(), 0)
    bufs, out, k = _setup(ctx, cornell, W, H)
    dst = ctx.create_buffer(N.MEM_READ_WRITE, W * H * 16)
    for f in (1, 2, 3):
        k.set_uint(N.FRAME_COUNT, f)
        ctx.ExecuteKernel(k, W * H)
    mg.Comm.gather_bands([comm], [out], W, H, root=0, dst=dst)
    assert _read(ctx, dst, W * H).tobytes() == _read(ctx, out, W * H).tobytes()
    comm.destroy()
    for b in bufs + [out, dst]:
        b.release()
    k.release()
    ctx.release()


@pytest.mark.gpu
def test_allreduce_and_barrier_world_of_one():
    import clrt
    ctx = clrt.CLContext(0)
    comm = mg.Comm.init_rank(ctx, 1, mg.Comm.unique_id(), 0)
    v = mg.Comm.allreduce([comm], [1.5, -2.0, 7.25], N.COMM_MAX)
    assert v.tolist() == [[1.5, -2.0, 7.25]]
    mg.Comm.barrier([comm])
    comm.destroy()
    ctx.release()


@pytest.mark.gpu
def test_bench_rccl_flow_world_of_one(tmp_path):
    """bench.py's N > 1 flow (file rendezvous, RCCL communicator, sharded fused renders, the
    pipelined gather every step, max-over-ranks timing) at WORLD_SIZE 1; --check-gather makes
    rank 0 re-render the frame unsharded and compare the gathered image byte for byte."""
    env = dict(os.environ, RT_COMM_ID_FILE=str(tmp_path / "comm.id"))
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--force-dist", "--check-gather",
                        "--width", "1280", "--height", "720", "--steps", "3", "--warmup", "1", "--no-cpu-baseline"],
                       env=env, capture_output=True, text=True, timeout=110)
    assert p.returncode == 0, p.stderr[-2000:]
    assert "byte-identical" in p.stdout
