"""The multi-GPU component of the library (rtComm*, csrc/rt_comm.cpp).

CPU: the library's band pack plan equals the Python plan the gloo tests use, for every rank
of many image sizes, and covers every row exactly once.
GPU (one MI355X, so a world of one rank -- the root's own bands still travel the whole RCCL
path: pack on the accumulation stream, a send/receive to itself, unpack): the gathered image
is byte-identical to the rendered one, through ncclCommInitRank and ncclCommInitAll, gathered
into a separate buffer or into the output itself, pipelined over back-to-back steps, after
per-frame launches; and bench.py's own N > 1 flow (--force-dist --check-gather) in a fresh
process.  Worlds of 2..8 ranks run on the one GPU as a loopback world (rtCommInitLoopback: every
rank its own context, the RCCL transfer replaced by device copies, the rest of the gather as is),
at the bench's full 4K 8-spp size; the RCCL transfer between N > 1 GPUs is the driver's 8-GPU
bench.  The band arithmetic is also the CPU part here and tests/test_multigpu_gloo.py.
"""
import json
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


def test_rendezvous_path_is_per_attempt(monkeypatch):
    """A torchrun restart keeps the agent pid and MASTER_PORT; the id file must still change, so
    no rank reads a communicator id a failed attempt left behind."""
    monkeypatch.delenv("RT_COMM_ID_FILE", raising=False)
    monkeypatch.setenv("MASTER_PORT", "29500")
    monkeypatch.setenv("TORCHELASTIC_RUN_ID", "job/1")
    monkeypatch.setenv("TORCHELASTIC_RESTART_COUNT", "0")
    a = mg._rendezvous_path()
    monkeypatch.setenv("TORCHELASTIC_RESTART_COUNT", "1")
    b = mg._rendezvous_path()
    monkeypatch.setenv("TORCHELASTIC_RUN_ID", "job2")
    c = mg._rendezvous_path()
    assert len({a, b, c}) == 3 and "/" not in os.path.basename(a)
    monkeypatch.setenv("RT_COMM_ID_FILE", "/tmp/x.id")
    assert mg._rendezvous_path() == "/tmp/x.id"
    uid = bytes(range(N.COMM_ID_BYTES))
    monkeypatch.setenv("RT_COMM_ID_FILE", "")
    monkeypatch.delenv("RT_COMM_ID_FILE")
    monkeypatch.setenv("TORCHELASTIC_RESTART_COUNT", "7")
    monkeypatch.setenv("MASTER_PORT", str(40000 + os.getpid() % 1000))
    assert mg.file_rendezvous(0, 2, lambda: uid) == uid
    assert mg.file_rendezvous(1, 2, None, timeout=5) == uid
    mg.rendezvous_cleanup()
    assert not os.path.exists(mg._rendezvous_path())


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
@pytest.mark.parametrize("init,into_out,transport",
                         [(i, o, t) for i, o in (("rank", False), ("rank", True), ("all", False))
                          for t in ("copy", "rccl", "copy-ipc")
                          if not (i == "all" and t == "copy-ipc")])  # (IPC links: one process per GPU)
def test_gather_world_of_one(cornell, init, into_out, transport):
    import clrt
    W, H = 640, 360
    ctx = clrt.CLContext(0)
    if init == "rank":
        comm = mg.Comm.init_rank(ctx, 1, mg.Comm.unique_id(), 0)
    else:
        (comm,) = mg.Comm.init_all([ctx])
    assert (comm.rank, comm.nranks) == (0, 1)
    want = {"rccl": N.COMM_TRANSPORT_RCCL, "copy": N.COMM_TRANSPORT_COPY_ENGINES,
            "copy-ipc": N.COMM_TRANSPORT_COPY_ENGINES_IPC}[transport]
    comm.set_transport(want)
    assert comm.transport() == (want, -1)
    bufs, out, k = _setup(ctx, cornell, W, H)
    comm.shard(k)
    dst = None if into_out else ctx.create_buffer(N.MEM_READ_WRITE, W * H * 16)
    images = []
    for step in range(5):  # pipelined: gathers queued behind back-to-back fused renders (slots reused)
        k.set_uint(N.FRAME_COUNT, 1 + 8 * step)
        ctx.ExecuteKernelFrames(k, W * H, 8)
        mg.Comm.gather_bands([comm], [out], W, H, root=0, dst=dst)
        if step == 0:
            images.append(_read(ctx, dst or out, W * H))
            assert comm.transport() == (want, want)
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
@pytest.mark.parametrize("transport,hooks", [("copy", ()), ("copy-ipc", ()), ("copy-ipc", ("acquire",)),
                                             ("copy", ("acquire", "replan")), ("copy-ipc", ("replan",))])
def test_gather_images_read_by_kernels_are_current(cornell, transport, hooks):
    """The copy engines write the root's image behind the GPU caches' back (SDMA, from another
    device's engine between GPUs): a kernel that reads the image after each gather -- here the
    runtime's 2-D blit copy, an L2-cached read of an image small enough to stay in L2 from one
    step to the next -- must see that gather's bytes, never the previous step's lines.  Hooks:
    the root's system-scope acquire, which a root whose image other devices write runs before its
    first read (RT_COMM_OPT_SYSTEM_ACQUIRE forces it here, on one device), and a collective
    re-plan every second gather (RT_COMM_OPT_REPLAN_PERIOD: the flag values start over)."""
    import clrt
    W, H, steps = 256, 144, 6
    ctx = clrt.CLContext(0)
    comm = mg.Comm.init_rank(ctx, 1, mg.Comm.unique_id(), 0)
    comm.set_transport(N.COMM_TRANSPORT_COPY_ENGINES if transport == "copy" else N.COMM_TRANSPORT_COPY_ENGINES_IPC)
    if "acquire" in hooks:
        comm.set_option(N.COMM_OPT_SYSTEM_ACQUIRE, 1)
    if "replan" in hooks:
        comm.set_option(N.COMM_OPT_REPLAN_PERIOD, 2)
    bufs, out, k = _setup(ctx, cornell, W, H)
    comm.shard(k)
    dst = ctx.create_buffer(N.MEM_READ_WRITE, W * H * 16)
    snaps = [ctx.create_buffer(N.MEM_READ_WRITE, W * H * 16) for _ in range(steps)]
    for step in range(steps):
        k.set_uint(N.FRAME_COUNT, 1 + 8 * step)
        ctx.ExecuteKernelFrames(k, W * H, 8)
        mg.Comm.gather_bands([comm], [out], W, H, root=0, dst=dst)
        ctx.CopyRectToDevicePointer(dst, 0, W * 16, W * 16, H, snaps[step].device_pointer(), W * 16)
    ctx.Finish()
    got = [_read(ctx, s, W * H) for s in snaps]
    bufs2, out2, k2 = _setup(ctx, cornell, W, H)
    for step in range(steps):
        k2.set_uint(N.FRAME_COUNT, 1 + 8 * step)
        ctx.ExecuteKernelFrames(k2, W * H, 8)
        assert got[step].tobytes() == _read(ctx, out2, W * H).tobytes(), f"step {step}: stale or torn image"
    if "replan" in hooks:
        assert comm.status()["gathers"] <= 2  # the plan was rebuilt every second gather
    comm.destroy()
    for b in bufs + bufs2 + [out, out2, dst] + snaps:
        b.release()
    k.release()
    k2.release()
    ctx.release()


@pytest.mark.gpu
def test_comm_options_are_checked():
    import clrt
    ctx = clrt.CLContext(0)
    comm = mg.Comm.init_rank(ctx, 1, mg.Comm.unique_id(), 0)
    for bad in (0, -1, 65535):
        with pytest.raises(clrt.RTError):
            comm.set_option(N.COMM_OPT_REPLAN_PERIOD, bad)
    comm.set_option(N.COMM_OPT_REPLAN_PERIOD, 65534)
    with pytest.raises(clrt.RTError):
        comm.set_option(99, 1)
    comm.destroy()
    ctx.release()


@pytest.mark.gpu
def test_rccl_plan_does_not_hold_the_destination(cornell):
    """An RCCL plan unpacks into whatever each gather names: a destination released after its
    gather is not kept by the plan, and the next gather into another buffer needs no re-plan."""
    import clrt
    W, H = 320, 200
    ctx = clrt.CLContext(0)
    comm = mg.Comm.init_rank(ctx, 1, mg.Comm.unique_id(), 0)
    comm.set_transport(N.COMM_TRANSPORT_RCCL)
    bufs, out, k = _setup(ctx, cornell, W, H)
    comm.shard(k)
    d1 = ctx.create_buffer(N.MEM_READ_WRITE, W * H * 16)
    k.set_uint(N.FRAME_COUNT, 1)
    ctx.ExecuteKernelFrames(k, W * H, 8)
    mg.Comm.gather_bands([comm], [out], W, H, root=0, dst=d1)
    assert _read(ctx, d1, W * H).tobytes() == _read(ctx, out, W * H).tobytes()
    d1.release()
    d2 = ctx.create_buffer(N.MEM_READ_WRITE, W * H * 16)
    k.set_uint(N.FRAME_COUNT, 9)
    ctx.ExecuteKernelFrames(k, W * H, 8)
    mg.Comm.gather_bands([comm], [out], W, H, root=0, dst=d2)
    assert _read(ctx, d2, W * H).tobytes() == _read(ctx, out, W * H).tobytes()
    assert comm.status()["gathers"] == 2
    comm.destroy()
    for b in bufs + [out, d2]:
        b.release()
    k.release()
    ctx.release()


@pytest.mark.gpu
def test_gather_forced_link_failure_falls_back_to_rccl(cornell):
    """A world whose copy-engine links fail (the test hook makes this rank report them broken at
    the link step) falls back to RCCL transfers for the plan, says so in its status, and gathers
    the same bytes."""
    import clrt
    W, H = 640, 360
    ctx = clrt.CLContext(0)
    comm = mg.Comm.init_rank(ctx, 1, mg.Comm.unique_id(), 0)
    comm.set_transport(N.COMM_TRANSPORT_COPY_ENGINES_IPC)
    comm.set_option(N.COMM_OPT_FAIL_LINKS, 1)
    bufs, out, k = _setup(ctx, cornell, W, H)
    comm.shard(k)
    dst = ctx.create_buffer(N.MEM_READ_WRITE, W * H * 16)
    for step in range(3):
        k.set_uint(N.FRAME_COUNT, 1 + 8 * step)
        ctx.ExecuteKernelFrames(k, W * H, 8)
        mg.Comm.gather_bands([comm], [out], W, H, root=0, dst=dst)
    ctx.Finish()
    st = comm.status()
    assert comm.transport() == (N.COMM_TRANSPORT_COPY_ENGINES_IPC, N.COMM_TRANSPORT_RCCL)
    assert st["fallback"] and st["fallback_reason"] == "link trial round failed" and st["active"] == "RCCL"
    assert st["gathers"] == 3 and st["last_xfer_ms"] is not None
    assert _read(ctx, dst, W * H).tobytes() == _read(ctx, out, W * H).tobytes()
    # the hook off and a new plan: the copy engines again, no fallback
    comm.set_option(N.COMM_OPT_FAIL_LINKS, 0)
    comm.set_transport(N.COMM_TRANSPORT_COPY_ENGINES_IPC)
    k.set_uint(N.FRAME_COUNT, 25)
    ctx.ExecuteKernelFrames(k, W * H, 8)
    mg.Comm.gather_bands([comm], [out], W, H, root=0, dst=dst)
    ctx.Finish()
    st = comm.status()
    assert not st["fallback"] and st["active"] == "copy engines (IPC links)"
    assert st["bytes_per_gather"] == W * H * 16 and st["copies_per_gather"] == 1
    assert _read(ctx, dst, W * H).tobytes() == _read(ctx, out, W * H).tobytes()
    comm.destroy()
    for b in bufs + [out, dst]:
        b.release()
    k.release()
    ctx.release()


@pytest.mark.gpu
def test_gather_destination_is_part_of_the_plan(cornell):
    """One rank per process (IPC links): the root cannot tell the other ranks about a new
    destination, so it refuses one until the plan is rebuilt; a destination released meanwhile
    stays allocated for the plan (the others' copies may still land in it)."""
    import clrt
    W, H = 320, 200
    ctx = clrt.CLContext(0)
    comm = mg.Comm.init_rank(ctx, 1, mg.Comm.unique_id(), 0)
    comm.set_transport(N.COMM_TRANSPORT_COPY_ENGINES_IPC)
    bufs, out, k = _setup(ctx, cornell, W, H)
    comm.shard(k)
    d1 = ctx.create_buffer(N.MEM_READ_WRITE, W * H * 16)
    d2 = ctx.create_buffer(N.MEM_READ_WRITE, W * H * 16)
    k.set_uint(N.FRAME_COUNT, 1)
    ctx.ExecuteKernelFrames(k, W * H, 8)
    mg.Comm.gather_bands([comm], [out], W, H, root=0, dst=d1)
    with pytest.raises(clrt.RTError) as e:
        mg.Comm.gather_bands([comm], [out], W, H, root=0, dst=d2)
    assert e.value.code == -59
    d1.release()  # pinned by the plan: released when the plan lets go
    comm.set_transport(N.COMM_TRANSPORT_COPY_ENGINES_IPC)  # collective re-plan
    mg.Comm.gather_bands([comm], [out], W, H, root=0, dst=d2)
    assert _read(ctx, d2, W * H).tobytes() == _read(ctx, out, W * H).tobytes()
    comm.destroy()
    for b in bufs + [out, d2]:
        b.release()
    k.release()
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
def test_gather_plan_rebuilt_on_size_and_transport_change(cornell):
    """A new image size (or transport) rebuilds the plan -- flags and sequence numbers start over
    -- between pipelined gathers of the old one; every gathered image equals its render."""
    import clrt
    ctx = clrt.CLContext(0)
    comm = mg.Comm.init_rank(ctx, 1, mg.Comm.unique_id(), 0)
    for (W, H), transport in (((256, 144), 0), ((200, 120), 0), ((200, 120), 1), ((256, 144), 0)):
        comm.set_transport(transport)
        bufs, out, k = _setup(ctx, cornell, W, H)
        comm.shard(k)
        dst = ctx.create_buffer(N.MEM_READ_WRITE, W * H * 16)
        for step in range(4):
            k.set_uint(N.FRAME_COUNT, 1 + 8 * step)
            ctx.ExecuteKernelFrames(k, W * H, 8)
            mg.Comm.gather_bands([comm], [out], W, H, root=0, dst=dst)
        assert _read(ctx, dst, W * H).tobytes() == _read(ctx, out, W * H).tobytes()
        assert comm.transport() == (transport, transport)
        for b in bufs + [out, dst]:
            b.release()
        k.release()
    comm.destroy()
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
@pytest.mark.parametrize("transport", ["copy", "rccl", "copy-ipc"])
def test_bench_rccl_flow_world_of_one(tmp_path, transport):
    """bench.py's N > 1 flow (file rendezvous, RCCL communicator, sharded fused renders, the
    pipelined gather every step into the root's image buffer, max-over-ranks timing) at
    WORLD_SIZE 1, on either transport; --check-gather makes rank 0 re-render the frame unsharded
    and compare the gathered image byte for byte."""
    env = dict(os.environ, RT_COMM_ID_FILE=str(tmp_path / "comm.id"))
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--force-dist", "--check-gather",
                        "--transport", transport,
                        "--width", "1280", "--height", "720", "--steps", "3", "--warmup", "1", "--no-cpu-baseline"],
                       env=env, capture_output=True, text=True, timeout=110)
    assert p.returncode == 0, p.stderr[-2000:]
    assert "byte-identical" in p.stdout
    line = json.loads(p.stdout.strip().splitlines()[-1])
    want = {"copy": "copy engines", "rccl": "RCCL", "copy-ipc": "copy engines (IPC links)"}[transport]
    assert line["n_gpus"] == 1 and line["comm"]["nranks"] == 1
    assert line["comm"]["effective"] == want and not line["comm"]["fallback"]
    assert want in line["config"]["parallelism"]
    (r0,) = line["comm"]["per_rank"]
    assert r0["render_ms"] > 0 and r0["last_gather_ms"] is not None


@pytest.mark.gpu
def test_bench_line_reports_a_fallback(tmp_path):
    """The driver's N > 1 line says which transport actually ran: a world whose copy-engine links
    fail (the test hook) runs -- and is labelled -- RCCL, with the reason, byte-identical."""
    env = dict(os.environ, RT_COMM_ID_FILE=str(tmp_path / "comm.id"))
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--force-dist", "--check-gather",
                        "--transport", "copy-ipc", "--fail-links",
                        "--width", "1280", "--height", "720", "--steps", "3", "--warmup", "1", "--no-cpu-baseline"],
                       env=env, capture_output=True, text=True, timeout=110)
    assert p.returncode == 0, p.stderr[-2000:]
    line = json.loads(p.stdout.strip().splitlines()[-1])
    assert line["comm"]["fallback"] and line["comm"]["effective"] == "RCCL"
    assert line["comm"]["per_rank"][0]["fallback"] == "link trial round failed"
    assert "over RCCL" in line["config"]["parallelism"] and "byte-identical" in line["check_gather"]


# ---- N > 1 on one GPU: the loopback world (rtCommInitLoopback) ----------------------------------
# The same sharding, pack on the accumulation stream, two-slot pipelining, per-rank receive slots
# parts[s] + q*stage_bytes, per-rank unpack plans (with the short last band) and the copy-engine
# transport's flag protocol (arrival flags in the root's memory, slot-free flags in each rank's)
# as a multi-GPU world -- only the ranks' links are addresses in this process instead of IPC
# mappings.  Every rank is its own context on the one GPU of the test box.  (Copies between GPUs
# over xGMI need N GPUs: the driver's 8-GPU bench.)
def _scene(cornell, name):
    if name == "cornell":
        return cornell
    import clrt.proxy as P
    return P.bunny_proxy()


def _unsharded(ctx, scene, W, H, steps):
    bufs, out, k = _setup(ctx, scene, W, H)
    for step in range(steps):
        k.set_uint(N.FRAME_COUNT, 1 + 8 * step)
        ctx.ExecuteKernelFrames(k, W * H, 8)
    img = _read(ctx, out, W * H)
    for b in bufs + [out]:
        b.release()
    k.release()
    return img


def _loopback_gather(scene, n, W, H, steps, root=0, into_out=False):
    """n ranks, each its own context: `steps` fused 8-frame renders of its bands (frames 1+8s ..
    8+8s, accumulating), each followed at once by the pipelined gather to `root`, as bench.py's
    timed loop queues them.  Returns (gathered image, every rank's own output buffer)."""
    import clrt
    ctxs = [clrt.CLContext(0) for _ in range(n)]
    comms = mg.Comm.init_loopback(ctxs)
    assert [(c.rank, c.nranks) for c in comms] == [(q, n) for q in range(n)]
    setups = [_setup(ctx, scene, W, H) for ctx in ctxs]
    for c, (_, _, k) in zip(comms, setups):
        c.shard(k)
    outs = [s[1] for s in setups]
    dst = None if into_out else ctxs[root].create_buffer(N.MEM_READ_WRITE, W * H * 16)
    for step in range(steps):
        for ctx, (_, _, k) in zip(ctxs, setups):
            k.set_uint(N.FRAME_COUNT, 1 + 8 * step)
            ctx.ExecuteKernelFrames(k, W * H, 8)
        mg.Comm.gather_bands(comms, outs, W, H, root=root, dst=dst)
    for ctx in ctxs:
        ctx.Finish()
    gathered = _read(ctxs[root], dst or outs[root], W * H)
    shares = [_read(ctx, o, W * H) for ctx, o in zip(ctxs, outs)]
    v = mg.Comm.allreduce(comms, [[float(q), 1.0] for q in range(n)], N.COMM_SUM)
    assert (v == [[n * (n - 1) / 2, float(n)]] * n).all()
    mg.Comm.barrier(comms)
    for c in comms:
        c.destroy()
    for (bufs, out, k) in setups:
        for b in bufs + [out]:
            b.release()
        k.release()
    if dst:
        dst.release()
    for ctx in ctxs:
        ctx.release()
    return gathered, shares


@pytest.mark.gpu
@pytest.mark.parametrize("n", [2, 4, 8])
def test_loopback_gather_4k_8spp_pipelined_equals_unsharded(cornell, n):
    """The 4K 8-spp bench workload on n ranks: three pipelined steps, the gathered image
    byte-identical to the unsharded render (itself pinned to the reference kernel in
    test_benched_path.py), and every rank's buffer holding exactly its bands."""
    import clrt
    W, H = 3840, 2160
    ctx = clrt.CLContext(0)
    full = _unsharded(ctx, cornell, W, H, 3)
    ctx.release()
    gathered, shares = _loopback_gather(cornell, n, W, H, 3)
    assert gathered.tobytes() == full.tobytes()
    rows = np.arange(H)
    f = full.reshape(H, W, 4)
    for q, s in enumerate(shares):
        s = s.reshape(H, W, 4)
        mine = (rows // 8) % n == q
        assert s[mine].tobytes() == f[mine].tobytes(), f"rank {q}/{n}: band rows differ"
        assert not s[~mine].any(), f"rank {q}/{n} wrote rows outside its bands"


@pytest.mark.gpu
def test_loopback_gather_bunny_n8(cornell):
    """Config 5's shape (the 70k-triangle proxy, octant walk over HBM/L2) at N = 8."""
    import clrt
    sc = _scene(cornell, "bunny")
    W, H = 3840, 2160
    ctx = clrt.CLContext(0)
    full = _unsharded(ctx, sc, W, H, 2)
    ctx.release()
    gathered, _ = _loopback_gather(sc, 8, W, H, 2)
    assert gathered.tobytes() == full.tobytes()


@pytest.mark.gpu
@pytest.mark.parametrize("W,H,n,root,into_out", [(1277, 731, 3, 2, False), (640, 37, 8, 5, True),
                                                  (333, 9, 2, 1, True), (64, 8, 4, 0, False)])
def test_loopback_gather_ragged(cornell, W, H, n, root, into_out):
    """Odd sizes (short last band, ranks with no band at all), a root other than 0, gathering
    into the root's own output buffer."""
    import clrt
    ctx = clrt.CLContext(0)
    full = _unsharded(ctx, cornell, W, H, 3)
    ctx.release()
    gathered, _ = _loopback_gather(cornell, n, W, H, 3, root=root, into_out=into_out)
    assert gathered.tobytes() == full.tobytes()


@pytest.mark.gpu
def test_loopback_calls_must_name_the_whole_world(cornell):
    import clrt
    ctxs = [clrt.CLContext(0) for _ in range(3)]
    comms = mg.Comm.init_loopback(ctxs)
    setups = [_setup(ctx, cornell, 64, 64) for ctx in ctxs]
    with pytest.raises(clrt.RTError):
        mg.Comm.gather_bands(comms[:2], [s[1] for s in setups[:2]], 64, 64)
    with pytest.raises(clrt.RTError):
        mg.Comm.gather_bands([comms[0], comms[0], comms[1]], [s[1] for s in setups], 64, 64)
    with pytest.raises(clrt.RTError):
        mg.Comm.allreduce(comms[1:], [[1.0], [2.0]])
    # a comm-sharded kernel renders whole frames: work ranges are refused both ways
    k = setups[0][2]
    comms[0].shard(k)
    with pytest.raises(clrt.RTError) as e:
        k.set_work_range(0, 64 * 8)
    assert e.value.code == -59  # CL_INVALID_OPERATION
    k2 = setups[1][2]
    k2.set_work_range(64, 64 * 20)
    with pytest.raises(clrt.RTError) as e:
        comms[1].shard(k2)
    assert e.value.code == -59
    for c in comms:
        c.destroy()
    for (bufs, out, kk) in setups:
        for b in bufs + [out]:
            b.release()
        kk.release()
    for ctx in ctxs:
        ctx.release()
