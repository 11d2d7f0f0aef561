"""GPU: frame coalescing (RT_TUNE_PERFRAME_BATCH) -- rtEnqueueKernel calls queued back to back
with consecutive frameCount are launched as fused launches of up to 8 frames, before anything
else touches the context.  The reference's host issues one ExecuteKernel per frame
(CLRaytracer.cpp:35-55); whatever the host does between the calls -- nothing, a read, a camera
move, a new FRAME_SEED, a kernel setting, a buffer write, a release -- every image it can read is
the bits of the uncoalesced per-frame launches."""
import numpy as np
import pytest

from clrt import _native as N
from hip_helpers import DEFAULT_CAMERA, HipRenderer

pytestmark = pytest.mark.gpu

W, H = 288, 160
MOVED = ((0.5, -24.0, 8.0), DEFAULT_CAMERA[1], DEFAULT_CAMERA[2])


def _run(scene, batch, script, math=N.MATH_SHIPPED, hits=False):
    """script: a list of ("frame", f[, camera]) / ("read",) / ("seed", v) / ("tune", name, v) /
    ("write",) steps; returns every read image and the final image (+ hits)."""
    r = HipRenderer(scene, W, H, math=math, hits=hits)
    r.k.set_tuning("perframe_batch", batch)
    assert r.k.get_tuning("perframe_batch") == batch
    reads = []
    seed = 12345
    for step in script:
        if step[0] == "frame":
            cam = step[2] if len(step) > 2 else DEFAULT_CAMERA
            r.k.set_uint(N.FRAME_COUNT, step[1])
            r.k.set_uint(N.FRAME_SEED, seed)
            r.k.set_int(N.LIGHT_BOUNCES, 9)
            r.k.set_int(N.LIGHT_TYPE, 0)
            r.k.set_float(N.SKYBOX_INTENSITY, 1.0)
            r.k.set_float3(N.CAMERA_POS, cam[0])
            r.k.set_float3(N.CAMERA_FRONT, cam[1])
            r.k.set_float3(N.CAMERA_UP, cam[2])
            r.ctx.ExecuteKernel(r.k, r.n)
        elif step[0] == "read":
            reads.append(r.result())
        elif step[0] == "seed":
            seed = step[1]
        elif step[0] == "tune":
            r.k.set_tuning(step[1], step[2])
        elif step[0] == "write":
            img = r.result()
            r.ctx.WriteBuffer(r.out, img[::-1].copy())  # the host replaces the image
    final = r.result()
    h = r.hits() if hits else None
    r.close()
    return reads, final, h


def _check(a, b):
    ra, fa, ha = a
    rb, fb, hb = b
    assert len(ra) == len(rb)
    for x, y in zip(ra + [fa], rb + [fb]):
        assert x.tobytes() == y.tobytes(), f"{(x != y).any(axis=1).sum()} pixels differ"
    if ha is not None:
        assert np.array_equal(ha[0], hb[0]) and ha[1].tobytes() == hb[1].tobytes()


@pytest.mark.parametrize("math", [N.MATH_PINNED, N.MATH_SHIPPED])
def test_queued_frames_coalesce_to_the_same_bits(cornell, math):
    """13 frames queued back to back (one fused launch of 8, then 5), frames starting at 0,
    the last frame's primary hits included"""
    script = [("frame", f) for f in range(0, 13)]
    _check(_run(cornell, 8, script, math, hits=True), _run(cornell, 1, script, math, hits=True))


def test_runs_break_where_the_host_looks_or_changes_something(cornell):
    script = ([("frame", f) for f in range(1, 4)] + [("read",)] +           # a read mid-run
              [("seed", 777), ("frame", 4), ("seed", 778), ("frame", 5)] +  # FRAME_SEED: never read
              [("frame", 6, MOVED), ("frame", 7, MOVED)] +                  # the camera moves
              [("frame", 9, MOVED)] +                                       # a gap in frameCount
              [("tune", "shade_min", 40), ("frame", 10, MOVED)] +           # a kernel setting
              [("write",), ("frame", 11, MOVED), ("frame", 12, MOVED)] +    # the host writes the image
              [("frame", 1), ("frame", 2)])                                 # a new run from frame 1
    _check(_run(cornell, 8, script), _run(cornell, 1, script))


def test_short_batches_and_the_global_scene_path(cornell):
    from clrt import proxy
    script = [("frame", f) for f in range(1, 10)] + [("read",)] + [("frame", f) for f in range(10, 13)]
    for batch in (2, 3):
        _check(_run(cornell, batch, script), _run(cornell, 1, script))
    sc = proxy.bunny_proxy()
    script = [("frame", f) for f in range(1, 7)]
    _check(_run(sc, 8, script), _run(sc, 1, script))


def test_pending_frames_survive_releases(cornell):
    """frames still coalescing when the kernel or the context is released are launched first"""
    r = HipRenderer(cornell, W, H, math=N.MATH_SHIPPED, perframe_batch=None)
    for f in (1, 2, 3):
        r.frame(f)
    r.k.release()  # launches frames 1-3, then releases
    out = np.zeros((r.n, 4), np.float32)
    r.ctx.ReadBuffer(r.out, out, r.n * 16, blocking=True)
    want = _run(cornell, 1, [("frame", f) for f in (1, 2, 3)])[1]
    assert out.tobytes() == want.tobytes()
    for b in r.bufs:
        b.release()
    r.out.release()
    r.ctx.release()


@pytest.mark.parametrize("expose", ["stream", "pointer"])
def test_no_coalescing_once_the_host_can_synchronise_outside_the_library(cornell, expose):
    """A host holding the context's stream or a buffer's device pointer may synchronise with
    hipStreamSynchronize and read the bytes directly: every frame it enqueued must have launched
    (the library default batch of 8 is in force)."""
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipStreamSynchronize.argtypes = [ctypes.c_void_p]
    hip.hipDeviceSynchronize.argtypes = []
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    r = HipRenderer(cornell, W, H, math=N.MATH_SHIPPED, perframe_batch=None)
    assert r.k.get_tuning("perframe_batch") == 8
    s = r.ctx.stream() if expose == "stream" else None
    ptr = r.out.device_pointer()
    for f in (1, 2, 3):
        r.frame(f)
    assert (hip.hipStreamSynchronize(ctypes.c_void_p(s)) if s else hip.hipDeviceSynchronize()) == 0
    got = np.zeros((r.n, 4), np.float32)
    assert hip.hipMemcpy(got.ctypes.data, ctypes.c_void_p(ptr), r.n * 16, 2) == 0  # hipMemcpyDeviceToHost
    want = _run(cornell, 1, [("frame", f) for f in (1, 2, 3)])[1]
    assert got.tobytes() == want.tobytes()
    r.close()


def test_batch_tuning_range(cornell):
    r = HipRenderer(cornell, 64, 64, perframe_batch=None)
    assert r.k.get_tuning("perframe_batch") == 8
    for bad in (0, 9):
        with pytest.raises(Exception):
            r.k.set_tuning("perframe_batch", bad)
    r.close()
