"""GPU: rtEnqueueKernelFrames -- F frames as one step launch over (frame, pixel) work items plus
a per-pixel accumulation launch -- must leave exactly the bits of F per-frame launches
(the reference's RenderFrame loop, CLRaytracer.cpp:35-47): output buffer, last frame's primary
hits and the §8(d) counters, in every math mode, on the LDS and global scene paths, for band
interleaves (multi-GPU ranks), work ranges and frame sequences starting at 0 or mid-way."""
import numpy as np
import pytest

from clrt import _native as N
from hip_helpers import HipRenderer, rgb

pytestmark = pytest.mark.gpu


def _render(scene, W, H, first, n, fused, math=N.MATH_SHIPPED, bounces=9, interleave=None,
            work_range=None, force_global=False, sched=N.SCHED_STEP, pre=None, tuning=None):
    r = HipRenderer(scene, W, H, math=math, hits=True, stats=True, force_global=force_global, sched=sched)
    for name, value in (tuning or {}).items():
        r.k.set_tuning(name, value)
    kw = dict(light_bounces=bounces, interleave=interleave, work_range=work_range)
    if pre is not None:  # earlier frames already in the buffer
        for f in pre:
            r.frame(f, **kw)
    r.k.reset_stats()
    if fused:
        r.frame(first, n_frames=n, **kw)
    else:
        for f in range(first, first + n):
            r.frame(f, **kw)
    out = (r.result(), r.hits(), r.k.stats())
    r.close()
    return out


def _same(a, b):
    assert a[0].tobytes() == b[0].tobytes(), f"{(a[0] != b[0]).any(axis=1).sum()} pixels differ"
    assert np.array_equal(a[1][0], b[1][0]) and a[1][1].tobytes() == b[1][1].tobytes()
    for key in ("rays", "node_visits", "tri_tests", "hits"):
        assert a[2][key] == b[2][key], key


@pytest.mark.parametrize("math", [N.MATH_PINNED, N.MATH_DEVICELIB, N.MATH_SHIPPED])
def test_fused_equals_per_frame(cornell, math):
    W, H = 320, 180
    _same(_render(cornell, W, H, 1, 8, True, math), _render(cornell, W, H, 1, 8, False, math))


def test_fused_pinned_equals_oracle(cornell, oracle_mod):
    W, H = 192, 108
    got, (ids, t), _ = _render(cornell, W, H, 1, 4, True, N.MATH_PINNED, bounces=5)
    res = np.zeros((W * H, 4), np.float32)
    for f in range(1, 5):
        res, wids, wt, _ = oracle_mod.render(cornell, W, H, frame_count=f, light_bounces=5, result=res,
                                             want_hits=True, threads=16)
    assert rgb(got).tobytes() == rgb(res).tobytes()
    assert np.array_equal(ids, wids) and t.tobytes() == wt.tobytes()


@pytest.mark.parametrize("first,n,pre", [(0, 3, None), (3, 5, (1, 2)), (1, 2, None), (1, 11, None)])
def test_fused_frame_sequences(cornell, first, n, pre):
    W, H = 200, 120
    _same(_render(cornell, W, H, first, n, True, pre=pre), _render(cornell, W, H, first, n, False, pre=pre))


@pytest.mark.parametrize("period,phase", [(2, 1), (8, 0), (8, 5)])
def test_fused_band_interleave(cornell, period, phase):
    W, H = 256, 200
    _same(_render(cornell, W, H, 1, 6, True, interleave=(period, phase)),
          _render(cornell, W, H, 1, 6, False, interleave=(period, phase)))


def test_fused_work_range_and_global_path(cornell):
    W, H = 240, 136
    n = W * H
    for wr, fg in (((n // 5, n - 77), False), ((0, n), True)):
        _same(_render(cornell, W, H, 1, 5, True, work_range=wr, force_global=fg),
              _render(cornell, W, H, 1, 5, False, work_range=wr, force_global=fg))


def test_fused_bunny_proxy():
    from clrt import proxy
    sc = proxy.bunny_proxy()
    W, H = 320, 180
    _same(_render(sc, W, H, 1, 4, True), _render(sc, W, H, 1, 4, False))


def test_fused_other_schedules_launch_per_frame(cornell):
    W, H = 160, 96
    _same(_render(cornell, W, H, 1, 3, True, sched=N.SCHED_TILES), _render(cornell, W, H, 1, 3, False))


@pytest.mark.parametrize("force_global", [False, True])
def test_fused_sky_shortcut_chain(cornell, force_global):
    """Repeated fused calls (the sky key chains from the previous call's result), a skybox change,
    a math-mode switch and a restart at frame 1 over a non-sky history: every call's output equals
    the per-frame launches (16:9 view: about half of the pixels see only sky).  force_global: the
    octant walk over HBM/L2, whose radiance sets carry no flags -- the accumulation reads a pixel's
    all-sky frames back from the radiance itself."""
    W, H = 320, 180
    seq = [(1, 4, 1.0, N.MATH_SHIPPED), (5, 4, 1.0, N.MATH_SHIPPED), (1, 8, 1.0, N.MATH_SHIPPED),
           (1, 3, 0.6, N.MATH_SHIPPED), (4, 2, 0.6, N.MATH_DEVICELIB), (0, 2, 2.0, N.MATH_PINNED),
           (1, 2, 2.0, N.MATH_PINNED)]
    outs = []
    for fused in (True, False):
        r = HipRenderer(cornell, W, H, math=N.MATH_SHIPPED, hits=True, force_global=force_global)
        if force_global:
            r.k.set_tuning("global_oct", 1)
        got = []
        for first, n, sky, math in seq:
            r.k.set_math_mode(math)
            if fused:
                r.frame(first, light_bounces=9, skybox=sky, n_frames=n)
            else:
                for f in range(first, first + n):
                    r.frame(f, light_bounces=9, skybox=sky)
            got.append(r.result())
        ids, _ = r.hits()
        r.close()
        outs.append(got)
    assert (ids < 0).mean() > 0.3
    for a, b in zip(*outs):
        assert a.tobytes() == b.tobytes()


def test_overlapped_accumulation_stays_in_order(cornell):
    """The accumulation of a fused launch runs on a second stream beside the next render
    (rt_capi.cpp qs()); mixing fused launches, per-frame launches, many back-to-back fused
    launches (both radiance sets in flight) and a host write of the output between them must
    still give the bits of one in-order queue of per-frame launches."""
    W, H = 224, 128
    a = HipRenderer(cornell, W, H, math=N.MATH_SHIPPED)
    b = HipRenderer(cornell, W, H, math=N.MATH_SHIPPED)
    for r, fused in ((a, True), (b, False)):
        def run(first, n):
            if fused:
                r.frame(first, n_frames=n, light_bounces=9)
            else:
                for f in range(first, first + n):
                    r.frame(f, light_bounces=9)
        run(1, 8)
        run(9, 1)
        run(10, 3)
        run(13, 4)
        run(17, 2)
        mid = r.result()  # read between launches: joins the pending accumulation
        run(19, 5)
        r.ctx.WriteBuffer(r.out, mid)  # host overwrite: later accumulation must start from it
        run(24, 8)
        run(32, 8)
        r.ctx.Finish()
    ga, gb = a.result(), b.result()
    a.close()
    b.close()
    assert ga.tobytes() == gb.tobytes(), f"{(ga != gb).any(axis=1).sum()} pixels differ"


@pytest.mark.parametrize("scene,n", [("cornell", 8), ("bunny", 8), ("cornell", 4), ("cornell", 2), ("cornell", 6),
                                     ("cornell_lds", 8), ("cornell_g64", 4)])  # (cornell_lds: the LDS walk ignores the order)
def test_fused_pixel_major_order(cornell, scene, n):
    """Pixel-major work order (tile_major 2, the default for large launches on scenes in HBM/L2): with F =
    2, 4 or 8 fused frames a work unit is 64 / F pixels of a tile x the F frames, a pixel's frames side by
    side in a wave; other F fall back to tile-major -- same bits as per-frame launches, with band
    interleaves."""
    from clrt import proxy
    sc = proxy.bunny_proxy() if scene == "bunny" else cornell
    W, H = 248, 136
    kw = {"cornell": dict(force_global=True, interleave=(2, 1)), "bunny": {}, "cornell_lds": dict(interleave=(2, 1)),
          "cornell_g64": dict(force_global=True)}[scene]
    tune = {"tile_major": 2, **({"global_oct": 0} if scene == "cornell_g64" else {})}  # (g64: the 64-B global records)
    _same(_render(sc, W, H, 2, n, True, tuning=tune, **kw), _render(sc, W, H, 2, n, False, **kw))


@pytest.mark.parametrize("force_global", [False, True])
def test_fused_tile_major_order(cornell, force_global):
    """Tile-major work order (tile_major 1; chosen automatically for large launches on the
    HBM/L2 scene path): the frames of a tile back to back -- same bits as per-frame launches."""
    W, H = 248, 136
    _same(_render(cornell, W, H, 2, 7, True, force_global=force_global, interleave=(2, 1),
                  tuning={"tile_major": 1}),
          _render(cornell, W, H, 2, 7, False, force_global=force_global, interleave=(2, 1)))


def test_readback_on_accum_stream(cornell):
    """rtContextSetReadbackOnAccumStream: a rect copy of the output queued after a fused launch
    runs right after that launch's accumulation on the accumulation stream, so it holds that
    step's image even though the next fused launch is queued before anything waits for it."""
    W, H = 224, 128
    r = HipRenderer(cornell, W, H, math=N.MATH_SHIPPED)
    r.ctx.set_readback_on_accum_stream(True)
    dst = r.ctx.create_buffer(N.MEM_READ_WRITE, W * H * 16)
    r.frame(1, n_frames=8, light_bounces=9)
    r.ctx.CopyRectToDevicePointer(r.out, 0, W * 16, W * 16, H, dst.device_pointer(), W * 16)
    r.frame(9, n_frames=8, light_bounces=9)
    step1 = np.zeros((W * H, 4), np.float32)
    r.ctx.ReadBuffer(dst, step1, blocking=True)  # ordered after the copy (rtEnqueueReadBuffer joins)
    step2 = r.result()
    dst.release()
    r.close()
    ref = HipRenderer(cornell, W, H, math=N.MATH_SHIPPED)
    ref.frame(1, n_frames=8, light_bounces=9)
    want1 = ref.result()
    ref.frame(9, n_frames=8, light_bounces=9)
    want2 = ref.result()
    ref.close()
    assert step1.tobytes() == want1.tobytes()
    assert step2.tobytes() == want2.tobytes()


@pytest.mark.parametrize("frames", [1, 9])
def test_readback_on_accum_stream_after_per_frame_launches(cornell, frames):
    """A rect copy on the accumulation stream after per-frame launches (frames = 1) or a fused
    launch with a 1-frame remainder (9 = 8 fused + 1 per-frame): the copy waits for the main
    stream's tail, so it holds the finished image, not a half-written one."""
    W, H = 256, 144
    r = HipRenderer(cornell, W, H, math=N.MATH_SHIPPED)
    r.ctx.set_readback_on_accum_stream(True)
    dst = r.ctx.create_buffer(N.MEM_READ_WRITE, W * H * 16)
    if frames == 1:
        for f in (1, 2, 3):
            r.frame(f, light_bounces=9)
    else:
        r.frame(1, n_frames=frames, light_bounces=9)
    r.ctx.CopyRectToDevicePointer(r.out, 0, W * 16, W * 16, H, dst.device_pointer(), W * 16)
    got = np.zeros((W * H, 4), np.float32)
    r.ctx.ReadBuffer(dst, got, blocking=True)
    want = r.result()
    dst.release()
    r.close()
    assert got.tobytes() == want.tobytes()


@pytest.mark.parametrize("math", [N.MATH_PINNED, N.MATH_DEVICELIB, N.MATH_SHIPPED])
@pytest.mark.parametrize("fused", [True, False])
@pytest.mark.parametrize("goct", [0, 1])
def test_global_scene_walks(cornell, math, fused, goct):
    """Scenes not in LDS: the octant-resolved records read from HBM/L2 (RT_TUNE_GLOBAL_OCT 1, the
    default) or the 64-B global node records with the top of the tree in LDS (0) -- the same
    visits in the same order as the LDS walk: same bits."""
    W, H = 256, 144
    _same(_render(cornell, W, H, 1, 5, fused, math, force_global=True, tuning={"global_oct": goct}),
          _render(cornell, W, H, 1, 5, False, math))


@pytest.mark.parametrize("case", ["whole", "bands", "work_range"])
def test_octant_walk_fused_ragged(cornell, case):
    """Fused octant walks over HBM/L2 (every path stores its radiance, no flags) on ragged edge tiles
    (250 x 139), band interleaves and work ranges that start and end inside a tile -- the bits of
    per-frame launches."""
    W, H = 250, 139
    kw = {"whole": {}, "bands": {"interleave": (3, 2)}, "work_range": {"work_range": (1234, W * H - 4321)}}[case]
    _same(_render(cornell, W, H, 1, 6, True, force_global=True, tuning={"global_oct": 1}, **kw),
          _render(cornell, W, H, 1, 6, False, **kw))


@pytest.mark.parametrize("sched", [N.SCHED_STEP, N.SCHED_WAVEFRONT])
def test_global_scene_walks_bunny_proxy(sched):
    from clrt import proxy
    sc = proxy.bunny_proxy()
    W, H = 320, 180
    want = _render(sc, W, H, 1, 4, False, tuning={"global_oct": 0})
    for goct in (0, 1):
        _same(_render(sc, W, H, 1, 4, True, sched=sched, tuning={"global_oct": goct}), want)


@pytest.mark.parametrize("math", [N.MATH_PINNED, N.MATH_SHIPPED])
@pytest.mark.parametrize("first,n,pre", [(0, 3, None), (3, 5, (1, 2)), (1, 9, None)])
def test_perframe_defer(cornell, math, first, n, pre):
    """rtEnqueueKernel with RT_TUNE_PERFRAME_DEFER: the frame renders into a radiance slot and a
    second launch accumulates it (as a fused launch of one frame), so consecutive frames' renders
    may overlap -- the same bits as accumulating inside the render."""
    W, H = 256, 144
    _same(_render(cornell, W, H, first, n, False, math, pre=pre, tuning={"perframe_defer": 1}),
          _render(cornell, W, H, first, n, False, math, pre=pre))


def test_perframe_defer_global_path_and_bands(cornell):
    W, H = 240, 136
    for kw in ({"force_global": True}, {"interleave": (3, 1)}, {"work_range": (500, W * H - 33)}):
        _same(_render(cornell, W, H, 1, 4, False, tuning={"perframe_defer": 1}, **kw),
              _render(cornell, W, H, 1, 4, False, **kw))


def test_perframe_defer_stays_in_order(cornell):
    """deferred per-frame launches mixed with fused launches, a read between them and a host
    overwrite of the output: the bits of one in-order queue of per-frame launches"""
    W, H = 224, 128
    outs = []
    for defer in (1, 2, 0):
        r = HipRenderer(cornell, W, H, math=N.MATH_SHIPPED)
        r.k.set_tuning("perframe_defer", defer)
        r.k.set_tuning("perframe_defer_min", 0)  # (2: defer whenever the previous frame still runs)
        for f in range(1, 4):
            r.frame(f, light_bounces=9)
        r.frame(4, light_bounces=9, n_frames=3)
        mid = r.result()
        for f in range(7, 10):
            r.frame(f, light_bounces=9)
        r.ctx.WriteBuffer(r.out, mid)
        for f in range(10, 13):
            r.frame(f, light_bounces=9)
        outs.append((mid, r.result()))
        r.close()
    for o in outs[:2]:
        assert o[0].tobytes() == outs[2][0].tobytes()
        assert o[1].tobytes() == outs[2][1].tobytes()


@pytest.mark.parametrize("math", [N.MATH_PINNED, N.MATH_SHIPPED])
def test_perframe_defer_auto_queued(cornell, math):
    """PERFRAME_DEFER 2 (the default): frames queued back to back defer while the previous render
    still runs, frames after a host wait do not -- whatever the mix, the bits of accumulating in
    the render"""
    W, H = 320, 180
    want = _render(cornell, W, H, 1, 12, False, math, tuning={"perframe_defer": 0})
    r = HipRenderer(cornell, W, H, math=math)
    r.k.set_tuning("perframe_defer_min", 0)
    assert r.k.get_tuning("perframe_defer") == 2
    for f in range(1, 13):
        r.frame(f, light_bounces=9)
        if f in (4, 9):
            r.ctx.Finish()
    got = r.result()
    r.close()
    assert got.tobytes() == want[0].tobytes(), f"{(got != want[0]).any(axis=1).sum()} pixels differ"
