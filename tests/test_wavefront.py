"""GPU: the wavefront schedule (RT_SCHED_WAVEFRONT) -- per bounce an extend launch
(BVH traversal from an HBM ray queue) and a shade launch (continuations compacted into the next
queue), radiance into per-frame slots and the fused accumulation -- must leave exactly the bits of
the reference's per-frame loop (CLRaytracer.cpp:35-47 over kernel_bvh.cl:415-456) as the step
schedule renders it: output buffer, the last frame's primary hits and the 8(d) counters, in every
math mode, on the LDS and global scene paths, for band interleaves, work ranges, odd sizes, frame
sequences, bounce counts and every queue/refill tuning."""
import numpy as np
import pytest

from clrt import _native as N
from hip_helpers import HipRenderer, rgb

pytestmark = pytest.mark.gpu


def _render(scene, W, H, first, n, sched, fused=True, math=N.MATH_SHIPPED, bounces=9, interleave=None,
            work_range=None, force_global=False, pre=None, tuning=None, skybox=1.0):
    r = HipRenderer(scene, W, H, math=math, hits=True, stats=True, force_global=force_global, sched=sched)
    for name, value in (tuning or {}).items():
        r.k.set_tuning(name, value)
    kw = dict(light_bounces=bounces, interleave=interleave, work_range=work_range, skybox=skybox)
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


def _step(scene, W, H, first, n, **kw):
    """the step schedule's per-frame launches: the drop-in path"""
    return _render(scene, W, H, first, n, N.SCHED_STEP, fused=False, **kw)


def _wf(scene, W, H, first, n, fused=True, **kw):
    return _render(scene, W, H, first, n, N.SCHED_WAVEFRONT, fused=fused, **kw)


def _same(a, b):
    assert a[0].tobytes() == b[0].tobytes(), f"{(a[0] != b[0]).any(axis=1).sum()} pixels differ"
    assert np.array_equal(a[1][0], b[1][0]) and a[1][1].tobytes() == b[1][1].tobytes()
    for key in ("rays", "node_visits", "tri_tests", "hits"):
        assert a[2][key] == b[2][key], key


@pytest.mark.parametrize("math", [N.MATH_PINNED, N.MATH_DEVICELIB, N.MATH_SHIPPED])
@pytest.mark.parametrize("fused", [True, False])
def test_wavefront_equals_step(cornell, math, fused):
    W, H = 320, 180
    _same(_wf(cornell, W, H, 1, 8, fused=fused, math=math), _step(cornell, W, H, 1, 8, math=math))


def test_wavefront_pinned_equals_oracle(cornell, oracle_mod):
    W, H = 192, 108
    got, (ids, t), _ = _wf(cornell, W, H, 1, 4, math=N.MATH_PINNED, bounces=5)
    res = np.zeros((W * H, 4), np.float32)
    for f in range(1, 5):
        res, wids, wt, _ = oracle_mod.render(cornell, W, H, frame_count=f, light_bounces=5, result=res,
                                             want_hits=True, threads=16)
    assert rgb(got).tobytes() == rgb(res).tobytes()
    assert np.array_equal(ids, wids) and t.tobytes() == wt.tobytes()


@pytest.mark.parametrize("first,n,pre", [(0, 3, None), (3, 5, (1, 2)), (1, 11, None)])
def test_wavefront_frame_sequences(cornell, first, n, pre):
    W, H = 200, 120
    _same(_wf(cornell, W, H, first, n, pre=pre), _step(cornell, W, H, first, n, pre=pre))


@pytest.mark.parametrize("bounces", [1, 2, 3, 0, 70])
def test_wavefront_bounce_counts(cornell, bounces):
    """1..64 bounces run the wavefront launches; 0 and > 64 fall back to the step schedule."""
    W, H = 160, 96
    _same(_wf(cornell, W, H, 1, 3, bounces=bounces), _step(cornell, W, H, 1, 3, bounces=bounces))


@pytest.mark.parametrize("period,phase", [(2, 1), (8, 0), (8, 5)])
def test_wavefront_band_interleave(cornell, period, phase):
    W, H = 256, 200
    _same(_wf(cornell, W, H, 1, 6, interleave=(period, phase)),
          _step(cornell, W, H, 1, 6, interleave=(period, phase)))


def test_wavefront_work_range_and_global_path(cornell):
    W, H = 240, 136
    n = W * H
    for wr, fg in (((n // 5, n - 77), False), ((0, n), True), ((333, n // 2), True)):
        _same(_wf(cornell, W, H, 1, 5, work_range=wr, force_global=fg),
              _step(cornell, W, H, 1, 5, work_range=wr, force_global=fg))


@pytest.mark.parametrize("W,H", [(77, 53), (8, 8), (1, 1), (513, 7)])
def test_wavefront_odd_sizes(cornell, W, H):
    _same(_wf(cornell, W, H, 1, 4), _step(cornell, W, H, 1, 4))


@pytest.mark.parametrize("tuning", [{"wf_streams_per_cu": 1}, {"wf_streams_per_cu": 64},
                                    {"wf_refill_min": 1}, {"wf_refill_min": 64},
                                    {"wf_top_nodes": 0, "tile_major": 1, "global_oct": 0},
                                    {"wf_top_nodes": 1024, "global_oct": 0}])
def test_wavefront_tuning_keeps_bits(cornell, tuning):
    W, H = 224, 128
    for fg in (False, True):
        _same(_wf(cornell, W, H, 1, 4, tuning=tuning, force_global=fg),
              _step(cornell, W, H, 1, 4, force_global=fg))


def test_wavefront_bunny_proxy():
    from clrt import proxy
    sc = proxy.bunny_proxy()
    W, H = 320, 180
    _same(_wf(sc, W, H, 1, 4), _step(sc, W, H, 1, 4))


def test_wavefront_repeated_calls_and_sky_chain(cornell):
    """Repeated wavefront renders on one kernel (queues reused, the accumulation's sky key chained
    from call to call, a skybox change, a restart at frame 1): every call equals the per-frame
    step launches."""
    W, H = 320, 180
    seq = [(1, 4, 1.0), (5, 4, 1.0), (9, 1, 1.0), (1, 8, 0.6), (9, 3, 0.6), (1, 2, 2.0)]
    outs = []
    for sched, fused in ((N.SCHED_WAVEFRONT, True), (N.SCHED_STEP, False)):
        r = HipRenderer(cornell, W, H, math=N.MATH_SHIPPED, hits=True, sched=sched)
        got = []
        for first, n, sky in seq:
            if fused:
                r.frame(first, light_bounces=9, skybox=sky, n_frames=n)
            else:
                for f in range(first, first + n):
                    r.frame(f, light_bounces=9, skybox=sky)
            got.append(r.result())
        r.close()
        outs.append(got)
    for a, b in zip(*outs):
        assert a.tobytes() == b.tobytes()

