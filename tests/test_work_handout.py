"""GPU: the persistent schedules' work hand-out hands every work item out exactly once, whatever
path a launch takes (rt_capi.cpp chunk rule, step_body take_tile / next_chunk): per-frame launches
with counter partitions (>= 256 work items per wave: 1080p and up), with a static first chunk and
one tail counter (smaller frames), with a bulk region (4K), odd sizes whose last tiles are partial,
and small tail chunks.  Consecutive per-frame launches also alternate between the two counter slots
(each launch zeroes the next one's).  A pixel handed out twice or never would change the gamma
accumulation or the primary hits, so per-frame launches must leave exactly the bits of the same
frames rendered as one fused launch (whose work is handed out from its own counters)."""
import numpy as np
import pytest

from clrt import _native as N
from hip_helpers import HipRenderer

pytestmark = pytest.mark.gpu


def _render(scene, W, H, n, fused, tuning=None, bounces=2, interleave=None):
    r = HipRenderer(scene, W, H, math=N.MATH_SHIPPED, hits=True)
    r.ctx.WriteBuffer(r.hit_bufs[0], np.full(W * H, -2, np.int32))  # "never written"
    # one real launch per frame: no coalescing (HipRenderer's default batch of 1), no deferral
    r.k.set_tuning("perframe_defer", 0)
    for name, value in (tuning or {}).items():
        r.k.set_tuning(name, value)
    if fused:
        r.frame(1, light_bounces=bounces, n_frames=n, interleave=interleave)
    else:
        for f in range(1, n + 1):
            r.frame(f, light_bounces=bounces, interleave=interleave)
    out = (r.result(), r.hits())
    r.close()
    return out


def _same(a, b, interleaved=False):
    assert a[0].tobytes() == b[0].tobytes(), f"{(a[0] != b[0]).any(axis=1).sum()} pixels differ"
    assert np.array_equal(a[1][0], b[1][0]) and a[1][1].tobytes() == b[1][1].tobytes()
    for x in (a, b):
        assert (x[1][0] >= -1).all() or interleaved  # every pixel's primary hit was written (-1: a miss)


@pytest.mark.parametrize("W,H", [(1920, 1080), (1930, 1091), (2560, 1440), (1280, 720), (3840, 2160)])
def test_per_frame_handout_matches_fused(cornell, W, H):
    _same(_render(cornell, W, H, 3, False), _render(cornell, W, H, 3, True))


@pytest.mark.parametrize("tail", [64, 128, 256])
def test_partitioned_tail_chunks(cornell, tail):
    """1080p per-frame launches (8 counter partitions) at every tail chunk size."""
    W, H = 1920, 1080
    _same(_render(cornell, W, H, 2, False, tuning={"tail_chunk": tail}), _render(cornell, W, H, 2, True))


def test_per_frame_handout_bunny_proxy():
    """The HBM/L2 octant walk's per-frame launches (no LDS ring) on the same hand-out."""
    from clrt import proxy
    sc = proxy.bunny_proxy()
    _same(_render(sc, 1920, 1080, 2, False), _render(sc, 1920, 1080, 2, True))


def test_counter_slots_across_launch_sizes(cornell):
    """Per-frame launches of different sizes on one kernel alternate between the two counter slots: a
    partitioned 1080p launch (slot 0, 8 partitions), a small work-range launch (slot 1, one counter),
    then the full frame again (slot 0).  Each launch zeroes every partition of the next slot, not just
    the ones it uses, or the third launch would start from the first one's spent counters and skip
    pixels.  Reference: the same sequence on the tile schedule (no counters)."""
    W, H = 1920, 1080

    def seq(sched):
        r = HipRenderer(cornell, W, H, math=N.MATH_SHIPPED, hits=True, sched=sched)
        r.ctx.WriteBuffer(r.hit_bufs[0], np.full(W * H, -2, np.int32))
        if sched == N.SCHED_STEP:
            r.k.set_tuning("perframe_defer", 0)
        r.frame(1, light_bounces=2)
        r.frame(2, light_bounces=2, work_range=(0, 64 * 1024))
        r.k.set_work_range(0, 0)  # the whole frame again
        r.frame(3, light_bounces=2)
        out = (r.result(), r.hits())
        r.close()
        return out

    _same(seq(N.SCHED_STEP), seq(N.SCHED_TILES))


@pytest.mark.parametrize("period,phase", [(2, 1), (3, 0)])
def test_per_frame_handout_band_interleave(cornell, period, phase):
    """A multi-GPU rank's share (every period-th 8-row band) of a 4K frame: 4.1 / 2.8 M work items per
    launch -- counter partitions over the rank's bands."""
    W, H = 3840, 2160
    _same(_render(cornell, W, H, 2, False, interleave=(period, phase)),
          _render(cornell, W, H, 2, True, interleave=(period, phase)), interleaved=True)
