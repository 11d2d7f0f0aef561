"""GPU: the exact code path bench.py times, at the bench's full size, against the REFERENCE.

bench.py's step is rtEnqueueKernelFrames(ctx, k, 3840*2160, 8) in the shipped math (frames
1..8, 9 bounces), queued back to back: fused (frame, pixel) work order, camera-ray ring, sky
flags, the accumulation launch overlapping the next step's render on the second stream with
alternating radiance sets.  Here that same sequence runs three steps deep and the image must
equal the reference kernel's 8-frame accumulation (kernel_bvh.cl:415-456, built as its host
builds it and run live through OpenCL, oracle/clref.py) bit for bit, with the last frame's
primary hit IDs and t.  The bunny-class proxy (config 5, the HBM/L2 scene path with its
tile-major fused order at this size) gets the same check.
"""
import numpy as np
import pytest

from clrt import _native as N
from hip_helpers import HipRenderer, rgb
from ref_compare import bits_differ, rel_err

pytestmark = pytest.mark.gpu

W4K, H4K = 3840, 2160


def _open_ref(variant):
    import clref
    ok, why = clref.available()
    if not ok:
        pytest.skip(why)
    try:
        return clref.ReferenceKernel(variant)
    except RuntimeError as e:
        pytest.skip(f"no OpenCL GPU device for the reference: {e}")


def _bench_steps(scene, steps=3, frames=8, sched=N.SCHED_STEP):
    """bench.py's timed loop on one GPU: `steps` fused 8-frame renders queued back to back."""
    r = HipRenderer(scene, W4K, H4K, math=N.MATH_SHIPPED, hits=True, sched=sched)
    for _ in range(steps):
        r.frame(1, light_bounces=9, n_frames=frames)
    r.ctx.Finish()
    got = rgb(r.result())
    ids, t = r.hits()
    in_lds = r.k.scene_in_lds()
    r.close()
    return got, ids, t, in_lds


def _check(scene, want_lds, frames, sched=N.SCHED_STEP):
    ref = _open_ref("shipped")
    want = ref.render(scene, W4K, H4K, frames=range(1, frames + 1), light_bounces=9)[:, :3]
    ids_r, t_r = ref.primary_hits(scene, W4K, H4K, frame=frames)
    ref.close()
    got, ids, t, in_lds = _bench_steps(scene, frames=frames, sched=sched)
    assert in_lds == want_lds
    nd = bits_differ(got, want)
    assert nd == 0, f"{nd} radiance words differ, max rel {rel_err(got, want).max():.3g}"
    assert np.array_equal(ids, ids_r), f"{(ids != ids_r).sum()} primary hit ids differ"
    assert bits_differ(t, t_r) == 0


def test_benched_cornell_4k_8spp_equals_live_reference(cornell):
    _check(cornell, True, 8)


def test_benched_bunny_4k_8spp_equals_live_reference():
    import clrt.proxy as P
    _check(P.bunny_proxy(), False, 8)


@pytest.mark.parametrize("scene_name", ["cornell", "bunny"])
def test_wavefront_4k_8spp_equals_live_reference(cornell, scene_name):
    """bench.py --sched wavefront (extend / shade launches per bounce over the HBM ray queues)
    at full size: the same bits as the reference."""
    if scene_name == "cornell":
        _check(cornell, True, 8, sched=N.SCHED_WAVEFRONT)
    else:
        import clrt.proxy as P
        _check(P.bunny_proxy(), False, 8, sched=N.SCHED_WAVEFRONT)


def _rank_steps(scene, period, phase, steps=3):
    """one rank's share of an N-GPU bench (bench.py --gpus N): its interleaved 8-row bands of the
    fused 4K 8-frame step, queued back to back as in the timed loop"""
    r = HipRenderer(scene, W4K, H4K, math=N.MATH_SHIPPED)
    if period > 1:
        r.k.set_row_interleave(period, phase)
    for _ in range(steps):
        r.frame(1, light_bounces=9, n_frames=8)
    r.ctx.Finish()
    out = r.result().reshape(H4K, W4K, 4)
    r.close()
    return out


@pytest.mark.parametrize("scene_name", ["cornell", "bunny"])
def test_rank_shares_at_full_size_compose_the_benched_image(cornell, scene_name):
    """The per-rank work of the 8-GPU bench (configs 4 and 5) at full size: every rank of 8 renders
    their bands with the small-launch chunking (tail reserve) and the frame-major order of small
    launches; their rows must be the bits of the one-GPU render (itself pinned to the reference
    above), and they must leave every other row untouched (zero)."""
    if scene_name == "cornell":
        sc = cornell
    else:
        import clrt.proxy as P
        sc = P.bunny_proxy()
    full = _rank_steps(sc, 1, 0)
    rows = np.arange(H4K)
    for phase in range(8):
        got = _rank_steps(sc, 8, phase)
        mine = (rows // 8) % 8 == phase
        assert got[mine].tobytes() == full[mine].tobytes(), f"rank {phase}: band rows differ"
        assert not got[~mine].any(), f"rank {phase} wrote rows outside its bands"
