"""GPU: host-side state of the C ABI across launches -- the derived scene data (octant / global
node records, packed triangles, shading records, LDS top of the tree) must follow whatever is
bound to the kernel's argument slots, as the reference's kernel arguments do (CLutils.cpp:68-77).
Checked bit-exact against the oracle (pinned math)."""
import dataclasses

import numpy as np
import pytest

from clrt import _native as N
from hip_helpers import HipRenderer, rgb

pytestmark = pytest.mark.gpu


def _oracle_frame(oracle_mod, scene, W, H, lb, first=0, last=None):
    res = np.zeros((W * H, 4), np.float32)
    res, _, _, _ = oracle_mod.render(scene, W, H, frame_count=1, light_bounces=lb, result=res, first=first,
                                     last=last, threads=16)
    return res


def _bind(r, scene):
    flags = N.MEM_READ_ONLY | N.MEM_COPY_HOST_PTR
    bufs = [r.ctx.create_buffer(flags, a.nbytes, a) for a in (scene.triangles, scene.nodes, scene.materials)]
    r.k.set_buffer(N.BUFFER_SCENE, bufs[0])
    r.k.set_buffer(N.BUFFER_NODE, bufs[1])
    r.k.set_buffer(N.BUFFER_MATERIAL, bufs[2])
    return bufs


def test_rebinding_scenes_switches_paths(cornell, oracle_mod):
    """Cornell (LDS path) -> bunny proxy (global path, top of tree in LDS) -> Cornell again on one
    kernel: each launch renders the scene currently bound."""
    from clrt import proxy
    bunny = proxy.bunny_proxy()
    W, H = 96, 64
    r = HipRenderer(cornell, W, H)
    keep = []
    for sc, in_lds in ((cornell, True), (bunny, False), (cornell, True)):
        keep.append(_bind(r, sc))
        r.frame(1, light_bounces=3)
        got = rgb(r.result())
        assert r.k.scene_in_lds() is in_lds
        want = rgb(_oracle_frame(oracle_mod, sc, W, H, 3))
        assert (got.view(np.uint32) == want.view(np.uint32)).all()
    r.ctx.Finish()
    for bufs in keep:
        for b in bufs:
            b.release()
    r.close()


def test_rewriting_a_bound_buffer_repacks(cornell, oracle_mod):
    """WriteBuffer into the bound material buffer (same size, new contents) is seen by the next
    launch: the derived shading records are rebuilt."""
    W, H = 80, 48
    r = HipRenderer(cornell, W, H)
    r.frame(1, light_bounces=4)
    mats = cornell.materials.copy()
    mats["diffuse"][:, :3] *= np.float32(0.5)
    mats["roughness"] = np.float32(20.0)
    r.ctx.WriteBuffer(r.bufs[2], mats)
    r.frame(1, light_bounces=4)
    got = rgb(r.result())
    r.close()
    sc2 = dataclasses.replace(cornell, materials=mats)
    want = rgb(_oracle_frame(oracle_mod, sc2, W, H, 4))
    assert (got.view(np.uint32) == want.view(np.uint32)).all()


def test_8k_frame_slice_matches_oracle(cornell, oracle_mod):
    """7680x4320 (33 M work-items): a band of rows through the middle, bit-exact."""
    W, H = 7680, 4320
    lo, hi = 2100 * W, 2132 * W
    r = HipRenderer(cornell, W, H)
    r.frame(1, light_bounces=2, work_range=(lo, hi))
    got = rgb(r.result())[lo:hi]
    r.close()
    want = rgb(_oracle_frame(oracle_mod, cornell, W, H, 2, first=lo, last=hi))[lo:hi]
    assert (got.view(np.uint32) == want.view(np.uint32)).all()


def test_retired_schedules_and_tunings_are_refused(cornell):
    """The path-regeneration (1) and LDS path-pool (3) schedules and the pool's three tunings
    (10-12) were retired in round 3: the C ABI refuses them (CL_INVALID_VALUE) and the kernel keeps
    its previous schedule, which still renders."""
    r = HipRenderer(cornell, 64, 48)
    for sched in (1, 3, 5, -1):
        with pytest.raises(N.RTError) as e:
            r.k.set_schedule(sched)
        assert e.value.code == -30  # CL_INVALID_VALUE
    lib = r.k._lib
    for tid in (10, 11, 12):
        assert lib.rtKernelSetTuning(r.k.handle, tid, 16) == -30
    for sched in (N.SCHED_TILES, N.SCHED_STEP, N.SCHED_WAVEFRONT):
        r.k.set_schedule(sched)
    r.frame(1, light_bounces=2)
    assert np.isfinite(r.result()).all()
    r.close()


def test_round5_tuning_ranges(cornell):
    """Round-5 tunings: TILE_MAJOR takes -1..2 (2: pixel-major), CHUNK_PIXELS takes 0 (auto) or multiples
    of 64 up to 4096, the HBM/L2 step weights take 0 (auto) ..1000; out-of-range values are refused and
    leave the setting as it was; 22 (the retired speculative walk) stays refused."""
    r = HipRenderer(cornell, 64, 48)
    lib, h = r.k._lib, r.k.handle
    ok = [(N.TUNING["tile_major"], v) for v in (-1, 0, 1, 2)] + \
         [(N.TUNING["chunk_pixels"], v) for v in (0, 64, 1024, 4096)] + \
         [(N.TUNING["step_weight_node_global"], v) for v in (0, 1, 1000)] + \
         [(N.TUNING["step_weight_leaf_global"], v) for v in (0, 65)]
    for tid, v in ok:
        assert lib.rtKernelSetTuning(h, tid, v) == 0, (tid, v)
        assert r.k.get_tuning([k for k, i in N.TUNING.items() if i == tid][0]) == v
    bad = [(N.TUNING["tile_major"], 3), (N.TUNING["tile_major"], -2), (N.TUNING["chunk_pixels"], 96),
           (N.TUNING["chunk_pixels"], 8192), (N.TUNING["step_weight_node_global"], 1001),
           (N.TUNING["step_weight_leaf_global"], -1), (22, 1)]
    for tid, v in bad:
        assert lib.rtKernelSetTuning(h, tid, v) == -30, (tid, v)
    r.frame(1, light_bounces=2)
    assert np.isfinite(r.result()).all()
    r.close()
