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
