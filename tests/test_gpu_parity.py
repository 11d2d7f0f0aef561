"""GPU parity: the HIP hot path (librt_hip.so, pinned math mode) against the CPU oracle
on the same inputs.  Bar: bit-exact hit IDs, hit t and radiance (the pinned math makes
every builtin identical on both sides), identical section-8(d) counters."""
import numpy as np
import pytest

from clrt import _native as N
from hip_helpers import HipRenderer, rgb

pytestmark = pytest.mark.gpu
ORACLE_THREADS = 16


def _oracle(oracle_mod, scene, W, H, frames, lb, lt=0, sky=1.0, hits=False, first=0, last=None):
    res = np.zeros((W * H, 4), np.float32)
    counts = {"rays": 0, "node_visits": 0, "tri_tests": 0, "hits": 0}
    ids = t = None
    for f in frames:
        res, i, tt, c = oracle_mod.render(scene, W, H, frame_count=f, light_bounces=lb, light_type=lt,
                                          skybox=sky, result=res, want_hits=hits, first=first, last=last,
                                          threads=ORACLE_THREADS)
        if ids is None:
            ids, t = i, tt
        for key in counts:
            counts[key] += c[key]
    return res, ids, t, counts


def _assert_bits(a, b, what):
    a = np.ascontiguousarray(a)
    b = np.ascontiguousarray(b)
    diff = np.flatnonzero(a.view(np.uint32).ravel() != b.view(np.uint32).ravel())
    assert diff.size == 0, f"{what}: {diff.size} words differ, first at {diff[:8]}"


@pytest.mark.parametrize("W,H", [(512, 512), (128, 72)])
def test_primary_hits_bit_exact(cornell, oracle_mod, W, H):
    """Config 1 (512x512, primary rays only): hit IDs, t, radiance."""
    r = HipRenderer(cornell, W, H, hits=True, stats=True)
    r.frame(1, light_bounces=1)
    got = r.result()
    ids, t = r.hits()
    st = r.k.stats()
    r.close()
    want, wids, wt, c = _oracle(oracle_mod, cornell, W, H, [1], 1, hits=True)
    assert np.array_equal(ids, wids), f"{(ids != wids).sum()} hit ids differ"
    _assert_bits(t, wt, "hit t")
    _assert_bits(rgb(got), rgb(want), "radiance")
    for key in ("rays", "node_visits", "tri_tests", "hits"):
        assert st[key] == c[key], key


def test_1080p_two_bounces_bit_exact(cornell, oracle_mod):
    """Config 2 (1920x1080, primary + one secondary ray per pixel)."""
    r = HipRenderer(cornell, 1920, 1080, hits=True, stats=True)
    r.frame(1, light_bounces=2)
    got = r.result()
    ids, _ = r.hits()
    st = r.k.stats()
    r.close()
    want, wids, _, c = _oracle(oracle_mod, cornell, 1920, 1080, [1], 2, hits=True)
    assert np.array_equal(ids, wids)
    _assert_bits(rgb(got), rgb(want), "radiance")
    assert (st["rays"], st["node_visits"], st["tri_tests"], st["hits"]) == (
        c["rays"], c["node_visits"], c["tri_tests"], c["hits"])


def test_accumulate_8_frames_nine_bounces(cornell, oracle_mod):
    """Progressive 8 spp (frames 1..8 into one buffer, kernel_bvh.cl:449-455)."""
    W, H = 160, 90
    r = HipRenderer(cornell, W, H)
    for f in range(1, 9):
        r.frame(f, light_bounces=9)
    got = r.result()
    r.close()
    want, _, _, _ = _oracle(oracle_mod, cornell, W, H, range(1, 9), 9)
    _assert_bits(rgb(got), rgb(want), "8-frame radiance")


def test_4k_nine_bounces_frame1_bit_exact(cornell, oracle_mod):
    """Config 3's frame at full size: every pixel of a 3840x2160, 9-bounce frame."""
    W, H = 3840, 2160
    r = HipRenderer(cornell, W, H, stats=True)
    r.frame(1, light_bounces=9)
    got = r.result()
    st = r.k.stats()
    r.close()
    want, _, _, c = _oracle(oracle_mod, cornell, W, H, [1], 9)
    _assert_bits(rgb(got), rgb(want), "4K radiance")
    assert st["rays"] == c["rays"] and st["node_visits"] == c["node_visits"]


@pytest.mark.parametrize("lt,sky", [(1, 1.0), (2, 0.3), (-1, 2.0)])
def test_light_types_and_sky(cornell, oracle_mod, lt, sky):
    W, H = 200, 120
    r = HipRenderer(cornell, W, H)
    for f in (1, 2):
        r.frame(f, light_bounces=4, light_type=lt, skybox=sky)
    got = r.result()
    r.close()
    want, _, _, _ = _oracle(oracle_mod, cornell, W, H, (1, 2), 4, lt=lt, sky=sky)
    _assert_bits(rgb(got), rgb(want), f"lightType {lt}")


def test_frame_count_zero_path(cornell, oracle_mod):
    """frameCount == 0 takes pow(radiance, 0.45454545f) (kernel_bvh.cl:449-450)."""
    r = HipRenderer(cornell, 96, 64)
    r.frame(0, light_bounces=3)
    got = r.result()
    r.close()
    want, _, _, _ = _oracle(oracle_mod, cornell, 96, 64, [0], 3)
    _assert_bits(rgb(got), rgb(want), "frame 0")


@pytest.mark.parametrize("math", [N.MATH_PINNED, N.MATH_DEVICELIB, N.MATH_SHIPPED])
def test_schedules_agree_bit_exact(cornell, math):
    """The tile schedule (one pixel per lane, the reference's shape) and the step schedule compute
    identical pixels, primary hits and counters."""
    outs = []
    for sched in (N.SCHED_TILES, N.SCHED_STEP):
        r = HipRenderer(cornell, 301, 157, math=math, hits=True, stats=True, sched=sched)
        for f in (1, 2, 3):
            r.frame(f, light_bounces=9)
        outs.append((r.result(), r.hits(), r.k.stats()))
        r.close()
    for o in outs[1:]:
        _assert_bits(outs[0][0], o[0], "schedules")
        assert np.array_equal(outs[0][1][0], o[1][0])
        for key in ("rays", "node_visits", "tri_tests", "hits"):
            assert outs[0][2][key] == o[2][key], key


def test_zero_bounces_writes_black(cornell, oracle_mod):
    r = HipRenderer(cornell, 64, 48)
    r.frame(1, light_bounces=0)
    got = r.result()
    r.close()
    want, _, _, _ = _oracle(oracle_mod, cornell, 64, 48, [1], 0)
    _assert_bits(rgb(got), rgb(want), "0 bounces")


@pytest.mark.parametrize("math", [N.MATH_PINNED, N.MATH_SHIPPED])
def test_global_scene_path_equals_lds_path(cornell, math):
    outs = []
    for force in (False, True):
        r = HipRenderer(cornell, 256, 144, math=math, hits=True, force_global=force)
        r.frame(1, light_bounces=9)
        r.frame(2, light_bounces=9)
        outs.append((r.result(), r.hits()[0], r.k.scene_in_lds()))
        r.close()
    assert outs[0][2] is True and outs[1][2] is False
    _assert_bits(outs[0][0], outs[1][0], "global vs LDS")
    assert np.array_equal(outs[0][1], outs[1][1])


def test_row_tiles_compose_to_full_frame(cornell):
    """Work-item ranges (multi-GPU row tiles) keep global seeds: tiles == whole frame."""
    W, H = 333, 101  # not multiples of the 16x16 tile
    full = HipRenderer(cornell, W, H)
    full.frame(1, light_bounces=5)
    a = full.result()
    full.close()
    tiled = HipRenderer(cornell, W, H)
    cuts = [0, 17 * W, 17 * W + 5, 60 * W, W * H]
    for lo, hi in zip(cuts[:-1], cuts[1:]):
        tiled.frame(1, light_bounces=5, work_range=(lo, hi))
    b = tiled.result()
    tiled.close()
    _assert_bits(a, b, "tiled")


@pytest.mark.parametrize("sched", [N.SCHED_STEP, N.SCHED_WAVEFRONT])
def test_interleaved_bands_compose_full_frame(cornell, sched):
    """Multi-GPU sharding on one device: period-3 band interleave, each phase launched in
    turn (frames 1 and 2), equals the unsharded render; pack -> unpack round trip too."""
    from clrt import multigpu as mg
    W, H, P = 203, 75, 3
    full = HipRenderer(cornell, W, H, sched=sched)
    for f in (1, 2):
        full.frame(f, light_bounces=6)
    a = full.result()
    full.close()
    r = HipRenderer(cornell, W, H, sched=sched)
    for f in (1, 2):
        for ph in range(P):
            r.frame(f, light_bounces=6, interleave=(P, ph))
    b = r.result()
    _assert_bits(a, b, "banded")
    # pack each phase's bands to device staging and unpack into a fresh buffer
    import clrt
    dst = r.ctx.create_buffer(N.MEM_READ_WRITE, W * H * 16)
    for ph in range(P):
        stage = r.ctx.create_buffer(N.MEM_READ_WRITE, mg.staging_bytes(W, H, P))
        plan = mg.pack_plan(W, H, P, ph)
        mg.pack_device(r.ctx, r.out, plan, stage.device_pointer())
        r.ctx.Finish()
        mg.unpack_device(r.ctx, stage.device_pointer(), plan, dst)
        r.ctx.Finish()
        stage.release()
    c = np.zeros((W * H, 4), np.float32)
    r.ctx.ReadBuffer(dst, c, blocking=True)
    dst.release()
    r.close()
    _assert_bits(a, c, "pack/unpack")


def test_odd_global_size(cornell, oracle_mod):
    """global_work_size need not be W*H (the reference launches any 1-D NDRange)."""
    W, H = 100, 37
    n = W * H - 53
    r = HipRenderer(cornell, W, H, global_size=n)
    r.frame(1, light_bounces=2)
    got = r.result()
    r.close()
    want, _, _, _ = _oracle(oracle_mod, cornell, W, H, [1], 2, last=n)
    _assert_bits(rgb(got)[:n], rgb(want)[:n], "odd size")


def test_argument_validation_codes(cornell):
    import clrt
    ctx = clrt.CLContext(0)
    k = clrt.CLKernel(ctx)
    with pytest.raises(clrt.RTError) as e:
        ctx.ExecuteKernel(k, 16)
    assert e.value.code == -52  # CL_INVALID_KERNEL_ARGS
    with pytest.raises(clrt.RTError) as e:
        k.SetArgument(14, b"\0\0\0\0")
    assert e.value.code == -49  # CL_INVALID_ARG_INDEX
    with pytest.raises(clrt.RTError) as e:
        k.SetArgument(N.WIDTH, b"\0\0")
    assert e.value.code == -51  # CL_INVALID_ARG_SIZE
    with pytest.raises(clrt.RTError) as e:
        k.SetArgument(N.CAMERA_POS, b"\0" * 12)
    assert e.value.code == -51
    with pytest.raises(clrt.RTError) as e:
        clrt.CLKernel(ctx, "NotAKernel")
    assert e.value.code == -46
    with pytest.raises(clrt.RTError) as e:
        ctx.create_buffer(N.MEM_READ_ONLY, 0)
    assert e.value.code == -61
    k.release()
    ctx.release()


def test_malformed_bvh_is_rejected_not_run(cornell):
    """A node array whose child index points backwards must be an error, never a GPU walk."""
    bad = cornell.nodes.copy()
    interior = np.flatnonzero(bad["nPrimitives"] == 0)[0]
    bad["offset"][interior] = interior  # cycle
    import clrt
    sc = clrt.Scene(cornell.triangles, bad, cornell.materials)
    r = HipRenderer(sc, 64, 64)
    with pytest.raises(clrt.RTError) as e:
        r.frame(1, light_bounces=1)
    assert e.value.code == -38
    r.close()


@pytest.mark.parametrize("n_tris,in_lds", [(100, True), (144, False)])
def test_large_leaf_layouts(cornell, oracle_mod, n_tris, in_lds):
    """A root-only BVH whose one leaf holds n_tris triangles (Cornell's, repeated): up to 127
    fit the LDS node records' inline leaf code, more are rendered from the global layout;
    bit-exact against the oracle either way."""
    import dataclasses
    tris = np.concatenate([cornell.triangles, cornell.triangles])[:n_tris]
    p = np.concatenate([tris["v1"]["position"], tris["v2"]["position"], tris["v3"]["position"]])[:, :3]
    root = np.zeros(1, N.NODE_DTYPE)
    root["bmin"][0, :3] = p.min(0)
    root["bmax"][0, :3] = p.max(0)
    root["nPrimitives"] = len(tris)
    sc = dataclasses.replace(cornell, triangles=tris, nodes=root)
    W, H = 96, 64
    r = HipRenderer(sc, W, H, hits=True, stats=True)
    r.frame(1, light_bounces=4)
    got = r.result()
    ids, _ = r.hits()
    st = r.k.stats()
    assert r.k.scene_in_lds() == in_lds
    r.close()
    want, wids, _, c = _oracle(oracle_mod, sc, W, H, [1], 4, hits=True)
    assert np.array_equal(ids, wids)
    _assert_bits(rgb(got), rgb(want), "root-leaf radiance")
    assert (st["node_visits"], st["tri_tests"]) == (c["node_visits"], c["tri_tests"])


@pytest.mark.parametrize("math", [N.MATH_PINNED, N.MATH_SHIPPED])
def test_per_frame_sky_shortcut(cornell, oracle_mod, math):
    """Per-frame launches with the sky shortcut forced on (perframe_sky 2; by default it is used
    from ~1k pixels per wave): frames 1..6, then a frame with another skybox intensity (the key
    chain no longer matches the stored sky values, so the bit check must fall back to the full
    accumulation), then frames 8..9 -- bit-identical to the shortcut off and, pinned, to the oracle."""
    W, H = 192, 96
    seq = [(f, 1.0) for f in range(1, 7)] + [(7, 1.5)] + [(8, 1.5), (9, 1.0)]
    outs = []
    for mode in (2, 0):
        r = HipRenderer(cornell, W, H, math=math)
        r.k.set_tuning("perframe_sky", mode)
        for f, sky in seq:
            r.frame(f, light_bounces=3, skybox=sky)
        outs.append(r.result())
        r.close()
    assert outs[0].tobytes() == outs[1].tobytes()
    if math == N.MATH_PINNED:
        res = np.zeros((W * H, 4), np.float32)
        for f, sky in seq:
            res, _, _, _ = oracle_mod.render(cornell, W, H, frame_count=f, light_bounces=3, skybox=sky,
                                             result=res, threads=16)
        _assert_bits(rgb(outs[0]), rgb(res), "per-frame sky shortcut vs oracle")
