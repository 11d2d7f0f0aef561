"""GPU: the reference's INTERACTIVE inputs, in the default math modes, against the reference
kernel run live through OpenCL (oracle/clref.py).

The benched and fixture tests use the reference's startup state (light type 0, sky 1.0, the
default camera, frames from 1).  Its UI changes every one of those (Config):
  * camera rotation: CLCamera::Update (CLcamera.h:15-21), from the "Camera Rotation" drag
    (CLui.cpp:221-228); camera moves by the arrow keys (CLEngineBase.cpp:141-162);
  * point and spot lights: lightPixel's lightType 1 and 2 (kernel_bvh.cl:322-344), slider
    CLui.cpp:255;
  * frameCount 0: every slider resets it (CLui.cpp:218-262), so the next frame takes
    pow(radiance, 0.45454545f) (kernel_bvh.cl:449-450) and the following ones accumulate;
  * skybox intensity (CLui.cpp:240) and up to 20 light bounces (CLui.cpp:250).
With a rotated camera cross(front, up) is no longer (1, 0, 0), so the camera-basis sum
(kernel_bvh.cl:400) and its contraction site are exercised with non-trivial products; light
types 1 and 2 run the `origin + dir * t` point (kernel_bvh.cl:328) that type 0 never reaches.

Bar (as for the benched path): shipped math == the reference as its host builds it, devicelib
== the reference built strict, bit for bit on radiance, primary hit IDs and t; per-frame
launches (rtEnqueueKernel, the RenderFrame loop) and fused launches (rtEnqueueKernelFrames).
"""
import numpy as np
import pytest

from clrt import _native as N
from hip_helpers import DEFAULT_CAMERA, HipRenderer, reference_camera, rgb
from ref_compare import bits_differ, rel_err

pytestmark = pytest.mark.gpu

ROTATED = reference_camera(1.40, 1.25)
MOVED = reference_camera(1.40, 1.25, moves=("up", "up", "right", "left", "left", "left"))

# name -> (camera, light_type, skybox, bounces, first frame, frames)
SCENARIOS = {
    "light1": (DEFAULT_CAMERA, 1, 1.0, 9, 1, 3),
    "light2": (DEFAULT_CAMERA, 2, 1.0, 9, 1, 3),
    "frame0": (DEFAULT_CAMERA, 0, 1.0, 9, 0, 4),
    "rotated": (ROTATED, 0, 1.0, 9, 1, 3),
    "moved": (MOVED, 0, 1.0, 9, 1, 3),
    "sky07_b20": (DEFAULT_CAMERA, 0, 0.7, 20, 1, 3),
    "all": (MOVED, 2, 0.7, 20, 0, 4),
}
MODES = {"shipped": (N.MATH_SHIPPED, "shipped"), "devicelib": (N.MATH_DEVICELIB, "strict")}


def _open_ref(variant):
    import clref
    ok, why = clref.available()
    if not ok:
        pytest.skip(why)
    try:
        return clref.ReferenceKernel(variant)
    except RuntimeError as e:
        pytest.skip(f"no OpenCL GPU device for the reference: {e}")


@pytest.fixture(scope="module")
def refs():
    opened = {}

    def get(variant):
        if variant not in opened:
            opened[variant] = _open_ref(variant)
        return opened[variant]

    yield get
    for r in opened.values():
        r.close()


def _hip(scene, W, H, math, cam, lt, sky, lb, f0, nf, fused):
    r = HipRenderer(scene, W, H, math=math, hits=True)
    if fused:
        r.frame(f0, light_bounces=lb, light_type=lt, skybox=sky, camera=cam, n_frames=nf)
    else:
        for f in range(f0, f0 + nf):
            r.frame(f, light_bounces=lb, light_type=lt, skybox=sky, camera=cam)
    out = rgb(r.result())
    ids, t = r.hits()
    r.close()
    return out, ids, t


def _check(ref, scene, W, H, math, scenario, fused):
    cam, lt, sky, lb, f0, nf = SCENARIOS[scenario]
    want = ref.render(scene, W, H, frames=range(f0, f0 + nf), light_bounces=lb, light_type=lt,
                      skybox=sky, camera=cam)[:, :3]
    ids_r, t_r = ref.primary_hits(scene, W, H, frame=f0 + nf - 1, camera=cam)
    got, ids, t = _hip(scene, W, H, math, cam, lt, sky, lb, f0, nf, fused)
    nd = bits_differ(got, want)
    assert nd == 0, f"{scenario}: {nd} radiance words differ, max rel {rel_err(got, want).max():.3g}"
    assert np.array_equal(ids, ids_r), f"{scenario}: {(ids != ids_r).sum()} primary hit ids differ"
    assert bits_differ(t, t_r) == 0, f"{scenario}: primary t differs"
    return got, ids


def test_cameras_are_not_trivial():
    """The rotated/moved cameras exercise what the default one does not: a right vector
    cross(front, up) with two non-zero components, a front with three, and a position off the
    default."""
    for cam in (ROTATED, MOVED):
        right = np.cross(np.array(cam[1], np.float32), np.array(cam[2], np.float32))
        assert np.count_nonzero(right) >= 2 and np.count_nonzero(cam[1]) == 3
    assert MOVED[0] != DEFAULT_CAMERA[0] and MOVED[0] != ROTATED[0]


@pytest.mark.parametrize("fused", [False, True], ids=["perframe", "fused"])
@pytest.mark.parametrize("mode", list(MODES))
@pytest.mark.parametrize("scenario", list(SCENARIOS))
def test_cornell_interactive_inputs_equal_live_reference(cornell, refs, scenario, mode, fused):
    math, variant = MODES[mode]
    got, ids = _check(refs(variant), cornell, 512, 512, math, scenario, fused)
    assert (ids >= 0).sum() > 1000, "the view must hit the scene"
    assert np.isfinite(got).all()


@pytest.mark.parametrize("fused", [False, True], ids=["perframe", "fused"])
@pytest.mark.parametrize("scenario", ["rotated", "all"])
def test_cornell_interactive_1080p_shipped(cornell, refs, scenario, fused):
    """Config 2's size, the default build."""
    _check(refs("shipped"), cornell, 1920, 1080, N.MATH_SHIPPED, scenario, fused)


def test_cornell_interactive_4k_fused_shipped(cornell, refs):
    """The benched launch (fused, 3840x2160, the default build) with every interactive input."""
    _check(refs("shipped"), cornell, 3840, 2160, N.MATH_SHIPPED, "all", True)


@pytest.mark.parametrize("fused", [False, True], ids=["perframe", "fused"])
@pytest.mark.parametrize("mode", list(MODES))
def test_bunny_interactive_inputs_equal_live_reference(refs, mode, fused):
    """The 70k-triangle proxy (octant walk over HBM/L2) with every interactive input at once."""
    import clrt.proxy as P
    math, variant = MODES[mode]
    _, ids = _check(refs(variant), P.bunny_proxy(), 640, 360, math, "all", fused)
    assert (ids >= 0).sum() > 1000


@pytest.mark.parametrize("mode", list(MODES))
def test_ui_session_sequence_equals_live_reference(cornell, refs, mode):
    """An interactive session on one output buffer, per-frame launches as RenderFrame issues them:
    frames 1-3 at startup; the rotation drag resets frameCount to 0 (CLui.cpp:227), frames 0-2
    with the new camera; an arrow key sets frameCount 1 (CLEngineBase.cpp:146), frames 1-2 with
    the moved camera; the light-type and bounce sliders reset to 0, frames 0-2.  The buffer carries
    over between the segments, as the reference's output buffer does."""
    math, variant = MODES[mode]
    ref = refs(variant)
    W, H = 384, 256
    session = [  # (camera, light_type, sky, bounces, frames)
        (DEFAULT_CAMERA, 0, 1.0, 9, range(1, 4)),
        (ROTATED, 0, 1.0, 9, range(0, 3)),
        (reference_camera(1.40, 1.25, moves=("up",)), 0, 1.0, 9, range(1, 3)),
        (reference_camera(1.40, 1.25, moves=("up",)), 1, 0.7, 20, range(0, 3)),
    ]
    want = np.zeros((W * H, 4), np.float32)
    for cam, lt, sky, lb, frames in session:
        want = ref.render(cornell, W, H, frames=frames, light_bounces=lb, light_type=lt, skybox=sky,
                          camera=cam, result=want)
    r = HipRenderer(cornell, W, H, math=math)
    for cam, lt, sky, lb, frames in session:
        for f in frames:
            r.frame(f, light_bounces=lb, light_type=lt, skybox=sky, camera=cam)
    got = rgb(r.result())
    r.close()
    nd = bits_differ(got, want[:, :3])
    assert nd == 0, f"{nd} words differ"


@pytest.mark.parametrize("scenario", ["rotated", "moved", "all"])
def test_pinned_interactive_inputs_equal_oracle(cornell, oracle_mod, scenario):
    """Pinned math vs the CPU oracle (include/rt_pinned_math.h on both sides) on the same
    interactive inputs: bit-exact radiance, primary hit IDs and t, and the section-8(d) counters."""
    cam, lt, sky, lb, f0, nf = SCENARIOS[scenario]
    W, H = 320, 200
    r = HipRenderer(cornell, W, H, math=N.MATH_PINNED, hits=True, stats=True)
    for f in range(f0, f0 + nf):
        r.frame(f, light_bounces=lb, light_type=lt, skybox=sky, camera=cam)
    got = rgb(r.result())
    ids, t = r.hits()
    st = r.k.stats()
    r.close()
    res = np.zeros((W * H, 4), np.float32)
    counts = dict.fromkeys(("rays", "node_visits", "tri_tests", "hits"), 0)
    for f in range(f0, f0 + nf):
        res, wids, wt, c = oracle_mod.render(cornell, W, H, frame_count=f, light_bounces=lb, light_type=lt,
                                             skybox=sky, camera=cam, result=res, want_hits=True, threads=16)
        for key in counts:
            counts[key] += c[key]
    assert bits_differ(got, rgb(res)) == 0
    assert np.array_equal(ids, wids)
    assert bits_differ(t, wt) == 0
    for key in counts:
        assert st[key] == counts[key], key
