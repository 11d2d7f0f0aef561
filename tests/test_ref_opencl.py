"""GPU: the HIP path against the REFERENCE kernel itself.

Two sources for the reference's outputs:
  * the committed fixtures tests/golden/ref_*.npz (made on an MI355X by
    scripts/make_ref_goldens.py);
  * a live run: oracle/_ref/kernel_bvh_strict.co -- the unmodified kernel_bvh.cl built by
    the image's OpenCL compiler -- loaded through the system OpenCL runtime
    (oracle/clref.py).  Skipped when that runner or an OpenCL GPU device is absent.

Two reference builds (oracle/Makefile): `strict` (-ffp-contract=off
-cl-fp32-correctly-rounded-divide-sqrt) and `shipped` (the compiler's OpenCL defaults, what
the reference's clBuildProgram(" -I . ") gets: FP contraction, 2.5-ulp division, 3-ulp sqrt).
Bar for the devicelib math mode vs `strict` and the shipped mode vs `shipped`: bit-exact
primary hit IDs, hit t and radiance.  Bar for the pinned mode (bit-exact with the CPU oracle
elsewhere): the north-star tolerance, 1e-4 relative radiance.
"""
import numpy as np
import pytest

from clrt import _native as N
from hip_helpers import HipRenderer, rgb
from ref_compare import bits_differ, face_ids, load_golden, map_faces, rel_err

pytestmark = pytest.mark.gpu


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
def live_ref():
    r = _open_ref("strict")
    yield r
    r.close()


@pytest.fixture(scope="module")
def live_shipped():
    r = _open_ref("shipped")
    yield r
    r.close()


def _hip(scene, W, H, frames, bounces, math, hits=False):
    r = HipRenderer(scene, W, H, math=math, hits=hits)
    for f in frames:
        r.frame(f, light_bounces=bounces)
    out = rgb(r.result())
    h = r.hits() if hits else None
    r.close()
    return out, h


@pytest.mark.parametrize("W,H", [(128, 72), (512, 512)])
def test_devicelib_primary_hits_equal_reference_fixture(cornell, W, H):
    g = load_golden(f"ref_strict_hits_{W}x{H}")
    _, (ids, t) = _hip(cornell, W, H, [1], 1, N.MATH_DEVICELIB, hits=True)
    assert np.array_equal(ids, g["ids"]), f"{(ids != g['ids']).sum()} ids differ"
    assert bits_differ(t, g["t"]) == 0


@pytest.mark.parametrize("bounces,frames", [(1, 1), (2, 1), (9, 1), (9, 8)])
def test_devicelib_radiance_equals_reference_fixture(cornell, bounces, frames):
    g = load_golden(f"ref_strict_rad_128x72_b{bounces}_f{frames}")["rgb"]
    got, _ = _hip(cornell, 128, 72, range(1, frames + 1), bounces, N.MATH_DEVICELIB)
    assert bits_differ(got, g) == 0, f"{bits_differ(got, g)} words differ, max rel {rel_err(got, g).max():.3g}"


@pytest.mark.parametrize("W,H,bounces,frames", [(1920, 1080, 2, 1), (512, 512, 9, 8), (3840, 2160, 9, 1)])
def test_devicelib_equals_live_reference(cornell, live_ref, W, H, bounces, frames):
    want = live_ref.render(cornell, W, H, frames=range(1, frames + 1), light_bounces=bounces)[:, :3]
    got, _ = _hip(cornell, W, H, range(1, frames + 1), bounces, N.MATH_DEVICELIB)
    nd = bits_differ(got, want)
    assert nd == 0, f"{nd} words differ, max rel {rel_err(got, want).max():.3g}"


def test_devicelib_primary_hits_equal_live_reference_1080p(cornell, live_ref):
    ids_r, t_r = live_ref.primary_hits(cornell, 1920, 1080)
    _, (ids, t) = _hip(cornell, 1920, 1080, [1], 1, N.MATH_DEVICELIB, hits=True)
    assert np.array_equal(ids, ids_r)
    assert bits_differ(t, t_r) == 0


@pytest.mark.parametrize("W,H,bounces,frames", [(1920, 1080, 2, 1), (512, 512, 9, 8)])
def test_pinned_within_tolerance_of_live_reference(cornell, live_ref, W, H, bounces, frames):
    """Pinned mode vs the reference build: north-star tolerance on radiance (1e-4 rel) for
    all but paths that diverge (a ray that grazes an edge can take another branch after a
    1-ulp difference); those must stay rare."""
    want = live_ref.render(cornell, W, H, frames=range(1, frames + 1), light_bounces=bounces)[:, :3]
    got, _ = _hip(cornell, W, H, range(1, frames + 1), bounces, N.MATH_PINNED)
    err = rel_err(got, want).max(axis=1)
    frac_out = float((err > 1e-4).mean())
    assert frac_out <= 1e-4, f"{frac_out:.2e} of pixels beyond 1e-4"


def test_pinned_primary_faces_equal_live_reference(cornell, live_ref):
    ids_r, t_r = live_ref.primary_hits(cornell, 1920, 1080)
    _, (ids, t) = _hip(cornell, 1920, 1080, [1], 1, N.MATH_PINNED, hits=True)
    faces = face_ids(cornell)
    agree = (map_faces(ids, faces) == map_faces(ids_r, faces)).mean()
    assert np.array_equal(ids >= 0, ids_r >= 0)
    assert agree >= 0.9995


# ---- the shipped math mode vs the reference as its host builds it ---------------------------
def test_shipped_primary_hits_equal_reference_fixture(cornell):
    g = load_golden("ref_shipped_hits_128x72")
    _, (ids, t) = _hip(cornell, 128, 72, [1], 1, N.MATH_SHIPPED, hits=True)
    assert np.array_equal(ids, g["ids"]), f"{(ids != g['ids']).sum()} ids differ"
    assert bits_differ(t, g["t"]) == 0


@pytest.mark.parametrize("bounces,frames", [(1, 1), (2, 1), (9, 1), (9, 8)])
def test_shipped_radiance_equals_reference_fixture(cornell, bounces, frames):
    g = load_golden(f"ref_shipped_rad_128x72_b{bounces}_f{frames}")["rgb"]
    got, _ = _hip(cornell, 128, 72, range(1, frames + 1), bounces, N.MATH_SHIPPED)
    assert bits_differ(got, g) == 0, f"{bits_differ(got, g)} words differ, max rel {rel_err(got, g).max():.3g}"


@pytest.mark.parametrize("W,H", [(512, 512), (1920, 1080)])
def test_shipped_primary_hits_equal_live_reference(cornell, live_shipped, W, H):
    ids_r, t_r = live_shipped.primary_hits(cornell, W, H)
    _, (ids, t) = _hip(cornell, W, H, [1], 1, N.MATH_SHIPPED, hits=True)
    assert np.array_equal(ids, ids_r), f"{(ids != ids_r).sum()} ids differ"
    assert bits_differ(t, t_r) == 0


@pytest.mark.parametrize("W,H,bounces,frames", [(1920, 1080, 2, 1), (512, 512, 9, 8), (3840, 2160, 9, 1)])
def test_shipped_equals_live_reference(cornell, live_shipped, W, H, bounces, frames):
    want = live_shipped.render(cornell, W, H, frames=range(1, frames + 1), light_bounces=bounces)[:, :3]
    got, _ = _hip(cornell, W, H, range(1, frames + 1), bounces, N.MATH_SHIPPED)
    nd = bits_differ(got, want)
    assert nd == 0, f"{nd} words differ, max rel {rel_err(got, want).max():.3g}"
