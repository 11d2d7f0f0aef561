"""CPU tests of the oracle (test infrastructure) and the pinned math it shares with the
HIP kernels.  Known answers come from the reference's own definitions
(/root/reference/kernel_bvh.cl) and from the survey's probe of the reference kernel
(BASELINE.md section 3)."""
import ctypes
import math
import struct

import numpy as np
import pytest


def f32(x):
    return struct.unpack("<f", struct.pack("<f", x))[0]


def test_frame_hash_and_hash_known_answers(oracle_mod):
    L = oracle_mod.lib()
    # HashUInt32 (kernel_bvh.cl:57-59): 1103515245*x + 12345 mod 2^32
    for x in (0, 1, 2, 7, 0xFFFFFFFF, 123456789):
        assert L.oracle_frame_hash(x) == (1103515245 * x + 12345) & 0xFFFFFFFF
    # hash (kernel_bvh.cl:60-67) restated in Python integers
    def h(x):
        x ^= x >> 16
        x = (x * 0x7FEB352D) & 0xFFFFFFFF
        x ^= x >> 15
        x = (x * 0x846CA68B) & 0xFFFFFFFF
        x ^= x >> 16
        return x
    rng = np.random.default_rng(1)
    for x in [0, 1, 0xFFFFFFFF] + [int(v) for v in rng.integers(0, 2**32, 200, dtype=np.uint64)]:
        assert L.oracle_hash(x) == h(x)


def test_get_random_float_is_hash_over_2pow32(oracle_mod):
    L = oracle_mod.lib()
    s = ctypes.c_uint32(12345)
    for _ in range(100):
        before = s.value
        r = L.oracle_rand(ctypes.byref(s))
        # float(hash)/float(0xffffffff): 0xffffffff rounds to 2^32 in fp32
        assert r == f32(float(np.float32(s.value)) / 4294967296.0)
        assert s.value == L.oracle_hash(before)
        assert 0.0 <= r <= 1.0


def test_pinned_pow_special_and_accuracy(oracle_mod):
    L = oracle_mod.lib()
    inf, nan = float("inf"), float("nan")
    assert L.oracle_pow(0.0, 2.0) == 0.0
    assert L.oracle_pow(0.0, -1.5) == inf           # roughness Ns 0 -> alpha = inf path
    assert L.oracle_pow(5.0, 0.0) == 1.0
    assert L.oracle_pow(1.0, nan) == 1.0
    assert math.isnan(L.oracle_pow(-2.0, 0.5))
    assert L.oracle_pow(-2.0, 3.0) == -8.0
    assert L.oracle_pow(inf, 2.0) == inf
    assert L.oracle_pow(3.0, 2.0) == 9.0
    rng = np.random.default_rng(7)
    xs = rng.uniform(1e-6, 50.0, 4000).astype(np.float32)
    ys = rng.uniform(-3.0, 3.0, 4000).astype(np.float32)
    for x, y in zip(xs, ys):
        got = L.oracle_pow(float(x), float(y))
        want = float(np.float32(float(x) ** float(y)))
        assert got == pytest.approx(want, rel=2.5e-7), (x, y)


def test_pinned_trig(oracle_mod):
    L = oracle_mod.lib()
    rng = np.random.default_rng(3)
    for x in rng.uniform(0.0, 6.3, 4000).astype(np.float32):
        assert L.oracle_sin(float(x)) == pytest.approx(float(np.float32(math.sin(float(x)))), abs=1.2e-7)
        assert L.oracle_cos(float(x)) == pytest.approx(float(np.float32(math.cos(float(x)))), abs=1.2e-7)
    a = f32(0.5 * f32(f32(45.0 * f32(3.1415)) / 180.0))
    assert L.oracle_tan(a) == f32(math.tan(a))


def test_pinned_sincos_equals_sin_and_cos(oracle_mod):
    """pm_sincos (one reduction, used by the kernels) == pm_sin / pm_cos bit for bit."""
    L = oracle_mod.lib()
    rng = np.random.default_rng(11)
    xs = np.concatenate([rng.uniform(0.0, 6.2831855, 2_000_000), rng.uniform(-1e6, 1e6, 200_000),
                         [0.0, -0.0, 1e-30, np.pi / 2, np.pi, 3 * np.pi / 2, 2 * np.pi, 1e30, np.inf,
                          -np.inf, np.nan]]).astype(np.float32)
    assert L.oracle_sincos_mismatches(xs.ctypes.data, xs.size) == 0


def test_pinned_max_min_rules(oracle_mod):
    L = oracle_mod.lib()
    nan = float("nan")
    assert L.oracle_max(0.0, nan) == 0.0 and L.oracle_max(nan, 2.0) == 2.0
    assert L.oracle_min(5.0, nan) == 5.0
    # OpenCL common-function tie rule: max(x, y) = y if x < y else x
    assert math.copysign(1, L.oracle_max(0.0, -0.0)) == 1.0
    assert math.copysign(1, L.oracle_max(-0.0, 0.0)) == -1.0


def _node(bmin, bmax):
    import clrt
    n = np.zeros(1, clrt.NODE_DTYPE)
    n["bmin"][0, :3] = bmin
    n["bmax"][0, :3] = bmax
    return n


def _tri(p1, p2, p3):
    import clrt
    t = np.zeros(1, clrt.TRIANGLE_DTYPE)
    t["v1"]["position"][0, :3] = p1
    t["v2"]["position"][0, :3] = p2
    t["v3"]["position"][0, :3] = p3
    return t


def _rt(L, org, d, tri, t_in=1e5):
    o = (ctypes.c_float * 3)(*org)
    dd = (ctypes.c_float * 3)(*d)
    out = ctypes.c_float()
    hit = L.oracle_ray_triangle(o, dd, tri.ctypes.data, t_in, ctypes.byref(out))
    return hit, out.value


def test_ray_triangle_cases(oracle_mod):
    """Hand-built Moller-Trumbore cases (kernel_bvh.cl:98-153)."""
    L = oracle_mod.lib()
    front = _tri((-1, -1, 0), (1, -1, 0), (0, 1, 0))      # CCW seen from +z
    hit, t = _rt(L, (0, 0, 5), (0, 0, -1), front)
    assert hit == 1 and t == 5.0
    hit, _ = _rt(L, (0, 0, -5), (0, 0, 1), front)           # back face: det < 1e-8 -> culled
    assert hit == 0
    hit, _ = _rt(L, (0, 0, 5), (1, 0, 0), front)            # parallel: det == 0
    assert hit == 0
    hit, t = _rt(L, (0, 0, -5), (0, 0, 1), _tri((-1, -1, 0), (0, 1, 0), (1, -1, 0)))
    assert hit == 1 and t == 5.0
    # negative t is accepted (no t > 0 test, kernel_bvh.cl:140)
    hit, t = _rt(L, (0, 0, 5), (0, 0, 1), _tri((-1, -1, 0), (0, 1, 0), (1, -1, 0)))
    assert hit == 1 and t == -5.0
    # t must beat the current closest strictly
    hit, _ = _rt(L, (0, 0, 5), (0, 0, -1), front, t_in=5.0)
    assert hit == 0
    # outside the edge
    hit, _ = _rt(L, (3, 0, 5), (0, 0, -1), front)
    assert hit == 0


def test_ray_bounds_cases(oracle_mod):
    """Slab test with precomputed sign and 0*inf NaNs (kernel_bvh.cl:156-169)."""
    L = oracle_mod.lib()
    box = _node((-1, -1, -1), (1, 1, 1))
    def rb(o, d, t=1e5):
        return L.oracle_ray_bounds((ctypes.c_float * 3)(*o), (ctypes.c_float * 3)(*d), box.ctypes.data, t)
    assert rb((0, 0, -5), (0, 0, 1)) == 1
    assert rb((0, 0, 5), (0, 0, 1)) == 0          # box behind the ray (t0 clamps at 0)
    assert rb((0, 0, 0), (0, 0, 1)) == 1          # origin inside
    assert rb((0, 0, -5), (0, 0, 1), 3.0) == 0    # beyond current closest t
    assert rb((1, 0, -5), (0, 0, 1)) == 1         # grazing the x = 1 face: (1-1)*inf = NaN loses
    assert rb((2, 0, -5), (0, 0, 1)) == 0
    assert rb((0, 0, -5), (0, 0, 1), -1.0) == 0   # a negative closest t prunes everything


# Probe values of the reference kernel on Cornell.
SURVEY_PROBES = [
    # (W, H, bounces, hits, zero_pixels, node visits/ray, tri tests/ray, rays/sample)
    (512, 512, 1, 203790, 84828, 12.40, 3.91, 1.0),
    (1920, 1080, 1, 906676, None, 7.41, 2.20, 1.0),
    (512, 512, 9, None, None, 16.73, 5.83, 4.11),
]


@pytest.mark.parametrize("W,H,lb,hits,zeros,visits,tests,rps", SURVEY_PROBES)
def test_oracle_matches_survey_probe_counts(cornell, oracle_mod, W, H, lb, hits, zeros, visits, tests, rps):
    res, ids, _, c = oracle_mod.render(cornell, W, H, frame_count=1, light_bounces=lb, want_hits=True)
    if hits is not None:
        assert int((ids >= 0).sum()) == hits
    if zeros is not None:
        assert int((res[:, :3].sum(1) == 0).sum()) == zeros
    assert c["node_visits"] / c["rays"] == pytest.approx(visits, abs=0.005)
    assert c["tri_tests"] / c["rays"] == pytest.approx(tests, abs=0.005)
    assert c["rays"] / (W * H) == pytest.approx(rps, abs=0.005)


def test_oracle_threads_deterministic(cornell, oracle_mod):
    a, ia, ta, ca = oracle_mod.render(cornell, 96, 64, light_bounces=9, want_hits=True, threads=1)
    b, ib, tb, cb = oracle_mod.render(cornell, 96, 64, light_bounces=9, want_hits=True, threads=7)
    assert a.tobytes() == b.tobytes() and ia.tobytes() == ib.tobytes() and ca == cb
