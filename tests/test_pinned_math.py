"""GPU: the pinned math policy's device builtins (rtDiagPinnedMath, the functions KernelEntry's
pinned mode runs) against the CPU definition of the same semantics (include/rt_pinned_math.h).

The pinned `/`, reciprocal, sqrt and normalize's 1/sqrt are IEEE correctly rounded operations; on
the GPU the reciprocal is the hardware approximation plus one fma Newton step, which equals the
IEEE quotient for every float with an exponent field in [2, 251] (exhaustively,
scripts/probes/pinned_fast_probe.hip, profiles/r06/pinned_fast_probe_v1.txt); other operands take
the IEEE division.  numpy's float32 arithmetic is the reference here (IEEE, correctly rounded);
pow/sin/cos are compared with the C oracle's pm_pow/pm_sin/pm_cos (the same header for gcc).
"""
import numpy as np
import pytest

F32 = np.float32


def _specials():
    bits = [0x00000000, 0x80000000, 0x00000001, 0x80000001, 0x007fffff, 0x00800000, 0x00ffffff,
            0x01000000, 0x01000001, 0x017fffff, 0x3f800000, 0xbf800000, 0x3f7fffff, 0x3f800001,
            0x7e7fffff, 0x7e800000, 0x7effffff, 0x7f000000, 0x7f7fffff, 0xff7fffff, 0x7f800000,
            0xff800000, 0x7fc00000, 0x00400000, 0x5f000000, 0x20000000, 0x1f800000, 0x7dffffff]
    return np.array(bits, np.uint32).view(np.float32)


def _same(a, b):
    """bit equality, any NaN equal to any NaN"""
    a, b = np.asarray(a, F32), np.asarray(b, F32)
    return (a.view(np.uint32) == b.view(np.uint32)) | (np.isnan(a) & np.isnan(b))


@pytest.fixture(scope="module")
def rng():
    return np.random.default_rng(20261018)


def _random_floats(rng, n):
    x = rng.integers(0, 2**32, size=n, dtype=np.uint64).astype(np.uint32).view(np.float32)
    return np.concatenate([x, _specials()])


@pytest.mark.gpu
def test_pinned_reciprocal_is_the_ieee_quotient(rng):
    from clrt import _native as N
    # random bit patterns (every exponent), near-one significands, all-ones significands
    x = _random_floats(rng, 1 << 20)
    e = rng.integers(0, 255, size=1 << 16).astype(np.uint32)
    x = np.concatenate([x, ((e << 23) | 0x7fffff).view(np.float32), ((e << 23) | 1).view(np.float32)])
    with np.errstate(all="ignore"):
        want = F32(1.0) / x
    got = N.pinned_math("rcp", x)
    bad = ~_same(got, want)
    assert not bad.any(), f"{bad.sum()} reciprocals differ, e.g. x={x[bad][:4].view(np.uint32)}"


@pytest.mark.gpu
def test_pinned_division_sqrt_rsqrt(rng):
    from clrt import _native as N
    a = _random_floats(rng, 1 << 18)
    b = _random_floats(rng, 1 << 18)
    with np.errstate(all="ignore"):
        assert _same(N.pinned_math("div", a, b), a / b).all()
        s = np.abs(_random_floats(rng, 1 << 18))
        assert _same(N.pinned_math("sqrt", s), np.sqrt(s)).all()
        # normalize's 1/sqrt(d): d >= 2^-126 and finite (normalize rescales other d first)
        d = s[np.isfinite(s) & (s >= F32(2.0**-126))]
        assert _same(N.pinned_math("rsqrt", d), F32(1.0) / np.sqrt(d)).all()


@pytest.mark.gpu
def test_pinned_transcendentals_match_the_c_oracle(rng):
    import oracle
    from clrt import _native as N
    L = oracle.lib()
    x = np.concatenate([rng.uniform(0, 2 * np.pi, 4096), rng.uniform(-100, 100, 1024)]).astype(F32)
    assert _same(N.pinned_math("sin", x), [L.oracle_sin(float(v)) for v in x]).all()
    assert _same(N.pinned_math("cos", x), [L.oracle_cos(float(v)) for v in x]).all()
    base = rng.uniform(0, 4, 4096).astype(F32)
    ex = rng.choice(np.array([2.2, 0.454545, 0.45454545, 0.25, 1.0 / 3.0, 7.5], F32), 4096)
    assert _same(N.pinned_math("pow", base, ex), [L.oracle_pow(float(p), float(q)) for p, q in zip(base, ex)]).all()


def test_pinned_math_entry_point_refuses_bad_arguments():
    """host-side argument checks (no GPU needed for these)"""
    import ctypes
    from clrt import _native as N
    lib = N.hip_lib()
    a = np.ones(4, F32)
    out = np.empty(4, F32)
    assert lib.rtDiagPinnedMath(0, 99, a.ctypes.data, None, out.ctypes.data, 4) == -30
    assert lib.rtDiagPinnedMath(0, 1, a.ctypes.data, None, out.ctypes.data, 4) == -30  # div without b
    assert lib.rtDiagPinnedMath(0, 0, None, None, out.ctypes.data, 4) == -30
    assert lib.rtDiagPinnedMath(0, 0, a.ctypes.data, None, out.ctypes.data, ctypes.c_size_t(0)) == 0
