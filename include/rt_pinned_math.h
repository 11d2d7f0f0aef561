/*
 * rt_pinned_math.h -- the pinned builtin semantics of the raytracer hot path.
 *
 * The reference kernel (/root/reference/kernel_bvh.cl) calls OpenCL builtins whose
 * rounding is implementation-defined: dot/cross/normalize (:44, :86-89, :112-146, :400),
 * sqrt (:83, :232, :334), pow (:224, :231, :275, :407, :412, :450), sin/cos (:89, :238),
 * tan (:392), max/min (:158-165, :251-252, :284-289, :320-341, :383).  Bit-exact hit IDs
 * are impossible unless every implementation that claims parity uses ONE definition of
 * those builtins (hard parts 1 and 2).  This header IS that
 * definition ("pinned" math mode):
 *
 *   - fp32 arithmetic with no contraction (build with -ffp-contract=off);
 *   - + - * / and sqrt are IEEE correctly rounded (fp32), as are the fp64 ops used below;
 *   - dot(a,b)   = (a.x*b.x + a.y*b.y) + a.z*b.z          (left to right, no fma)
 *   - cross(a,b) = (a.y*b.z - a.z*b.y, a.z*b.x - a.x*b.z, a.x*b.y - a.y*b.x)
 *   - normalize  = v * rsqrt(dot(v,v)) with the scaling guards OpenCL libraries use
 *                  (all-zero -> v; tiny -> prescale 2^86; inf -> prescale 2^-66),
 *                  rsqrt(d) = 1.0f / sqrtf(d)  (two correctly rounded fp32 ops)
 *   - max/min    = OpenCL fmax/fmin for NaN (the non-NaN operand wins) and the OpenCL
 *                  common-function tie rule otherwise (max: y if x < y else x;
 *                  min: y if y < x else x) -- this fixes the sign of zero results;
 *   - pow(x, 2.0f) written with a literal 2 (kernel_bvh.cl:224, :275) = x*x, the
 *                  correctly rounded square (LLVM's generic and AMDGPU libcall
 *                  simplifiers both fold it so; the AMD OpenCL build of the reference
 *                  does, see its IR);
 *   - sin/cos/tan/pow = fp64 evaluation (Cody-Waite reduction, fdlibm-style kernels,
 *                  atanh-series log, Taylor exp2) rounded once to fp32.  Results are
 *                  faithful (correctly rounded except in rare near-midpoint cases) and,
 *                  more importantly, identical on x86-64 (gcc) and gfx950 (hipcc),
 *                  because only IEEE + - * / and fma appear.
 *
 * Consumers: the HIP kernels (product, "pinned" math mode) and the CPU oracle
 * (test infrastructure).  Both must compile this with -ffp-contract=off.
 */
#ifndef RT_PINNED_MATH_H
#define RT_PINNED_MATH_H

#include <stdint.h>

#if defined(__HIPCC__)
#define RT_PM_FN __host__ __device__ static inline
/* the fp64 transcendentals stay out of line in device code: six inlined pow expansions in
 * the pixel-accumulation step would otherwise overlap and cost the kernel ~30 VGPRs */
#ifndef RT_PM_HEAVY
#define RT_PM_HEAVY __attribute__((noinline)) __host__ __device__ static
#endif
#else
#define RT_PM_FN static inline
#define RT_PM_HEAVY static inline
#endif

#if defined(__HIPCC__) || defined(__clang__)
#pragma clang fp contract(off)
#endif

#ifdef __cplusplus
extern "C++" {
#endif

/* ---- bit casts ------------------------------------------------------------------ */
RT_PM_FN uint32_t pm_f2u(float f) { union { float f; uint32_t u; } c; c.f = f; return c.u; }
RT_PM_FN float pm_u2f(uint32_t u) { union { float f; uint32_t u; } c; c.u = u; return c.f; }
RT_PM_FN uint64_t pm_d2u(double d) { union { double d; uint64_t u; } c; c.d = d; return c.u; }
RT_PM_FN double pm_u2d(uint64_t u) { union { double d; uint64_t u; } c; c.u = u; return c.d; }

RT_PM_FN int pm_isnan(float x) { return (pm_f2u(x) & 0x7fffffffu) > 0x7f800000u; }
RT_PM_FN int pm_isinf(float x) { return (pm_f2u(x) & 0x7fffffffu) == 0x7f800000u; }
RT_PM_FN float pm_fabs(float x) { return pm_u2f(pm_f2u(x) & 0x7fffffffu); }
RT_PM_FN float pm_copysign(float mag, float sgn) {
    return pm_u2f((pm_f2u(mag) & 0x7fffffffu) | (pm_f2u(sgn) & 0x80000000u));
}

/* ---- fp32 primitives -------------------------------------------------------------- */
/* The compilers lower these to correctly rounded instructions (x86 sqrtss; the gfx950
 * v_sqrt_f32 + fixup sequence that hipcc emits by default). */
RT_PM_FN float pm_sqrt(float x) { return __builtin_sqrtf(x); }
RT_PM_FN double pm_fma_d(double a, double b, double c) { return __builtin_fma(a, b, c); }

/* OpenCL max/min, pinned (see header comment). */
RT_PM_FN float pm_max(float x, float y) {
    if (pm_isnan(x)) return y;
    if (pm_isnan(y)) return x;
    return (x < y) ? y : x;
}
RT_PM_FN float pm_min(float x, float y) {
    if (pm_isnan(x)) return y;
    if (pm_isnan(y)) return x;
    return (y < x) ? y : x;
}

RT_PM_FN float pm_rsqrt(float d) { return 1.0f / pm_sqrt(d); }

/* pow(x, 2.0f) with a literal exponent */
RT_PM_FN float pm_sq(float x) { return x * x; }

/* ---- fp64 helpers ------------------------------------------------------------------ */
/* round-to-nearest-even integer value of |x| < 2^51 via the 1.5*2^52 shifter */
RT_PM_FN double pm_rint_d(double x) {
    const double shifter = 6755399441055744.0; /* 1.5 * 2^52 */
    double t = x + shifter;
    return t - shifter;
}

/* 2^n for integer n in [-1074, 1023], exact */
RT_PM_FN double pm_pow2i(int n) {
    if (n >= -1022) return pm_u2d((uint64_t)(n + 1023) << 52);
    return pm_u2d((uint64_t)1 << (n + 1074)); /* subnormal powers of two */
}

/* sin/cos kernels on |r| <= pi/4 (fdlibm __kernel_sin / __kernel_cos coefficients) */
RT_PM_FN double pm_ksin(double r) {
    const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
                 S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
                 S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
    double z = r * r;
    double p = pm_fma_d(z, S6, S5);
    p = pm_fma_d(z, p, S4);
    p = pm_fma_d(z, p, S3);
    p = pm_fma_d(z, p, S2);
    p = pm_fma_d(z, p, S1);
    return pm_fma_d(r * z, p, r);
}
RT_PM_FN double pm_kcos(double r) {
    const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
                 C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
                 C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
    double z = r * r;
    double p = pm_fma_d(z, C6, C5);
    p = pm_fma_d(z, p, C4);
    p = pm_fma_d(z, p, C3);
    p = pm_fma_d(z, p, C2);
    p = pm_fma_d(z, p, C1);
    /* 1 - z/2 + z^2 * p */
    return pm_fma_d(z * z, p, pm_fma_d(-0.5, z, 1.0));
}

/* Cody-Waite reduction x = k*pi/2 + r, |r| <= ~pi/4; accurate for |x| < 2^20, and
 * deterministic (if inaccurate) beyond. Returns quadrant k mod 4. */
RT_PM_FN int pm_reduce_pio2(double x, double* r) {
    const double invpio2 = 6.36619772367581382433e-01;
    const double pio2_1 = 1.57079632673412561417e+00;  /* first 33 bits of pi/2 */
    const double pio2_1t = 6.07710050650619224932e-11; /* pi/2 - pio2_1 */
    double k = pm_rint_d(x * invpio2);
    double rr = pm_fma_d(-k, pio2_1, x);
    rr = pm_fma_d(-k, pio2_1t, rr);
    *r = rr;
    long long ki = (long long)k;
    return (int)(ki & 3);
}

RT_PM_FN double pm_sin_d(double x) {
    double r;
    int q = pm_reduce_pio2(x, &r);
    switch (q) {
        case 0: return pm_ksin(r);
        case 1: return pm_kcos(r);
        case 2: return -pm_ksin(r);
        default: return -pm_kcos(r);
    }
}
RT_PM_FN double pm_cos_d(double x) {
    double r;
    int q = pm_reduce_pio2(x, &r);
    switch (q) {
        case 0: return pm_kcos(r);
        case 1: return -pm_ksin(r);
        case 2: return -pm_kcos(r);
        default: return pm_ksin(r);
    }
}

RT_PM_FN float pm_sin(float x) {
    if (pm_isnan(x) || pm_isinf(x)) return pm_u2f(0x7fc00000u);
    return (float)pm_sin_d((double)x);
}
RT_PM_FN float pm_cos(float x) {
    if (pm_isnan(x) || pm_isinf(x)) return pm_u2f(0x7fc00000u);
    return (float)pm_cos_d((double)x);
}
/* sin and cos of one argument from one reduction: the same operations as pm_sin / pm_cos,
 * so the same bits, for half the reduction work */
RT_PM_FN void pm_sincos(float x, float* s, float* c) {
    if (pm_isnan(x) || pm_isinf(x)) {
        *s = *c = pm_u2f(0x7fc00000u);
        return;
    }
    double r;
    const int q = pm_reduce_pio2((double)x, &r);
    const double ks = pm_ksin(r), kc = pm_kcos(r);
    switch (q) {
        case 0: *s = (float)ks; *c = (float)kc; break;
        case 1: *s = (float)kc; *c = (float)(-ks); break;
        case 2: *s = (float)(-ks); *c = (float)(-kc); break;
        default: *s = (float)(-kc); *c = (float)ks; break;
    }
}
RT_PM_FN float pm_tan(float x) {
    if (pm_isnan(x) || pm_isinf(x)) return pm_u2f(0x7fc00000u);
    double xd = (double)x;
    return (float)(pm_sin_d(xd) / pm_cos_d(xd));
}

/* natural log of a positive finite double m in [sqrt(1/2), sqrt(2)): 2*atanh(s) */
RT_PM_FN double pm_log_mant(double m) {
    const double Lg1 = 6.666666666666735130e-01, Lg2 = 3.999999999940941908e-01,
                 Lg3 = 2.857142874366239149e-01, Lg4 = 2.222219843214978396e-01,
                 Lg5 = 1.818357216161805012e-01, Lg6 = 1.531383769920937332e-01,
                 Lg7 = 1.479819860511658591e-01;
    double f = m - 1.0;          /* exact (Sterbenz) */
    double s = f / (2.0 + f);
    double z = s * s;
    double R = pm_fma_d(z, Lg7, Lg6);
    R = pm_fma_d(z, R, Lg5);
    R = pm_fma_d(z, R, Lg4);
    R = pm_fma_d(z, R, Lg3);
    R = pm_fma_d(z, R, Lg2);
    R = pm_fma_d(z, R, Lg1);
    R = z * R;
    /* log(1+f) = f - hfsq + s*(hfsq + R), hfsq = f*f/2 (fdlibm form) */
    double hfsq = 0.5 * f * f;
    return f - (hfsq - s * (hfsq + R));
}

/* log2 of a positive finite float, in double */
RT_PM_FN double pm_log2_pos(float x) {
    const double invln2 = 1.44269504088896338700e+00;
    uint32_t u = pm_f2u(x);
    int e;
    double m;
    if (u < 0x00800000u) { /* subnormal: scale by 2^24 (exact) */
        double xd = (double)x * 16777216.0;
        uint64_t du = pm_d2u(xd);
        e = (int)((du >> 52) & 0x7ff) - 1023 - 24;
        m = pm_u2d((du & 0x000fffffffffffffull) | 0x3ff0000000000000ull);
    } else {
        e = (int)((u >> 23) & 0xff) - 127;
        m = pm_u2d(((uint64_t)(u & 0x007fffffu) << 29) | 0x3ff0000000000000ull);
    }
    if (m > 1.41421356237309504880) { m = m * 0.5; e += 1; }
    return (double)e + pm_log_mant(m) * invln2;
}

/* 2^z for |z| <= 1100, double result (may be 0/inf beyond the double range) */
RT_PM_FN double pm_exp2_d(double z) {
    const double ln2 = 6.93147180559945286227e-01;
    double n = pm_rint_d(z);
    double f = z - n;            /* exact, |f| <= 0.5 */
    double a = f * ln2;          /* |a| <= 0.347 */
    /* Taylor series of e^a to degree 13: truncation < 1e-18 */
    double p = 1.0 / 6227020800.0;                 /* 1/13! */
    p = pm_fma_d(p, a, 1.0 / 479001600.0);         /* 1/12! */
    p = pm_fma_d(p, a, 1.0 / 39916800.0);          /* 1/11! */
    p = pm_fma_d(p, a, 1.0 / 3628800.0);           /* 1/10! */
    p = pm_fma_d(p, a, 1.0 / 362880.0);
    p = pm_fma_d(p, a, 1.0 / 40320.0);
    p = pm_fma_d(p, a, 1.0 / 5040.0);
    p = pm_fma_d(p, a, 1.0 / 720.0);
    p = pm_fma_d(p, a, 1.0 / 120.0);
    p = pm_fma_d(p, a, 1.0 / 24.0);
    p = pm_fma_d(p, a, 1.0 / 6.0);
    p = pm_fma_d(p, a, 0.5);
    p = pm_fma_d(p, a, 1.0);
    p = pm_fma_d(p, a, 1.0);
    int ni = (int)n;
    int h = ni / 2;
    return (p * pm_pow2i(h)) * pm_pow2i(ni - h);
}

/* is the (finite) float y an integer? odd integer? */
RT_PM_FN int pm_is_int(float y) {
    float a = pm_fabs(y);
    if (a >= 8388608.0f) return 1;
    return (float)(int32_t)a == a;
}
RT_PM_FN int pm_is_odd_int(float y) {
    float a = pm_fabs(y);
    if (a >= 16777216.0f) return 0;
    if (!pm_is_int(y)) return 0;
    return ((int32_t)a & 1) != 0;
}

/* OpenCL/C99 pow special cases, then 2^(y*log2|x|) in fp64, rounded once.  pm_pow_body is the
 * definition; pm_pow the out-of-line copy most call sites use (same operations, same bits). */
RT_PM_FN float pm_pow_body(float x, float y) {
    const float qnan = pm_u2f(0x7fc00000u);
    if (y == 0.0f) return 1.0f;
    if (x == 1.0f) return 1.0f;
    if (pm_isnan(x) || pm_isnan(y)) return qnan;
    float ax = pm_fabs(x);
    int neg = pm_f2u(x) >> 31;
    if (pm_isinf(y)) {
        if (ax == 1.0f) return 1.0f;
        int big = ax > 1.0f;
        if (y > 0.0f) return big ? pm_u2f(0x7f800000u) : 0.0f;
        return big ? 0.0f : pm_u2f(0x7f800000u);
    }
    int yodd = pm_is_odd_int(y);
    if (ax == 0.0f) {
        float r = (y < 0.0f) ? pm_u2f(0x7f800000u) : 0.0f;
        return (neg && yodd) ? -r : r;
    }
    if (pm_isinf(x)) {
        float r = (y < 0.0f) ? 0.0f : pm_u2f(0x7f800000u);
        return (neg && yodd) ? -r : r;
    }
    if (neg && !pm_is_int(y)) return qnan;
    double z = (double)y * pm_log2_pos(ax);
    float r;
    if (z > 1100.0) r = pm_u2f(0x7f800000u);
    else if (z < -1100.0) r = 0.0f;
    else r = (float)pm_exp2_d(z);
    return (neg && yodd) ? -r : r;
}
RT_PM_HEAVY float pm_pow(float x, float y) { return pm_pow_body(x, y); }

#ifdef __cplusplus
}
#endif

#endif /* RT_PINNED_MATH_H */
