// rt_math.hpp -- float3 algebra and the two math policies of the HIP hot path.
//
// MathPinned   : the pinned builtin semantics of include/rt_pinned_math.h (identical,
//                bit for bit, to the CPU oracle; no hardware approximations).
// MathDeviceLib: the semantics the AMD OpenCL toolchain gives the reference kernel on
//                this GPU (device library opencl.bc / ocml.bc): dot/cross with fma
//                (opencl.bc _Z3dotDv3_fS_, _Z5crossDv3_fS_), normalize = v * rsqrt(d)
//                with the hardware-rsq based __ocml_rsqrt_f32 (_Z9normalizeDv3_f),
//                pow/sin/cos/tan = __ocml_*_f32, max/min = llvm.maxnum/minnum.  This is
//                the mode that is checked against the reference kernel itself, built by
//                the image's OpenCL compiler and run through the OpenCL runtime
//                (oracle/_ref, tests/test_ref_opencl.py) with contraction off and
//                correctly-rounded / and sqrt (the reference's `strict` build).
// MathShipped  : devicelib builtins plus the two things the AMD OpenCL compiler does to the
//                reference by default (clBuildProgram(" -I . "), CLutils.cpp:52-66): FP
//                contraction within an expression (fp-contract=on: a*b + c -> fma at exactly
//                the reference's source sites, `madd` below) and the 2.5-ulp `/` and 3-ulp
//                sqrt of OpenCL C (no -cl-fp32-correctly-rounded-divide-sqrt).  The latter is
//                a per-translation-unit setting, so this policy is instantiated only in
//                rt_kernels_shipped.hip, compiled with -fno-hip-fp32-correctly-rounded-divide-sqrt.
//
// Everything here is compiled with -ffp-contract=off: each + - * / below is one IEEE
// operation, in the association order the reference source spells out.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/rt_pinned_math.h"

#pragma clang fp contract(off)

namespace rtk {

struct F3 {
    float x, y, z;
};

__device__ __forceinline__ F3 f3(float x, float y, float z) { return F3{x, y, z}; }
__device__ __forceinline__ F3 f3s(float s) { return F3{s, s, s}; }
__device__ __forceinline__ F3 operator+(F3 a, F3 b) { return F3{a.x + b.x, a.y + b.y, a.z + b.z}; }
__device__ __forceinline__ F3 operator-(F3 a, F3 b) { return F3{a.x - b.x, a.y - b.y, a.z - b.z}; }
__device__ __forceinline__ F3 operator*(F3 a, F3 b) { return F3{a.x * b.x, a.y * b.y, a.z * b.z}; }
__device__ __forceinline__ F3 operator*(F3 a, float s) { return F3{a.x * s, a.y * s, a.z * s}; }
__device__ __forceinline__ F3 operator/(F3 a, float s) { return F3{a.x / s, a.y / s, a.z / s}; }
__device__ __forceinline__ F3 operator-(F3 a) { return F3{-a.x, -a.y, -a.z}; }

// ---------------------------------------------------------------------------------------
// RT_PINNED_DIAG_* (diagnostic variant builds only, scripts/build_variant.sh): swap one pinned
// operation for the hardware / device-library form to price it -- NOT bit-exact, never shipped
#ifndef RT_PINNED_DIAG_DIV
#define RT_PINNED_DIAG_DIV 0
#endif
#ifndef RT_PINNED_DIAG_SQRT
#define RT_PINNED_DIAG_SQRT 0
#endif
#ifndef RT_PINNED_DIAG_POW
#define RT_PINNED_DIAG_POW 0
#endif
#ifndef RT_PINNED_DIAG_TRIG
#define RT_PINNED_DIAG_TRIG 0
#endif
struct MathPinned {
    static constexpr int kId = 0;
    static constexpr bool kContract = false;
    // the reference's `/` and sqrt: IEEE, correctly rounded
    // 1.0f / x, correctly rounded, as the hardware reciprocal plus one Newton step (two fma): for
    // every float with an exponent field in [2, 251] this IS the IEEE quotient, bit for bit
    // (scripts/probes/pinned_fast_probe.hip, exhaustive: profiles/r06/pinned_fast_probe_v1.txt) --
    // 6 VALU against the 11 of the IEEE division sequence.  Other operands (0, denormals, |x| >=
    // 2^125, inf, NaN) take the IEEE division; the branch is wave-uniform.
    __device__ __forceinline__ static float rcp_fast(float x) {
        const float y = __builtin_amdgcn_rcpf(x);
        return __builtin_fmaf(__builtin_fmaf(-x, y, 1.0f), y, y);
    }
#if RT_PINNED_DIAG_DIV
    __device__ __forceinline__ static float rcp(float x) { return __builtin_amdgcn_rcpf(x); }
    __device__ __forceinline__ static float div(float a, float b) { return a * __builtin_amdgcn_rcpf(b); }
#else
    __device__ __forceinline__ static float rcp(float x) {
        const float r = rcp_fast(x);
        const bool ok = (__float_as_uint(x) & 0x7fffffffu) - 0x01000000u < 0x7d000000u;
        if (__builtin_expect(__ballot(!ok) != 0ull, 0)) return ok ? r : 1.0f / x;
        return r;
    }
    __device__ __forceinline__ static float div(float a, float b) { return a / b; }
#endif
#if RT_PINNED_DIAG_SQRT
    __device__ __forceinline__ static float sqrt(float x) { return __builtin_amdgcn_sqrtf(x); }
    __device__ __forceinline__ static float rsqrt(float d) { return __builtin_amdgcn_rsqf(d); }
#else
    // sqrt(x), correctly rounded, as the hardware reciprocal square root plus one Markstein step
    // (s = x*r, h = r/2, s + (x - s*s)*h with fma): for every float with an exponent field in
    // [25, 254] this IS the IEEE square root, bit for bit (scripts/probes/pinned_fast_probe2.hip,
    // exhaustive: profiles/r06/pinned_fast_probe_v2.txt) -- 5 VALU against the 14 of the IEEE
    // sequence.  Other operands (x < 2^-102, negative, 0, inf, NaN) take the IEEE square root.
    __device__ __forceinline__ static float sqrt_fast(float x) {
        const float r = __builtin_amdgcn_rsqf(x);
        const float s = x * r, h = 0.5f * r;
        return __builtin_fmaf(__builtin_fmaf(-s, s, x), h, s);
    }
    __device__ __forceinline__ static float sqrt(float x) {
        const float f = sqrt_fast(x);
        const bool ok = __float_as_uint(x) - 0x0c800000u < 0x73000000u;  // exponent field in [25, 254]
        if (__builtin_expect(__ballot(!ok) != 0ull, 0)) return ok ? f : __builtin_sqrtf(x);
        return f;
    }
    // normalize's 1/sqrt(d): two correctly rounded operations (rt_pinned_math.h pm_rsqrt), here the
    // two exact sequences above; d >= 2^-126 and finite there (normalize rescales other d first)
    __device__ __forceinline__ static float rsqrt(float d) {
        const float f = rcp_fast(sqrt_fast(d));  // (sqrt_fast(d) in [2^-51, 2^64]: rcp_fast's range)
        const bool ok = __float_as_uint(d) - 0x0c800000u < 0x73000000u;
        if (__builtin_expect(__ballot(!ok) != 0ull, 0)) return ok ? f : pm_rsqrt(d);
        return f;
    }
#endif
    __device__ __forceinline__ static float dot(F3 a, F3 b) {
        return (a.x * b.x + a.y * b.y) + a.z * b.z;
    }
    __device__ __forceinline__ static F3 cross(F3 a, F3 b) {
        return F3{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
    }
#if RT_PINNED_DIAG_POW
    __device__ __forceinline__ static float pow(float x, float y) { return ::powf(x, y); }
#else
    // (out of line; inlining the BRDF's call into the render costs 13 %: profiles/r06/pinned_ab.txt)
    __device__ __forceinline__ static float pow(float x, float y) { return pm_pow(x, y); }
#endif
    // pow(x, 2.0f) call sites of the reference (kernel_bvh.cl:224, :275): pinned as the
    // exact square, as LLVM's libcall simplifiers fold it (rt_pinned_math.h)
    __device__ __forceinline__ static float pow2(float x) { return pm_sq(x); }
#if RT_PINNED_DIAG_TRIG
    __device__ __forceinline__ static float sin(float x) { return ::sinf(x); }
    __device__ __forceinline__ static float cos(float x) { return ::cosf(x); }
    __device__ __forceinline__ static void sincos(float x, float& s, float& c) { ::sincosf(x, &s, &c); }
#else
    __device__ __forceinline__ static float sin(float x) { return pm_sin(x); }
    __device__ __forceinline__ static float cos(float x) { return pm_cos(x); }
    __device__ __forceinline__ static void sincos(float x, float& s, float& c) { pm_sincos(x, &s, &c); }
#endif
    __device__ __forceinline__ static float tan(float x) { return pm_tan(x); }
    __device__ __forceinline__ static float max(float x, float y) { return pm_max(x, y); }
    __device__ __forceinline__ static float min(float x, float y) { return pm_min(x, y); }
};

struct MathDeviceLib {
    static constexpr int kId = 1;
    static constexpr bool kContract = false;
    // the reference's `/` and sqrt: IEEE, correctly rounded
    __device__ __forceinline__ static float rcp(float x) { return 1.0f / x; }
    __device__ __forceinline__ static float div(float a, float b) { return a / b; }
    __device__ __forceinline__ static float sqrt(float x) { return __builtin_sqrtf(x); }
    // opencl.bc: dot = fma(z, z', fma(y, y', x*x'))
    __device__ __forceinline__ static float dot(F3 a, F3 b) {
        return __builtin_fmaf(a.z, b.z, __builtin_fmaf(a.y, b.y, a.x * b.x));
    }
    // opencl.bc: cross.x = fma(a.y, b.z, b.y * -a.z), ...
    __device__ __forceinline__ static F3 cross(F3 a, F3 b) {
        return F3{__builtin_fmaf(a.y, b.z, b.y * -a.z), __builtin_fmaf(a.z, b.x, b.z * -a.x),
                  __builtin_fmaf(a.x, b.y, b.x * -a.y)};
    }
    __device__ __forceinline__ static float rsqrt(float d) { return ::rsqrtf(d); }
    __device__ __forceinline__ static float pow(float x, float y) { return ::powf(x, y); }
    // the AMD OpenCL compiler folds pow(x, 2.0f) to x*x (AMDGPU libcall simplification;
    // visible in the reference's IR: DistributionGGX, SampleSpecular)
    __device__ __forceinline__ static float pow2(float x) { return x * x; }
    __device__ __forceinline__ static float sin(float x) { return ::sinf(x); }
    __device__ __forceinline__ static float cos(float x) { return ::cosf(x); }
    // ocml's sincos runs sin's and cos's reduction and polynomials once: same bits as the
    // two separate builtins the reference calls (checked against the reference kernel)
    __device__ __forceinline__ static void sincos(float x, float& s, float& c) { ::sincosf(x, &s, &c); }
    __device__ __forceinline__ static float tan(float x) { return ::tanf(x); }
    __device__ __forceinline__ static float max(float x, float y) { return __builtin_fmaxf(x, y); }
    __device__ __forceinline__ static float min(float x, float y) { return __builtin_fminf(x, y); }
};

struct MathShipped : MathDeviceLib {
    static constexpr int kId = 2;
    static constexpr bool kContract = true;
    // OpenCL C's 2.5-ulp `/` and 3-ulp sqrt as the AMDGPU backend expands them with IEEE
    // f32 denormals (AMDGPUCodeGenPrepare; read off the reference's shipped code object):
    //   1/x  = ldexp(rcp(frexp_mant(x)), -frexp_exp(x))
    //   a/b  = ldexp(frexp_mant(a) * rcp(frexp_mant(b)), frexp_exp(a) - frexp_exp(b))
    //   sqrt = x < 2^-126 ? ldexp(v_sqrt(ldexp(x, 32)), -16) : v_sqrt(x)
    // Spelled out with the hardware builtins rather than left to !fpmath metadata, which the
    // optimizer drops when it hoists a loop-invariant division (the camera's 1/W, 1/H, W/H).
    __device__ __forceinline__ static float rcp(float x) {
        return __builtin_amdgcn_ldexpf(__builtin_amdgcn_rcpf(__builtin_amdgcn_frexp_mantf(x)),
                                       -__builtin_amdgcn_frexp_expf(x));
    }
    __device__ __forceinline__ static float div(float a, float b) {
        const float r = __builtin_amdgcn_rcpf(__builtin_amdgcn_frexp_mantf(b));
        return __builtin_amdgcn_ldexpf(__builtin_amdgcn_frexp_mantf(a) * r,
                                       __builtin_amdgcn_frexp_expf(a) - __builtin_amdgcn_frexp_expf(b));
    }
    __device__ __forceinline__ static float sqrt(float x) {
        const bool scale = x < 0x1p-126f;
        const float r = __builtin_amdgcn_sqrtf(__builtin_amdgcn_ldexpf(x, scale ? 32 : 0));
        return __builtin_amdgcn_ldexpf(r, scale ? -16 : 0);
    }
};

// A source-level `a * b + c` of the reference (one expression).  Under fp-contract=on clang
// turns it into llvm.fmuladd (an fma on gfx950); where both operands of the + are products
// the LEFT one is fused: `p*q + r*s` -> fma(p, q, r*s).  Callers spell each site in that form.
template <class M>
__device__ __forceinline__ float madd(float a, float b, float c) {
    if (M::kContract) return __builtin_fmaf(a, b, c);
    return a * b + c;
}
template <class M>
__device__ __forceinline__ F3 madd(F3 a, F3 b, F3 c) {
    return F3{madd<M>(a.x, b.x, c.x), madd<M>(a.y, b.y, c.y), madd<M>(a.z, b.z, c.z)};
}
template <class M>
__device__ __forceinline__ F3 madd(F3 a, float b, F3 c) {
    return F3{madd<M>(a.x, b, c.x), madd<M>(a.y, b, c.y), madd<M>(a.z, b, c.z)};
}

// normalize with the guard structure shared by both policies (see rt_pinned_math.h)
template <class M>
__device__ __forceinline__ F3 normalize(F3 v) {
    if (v.x == 0.0f && v.y == 0.0f && v.z == 0.0f) return v;
    float d = M::dot(v, v);
    if (d < 0x1p-126f) {
        v = v * 0x1p86f;
        d = M::dot(v, v);
    } else if (pm_isinf(d)) {
        v = v * 0x1p-66f;
        d = M::dot(v, v);
        if (pm_isinf(d)) {
            v = F3{pm_copysign(pm_isinf(v.x) ? 1.0f : 0.0f, v.x),
                   pm_copysign(pm_isinf(v.y) ? 1.0f : 0.0f, v.y),
                   pm_copysign(pm_isinf(v.z) ? 1.0f : 0.0f, v.z)};
            d = M::dot(v, v);
        }
    }
    return v * M::rsqrt(d);
}

}  // namespace rtk
