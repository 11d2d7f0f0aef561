// Probe (not product code): which fp32 sequences built on the hardware approximations give the
// correctly rounded 1/x, sqrt(x) and a/b of IEEE arithmetic, bit for bit?  Exhaustive over every
// float for 1/x and sqrt, random + structured pairs for a/b.  Counts mismatches against the
// compiler's correctly rounded forms (hipcc's default -fhip-fp32-correctly-rounded-divide-sqrt).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#pragma clang fp contract(off)

__device__ __forceinline__ float rcp_nr(float x) {  // R1
    const float y = __builtin_amdgcn_rcpf(x);
    const float e = __builtin_fmaf(-x, y, 1.0f);
    return __builtin_fmaf(e, y, y);
}
__device__ __forceinline__ float sqrt_res(float x) {  // S1: v_sqrt + residual +-1ulp
    const float s = __builtin_amdgcn_sqrtf(x);
    const float lo = __uint_as_float(__float_as_uint(s) - 1u), hi = __uint_as_float(__float_as_uint(s) + 1u);
    const float rl = __builtin_fmaf(-lo, s, x), rh = __builtin_fmaf(-hi, s, x);
    float r = rl <= 0.0f ? lo : s;
    r = rh > 0.0f ? hi : r;
    return r;
}
__device__ __forceinline__ float sqrt_rsq(float x) {  // S2: rsq + one Markstein step
    const float r = __builtin_amdgcn_rsqf(x);
    const float s = x * r, h = 0.5f * r;
    const float e = __builtin_fmaf(-s, s, x);
    return __builtin_fmaf(e, h, s);
}
__device__ __forceinline__ float sqrt_v(float x) {  // S3: bare v_sqrt
    return __builtin_amdgcn_sqrtf(x);
}
__device__ __forceinline__ float div_m(float a, float b) {  // D1: Markstein with the CR reciprocal
    const float y = rcp_nr(b);
    const float q = a * y;
    const float r = __builtin_fmaf(-b, q, a);
    return __builtin_fmaf(r, y, q);
}

__device__ __forceinline__ bool in_range(float x, uint32_t lo, uint32_t hi) {
    const uint32_t e = (__float_as_uint(x) >> 23) & 0xffu;
    return e >= lo && e <= hi;
}

__global__ void unary(uint64_t base, unsigned long long* bad, unsigned long long* first) {
    const uint64_t u64 = base + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t u = (uint32_t)u64;
    const float x = __uint_as_float(u);
    const float rr = 1.0f / x;
    if (in_range(x, 2u, 251u) && __float_as_uint(rcp_nr(x)) != __float_as_uint(rr)) {
        if (atomicAdd(&bad[0], 1ull) < 4) first[0 + (bad[0] & 3)] = u;
    }
    if (x > 0.0f) {
        const float sr = __builtin_sqrtf(x);
        if (in_range(x, 1u, 254u) && __float_as_uint(sqrt_res(x)) != __float_as_uint(sr)) {
            if (atomicAdd(&bad[1], 1ull) < 4) first[4 + (bad[1] & 3)] = u;
        }
        if (in_range(x, 2u, 252u) && __float_as_uint(sqrt_rsq(x)) != __float_as_uint(sr)) {
            if (atomicAdd(&bad[2], 1ull) < 4) first[8 + (bad[2] & 3)] = u;
        }
        if (in_range(x, 1u, 254u) && __float_as_uint(sqrt_v(x)) != __float_as_uint(sr)) atomicAdd(&bad[3], 1ull);
        // 1/sqrt(x) as two correctly rounded operations (pm_rsqrt)
        const float rs = 1.0f / sr;
        if (in_range(x, 2u, 252u) && __float_as_uint(rcp_nr(sqrt_res(x))) != __float_as_uint(rs)) atomicAdd(&bad[4], 1ull);
    }
}

__device__ __forceinline__ uint32_t mix(uint64_t z) {
    z += 0x9e3779b97f4a7c15ull;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return (uint32_t)(z ^ (z >> 31));
}

__global__ void binary(uint64_t base, int mode, unsigned long long* bad, unsigned long long* first) {
    const uint64_t i = base + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t ua = mix(2 * i), ub = mix(2 * i + 1);
    // exponents in the guarded range: |a|, |b| in [2^-100, 2^100], |a/b| in [2^-101, 2^101]
    ua = (ua & 0x807fffffu) | ((27u + (ua >> 23) % 201u) << 23);
    ub = (ub & 0x807fffffu) | ((27u + (ub >> 23) % 201u) << 23);
    if (mode == 1) ub |= 0x007fffffu;                    // b's significand all ones
    if (mode == 2) ub = (ub & 0xff800000u) | (mix(3 * i) & 0x7fu);  // b's significand nearly 1
    if (mode == 3) ua = (ua & 0xff800000u) | 0x007fffffu;  // a's significand all ones
    const float a = __uint_as_float(ua), b = __uint_as_float(ub);
    const int ea = (int)((ua >> 23) & 0xffu), eb = (int)((ub >> 23) & 0xffu);
    if (ea - eb < -100 || ea - eb > 100) return;
    if (__float_as_uint(div_m(a, b)) != __float_as_uint(a / b)) {
        if (atomicAdd(&bad[5], 1ull) < 4) { first[12] = ua; first[13] = ub; }
    }
}

int main() {
    unsigned long long *bad, *first;
    hipMalloc(&bad, 8 * 8);
    hipMalloc(&first, 16 * 8);
    hipMemset(bad, 0, 64);
    hipMemset(first, 0, 128);
    const uint64_t per = 1ull << 28;
    for (uint64_t b = 0; b < (1ull << 32); b += per) hipLaunchKernelGGL(unary, dim3(per / 256), dim3(256), 0, 0, b, bad, first);
    hipDeviceSynchronize();
    unsigned long long h[8], f[16];
    hipMemcpy(h, bad, 64, hipMemcpyDeviceToHost);
    hipMemcpy(f, first, 128, hipMemcpyDeviceToHost);
    printf("exhaustive over 2^32 floats (in their guarded ranges):\n");
    printf("  rcp  v_rcp + 1 Newton (fma)         mismatches %llu  e.g. %08llx %08llx\n", h[0], f[0], f[1]);
    printf("  sqrt v_sqrt + residual +-1 ulp      mismatches %llu  e.g. %08llx %08llx\n", h[1], f[4], f[5]);
    printf("  sqrt v_rsq + Markstein step         mismatches %llu  e.g. %08llx %08llx\n", h[2], f[8], f[9]);
    printf("  sqrt bare v_sqrt                    mismatches %llu\n", h[3]);
    printf("  1/sqrt as rcp_nr(sqrt_res)          mismatches %llu\n", h[4]);
    const uint64_t n = 1ull << 34;
    for (int mode = 0; mode < 4; ++mode)
        for (uint64_t b = 0; b < n / 4; b += per) hipLaunchKernelGGL(binary, dim3(per / 256), dim3(256), 0, 0, b + mode * n, mode, bad, first);
    hipDeviceSynchronize();
    hipMemcpy(h, bad, 64, hipMemcpyDeviceToHost);
    hipMemcpy(f, first, 128, hipMemcpyDeviceToHost);
    printf("a/b Markstein (CR reciprocal, q = a*y, one fma correction), 2^34 pairs (random, b all-ones, b ~ 1, a all-ones):\n");
    printf("  mismatches %llu  e.g. a=%08llx b=%08llx\n", h[5], f[12], f[13]);
    return 0;
}
