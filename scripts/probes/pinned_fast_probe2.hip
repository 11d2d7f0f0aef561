// Probe (not product code), part 2: correctly rounded sqrt and 1/sqrt (two roundings) from v_sqrt_f32 /
// v_rsq_f32 plus fma corrections -- mismatches against hipcc's IEEE sqrtf and 1.0f / sqrtf per
// exponent field of x (positive normal floats, exhaustive).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#pragma clang fp contract(off)

__device__ __forceinline__ float rcp_nr(float x) {
    const float y = __builtin_amdgcn_rcpf(x);
    return __builtin_fmaf(__builtin_fmaf(-x, y, 1.0f), y, y);
}
__device__ __forceinline__ float sqrt_res(float x) {  // S1
    const float s = __builtin_amdgcn_sqrtf(x);
    const float lo = __uint_as_float(__float_as_uint(s) - 1u), hi = __uint_as_float(__float_as_uint(s) + 1u);
    const float rl = __builtin_fmaf(-lo, s, x), rh = __builtin_fmaf(-hi, s, x);
    float r = rl <= 0.0f ? lo : s;
    return rh > 0.0f ? hi : r;
}
__device__ __forceinline__ float sqrt_rsq(float x) {  // S2
    const float r = __builtin_amdgcn_rsqf(x);
    const float s = x * r, h = 0.5f * r;
    return __builtin_fmaf(__builtin_fmaf(-s, s, x), h, s);
}
__device__ __forceinline__ float sqrt_rsq2(float x) {  // S4: S2 then S1's +-1 ulp residual fix
    const float s = sqrt_rsq(x);
    const float lo = __uint_as_float(__float_as_uint(s) - 1u), hi = __uint_as_float(__float_as_uint(s) + 1u);
    const float rl = __builtin_fmaf(-lo, s, x), rh = __builtin_fmaf(-hi, s, x);
    float r = rl <= 0.0f ? lo : s;
    return rh > 0.0f ? hi : r;
}
__device__ __forceinline__ float sqrt_res_mid(float x) {  // S5: +-1 ulp by the midpoint test (exact)
    const float s = __builtin_amdgcn_sqrtf(x);
    // candidate c, midpoints m- = c - ulp/2, m+ = c + ulp/2 tested with fma residuals of the
    // neighbours: x - lo*s <= 0 ... (S1's test, but on the pair (lo, s) and (s, hi) symmetric)
    const float lo = __uint_as_float(__float_as_uint(s) - 1u), hi = __uint_as_float(__float_as_uint(s) + 1u);
    const float rl = __builtin_fmaf(-lo, hi, x);  // x - lo*hi ~ x - s^2 + ulp^2
    const float rh = __builtin_fmaf(-s, hi, x);   // x - s*hi
    const float rm = __builtin_fmaf(-lo, s, x);   // x - lo*s
    float r = s;
    if (rm <= 0.0f) r = lo;       // s^2 - s*ulp >= x: below the lower midpoint
    if (rh > 0.0f) r = hi;        // s^2 + s*ulp < x: above the upper midpoint
    (void)rl;
    return r;
}

__global__ void k(uint32_t e, unsigned long long* bad) {
    const uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;  // 2^23 significands
    const float x = __uint_as_float((e << 23) | m);
    const float sr = __builtin_sqrtf(x), rs = 1.0f / sr;
    if (__float_as_uint(sqrt_res(x)) != __float_as_uint(sr)) atomicAdd(&bad[e * 8 + 0], 1ull);
    if (__float_as_uint(sqrt_rsq(x)) != __float_as_uint(sr)) atomicAdd(&bad[e * 8 + 1], 1ull);
    if (__float_as_uint(sqrt_rsq2(x)) != __float_as_uint(sr)) atomicAdd(&bad[e * 8 + 2], 1ull);
    if (__float_as_uint(rcp_nr(sqrt_res(x))) != __float_as_uint(rs)) atomicAdd(&bad[e * 8 + 3], 1ull);
    if (__float_as_uint(rcp_nr(sqrt_rsq2(x))) != __float_as_uint(rs)) atomicAdd(&bad[e * 8 + 4], 1ull);
    if (__float_as_uint(sqrt_res_mid(x)) != __float_as_uint(sr)) atomicAdd(&bad[e * 8 + 5], 1ull);
}

int main() {
    unsigned long long* bad;
    (void)hipMalloc(&bad, 256 * 8 * 8);
    (void)hipMemset(bad, 0, 256 * 8 * 8);
    for (uint32_t e = 1; e < 255; ++e) hipLaunchKernelGGL(k, dim3((1u << 23) / 256), dim3(256), 0, 0, e, bad);
    (void)hipDeviceSynchronize();
    unsigned long long h[256 * 8];
    (void)hipMemcpy(h, bad, sizeof(h), hipMemcpyDeviceToHost);
    const char* names[6] = {"S1 v_sqrt + residual +-1ulp", "S2 v_rsq + Markstein", "S4 S2 + residual +-1ulp",
                            "1/sqrt rcp_nr(S1)", "1/sqrt rcp_nr(S4)", "S5 v_sqrt + midpoint residuals"};
    for (int v = 0; v < 6; ++v) {
        unsigned long long tot = 0;
        int lo = 999, hi = -1;
        for (int e = 1; e < 255; ++e)
            if (h[e * 8 + v]) { tot += h[e * 8 + v]; lo = e < lo ? e : lo; hi = e > hi ? e : hi; }
        printf("%-34s mismatches %llu, exponent fields with any: [%d, %d]\n", names[v], tot, lo, hi);
        if (tot) {
            printf("   per exponent field:");
            for (int e = 1; e < 255; ++e) if (h[e * 8 + v]) printf(" %d:%llu", e, h[e * 8 + v]);
            printf("\n");
        }
    }
    return 0;
}
