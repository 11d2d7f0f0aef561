// Microbenchmark: cost of the vector-memory address unit (TA) per divergent load, by load width and
// addressing form -- does a node visit's cost follow its load instructions or its bytes?
// Each lane walks a dependent chain of loads from a 16 KB table (L1-resident) at hashed addresses,
// like the octant walk over HBM/L2 (whose loads hit L1 97 %).  Modes (one "visit" per iteration):
//   0: global dwordx4               1: global dwordx3            2: global dwordx2      3: global dword
//   4: 2 x global dwordx4, two planes (the octant record today: A[o][n], B[o][n])
//   5: global dwordx4 + dwordx3 from one 32-B record
//   6: 2 x buffer dwordx4, two planes
//   7: buffer dwordx4 + dwordx3 from one 32-B record
// Run under rocprofv3 --pmc TA_TA_BUSY_sum GRBM_GUI_ACTIVE (ta_width_probe.sh); the program itself
// prints ns per visit per CU from HIP events.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef float v4f __attribute__((ext_vector_type(4)));
typedef float v3f __attribute__((ext_vector_type(3)));
typedef float v2f __attribute__((ext_vector_type(2)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* p, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}

template <int MODE>
__global__ __launch_bounds__(256) void chase(const float4* __restrict__ tab, float* out, int iters, int active) {
    const int lane = threadIdx.x & 63;
    float acc = 0.0f;
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(tab, 2048u * 16u);
    if (lane < active) {
        uint32_t i = (blockIdx.x * 256u + threadIdx.x) * 2654435761u;
        for (int k = 0; k < iters; ++k) {
            const uint32_t n = (i >> 8) & 511u;  // 512 records of 32 B (or 2 planes of 512 x 16 B)
            const char* base = reinterpret_cast<const char*>(tab);
            float x, y;
            if (MODE == 0) {
                const v4f a = *reinterpret_cast<const v4f*>(base + n * 16u);
                x = a.x + a.w; y = a.y + a.z;
            } else if (MODE == 1) {
                const v3f a = *reinterpret_cast<const v3f*>(base + n * 16u);
                x = a.x + a.z; y = a.y;
            } else if (MODE == 2) {
                const v2f a = *reinterpret_cast<const v2f*>(base + n * 16u);
                x = a.x; y = a.y;
            } else if (MODE == 3) {
                const float a = *reinterpret_cast<const float*>(base + n * 16u);
                x = a; y = a;
            } else if (MODE == 4) {
                const v4f a = *reinterpret_cast<const v4f*>(base + n * 16u);
                const v4f b = *reinterpret_cast<const v4f*>(base + 8192u + n * 16u);
                x = a.x + a.y + b.w + b.x; y = a.z + a.w + b.y + b.z;
            } else if (MODE == 5) {
                const v4f a = *reinterpret_cast<const v4f*>(base + n * 32u);
                const v3f b = *reinterpret_cast<const v3f*>(base + n * 32u + 16u);
                x = a.x + a.y + b.z; y = a.z + a.w + b.x + b.y;
            } else if (MODE == 6) {
                const v4f a = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(n * 16u), 0, 0);
                const v4f b = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(8192u + n * 16u), 0, 0);
                x = a.x + a.y + b.w + b.x; y = a.z + a.w + b.y + b.z;
            } else {
                const v4f a = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(n * 32u), 0, 0);
                const v3f b = __builtin_amdgcn_raw_buffer_load_b96(rs, (int)(n * 32u + 16u), 0, 0);
                x = a.x + a.y + b.z; y = a.z + a.w + b.x + b.y;
            }
            acc += x;
            i = i * 1664525u + 1013904223u + __float_as_uint(y);
        }
    }
    out[blockIdx.x * 256 + threadIdx.x] = acc;
}

template <int MODE>
static float run(const float4* tab, float* out, int blocks, int iters, int active) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    hipLaunchKernelGGL(chase<MODE>, dim3(blocks), dim3(256), 0, 0, tab, out, iters, active);
    (void)hipEventRecord(a);
    hipLaunchKernelGGL(chase<MODE>, dim3(blocks), dim3(256), 0, 0, tab, out, iters, active);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    return ms;
}

int main(int argc, char** argv) {
    const int active = argc > 1 ? atoi(argv[1]) : 64;
    const int blocks = 256 * 8, iters = 2000;
    float4* tab;
    float* out;
    if (hipMalloc(&tab, 2048 * sizeof(float4)) != hipSuccess || hipMalloc(&out, blocks * 256 * sizeof(float)) != hipSuccess)
        return 1;
    (void)hipMemset(tab, 0, 2048 * sizeof(float4));
    const char* names[8] = {"x4", "x3", "x2", "x1", "2 planes x4+x4", "record x4+x3", "buffer 2 planes x4+x4",
                            "buffer record x4+x3"};
    float ms[8];
    ms[0] = run<0>(tab, out, blocks, iters, active);
    ms[1] = run<1>(tab, out, blocks, iters, active);
    ms[2] = run<2>(tab, out, blocks, iters, active);
    ms[3] = run<3>(tab, out, blocks, iters, active);
    ms[4] = run<4>(tab, out, blocks, iters, active);
    ms[5] = run<5>(tab, out, blocks, iters, active);
    ms[6] = run<6>(tab, out, blocks, iters, active);
    ms[7] = run<7>(tab, out, blocks, iters, active);
    for (int m = 0; m < 8; ++m)
        printf("active %2d mode %d %-24s %.3f ms, %.2f ns per wave-visit per CU\n", active, m, names[m], ms[m],
               ms[m] * 1e6 / ((double)blocks * 4 * iters / 256));
    return 0;
}
