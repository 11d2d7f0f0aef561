// Microbenchmark: does the texture-address unit's cost per divergent 16-B load follow the number of
// distinct cache lines the wave's lanes touch?  Each lane walks a dependent chain of dwordx4 loads
// in a 64 KB table (L1/L2-resident); at every step the wave's 64 lanes are spread over L distinct
// 128-B lines (lanes of one line read different 16-B records of it).  L = 64 is fully divergent.
// usage: ta_lines_probe [L ...]   prints ns per wave-load per CU from HIP events
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef float v4f __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void chase(const v4f* __restrict__ tab, float* out, int iters, uint32_t lines) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t grp = lane % lines;  // this lane's line among the wave's `lines`
    uint32_t i = blockIdx.x * 2654435761u + (threadIdx.x >> 6) * 40503u;  // wave-uniform chain seed
    float acc = 0.0f;
    for (int k = 0; k < iters; ++k) {
        // wave-uniform base line (the chain), lanes spread over `lines` lines and 8 records per line
        const uint32_t line = ((i >> 8) + grp * 977u) & 511u;  // 512 lines of 128 B = 64 KB
        const v4f a = tab[line * 8u + ((lane / lines) & 7u)];
        acc += a.x + a.y + a.z + a.w;
        i = i * 1664525u + 1013904223u + (uint32_t)__builtin_amdgcn_readfirstlane(__float_as_uint(a.x));
    }
    out[blockIdx.x * 256 + threadIdx.x] = acc;
}

int main(int argc, char** argv) {
    const int blocks = 256 * 8, iters = 2000;
    v4f* tab;
    float* out;
    if (hipMalloc(&tab, 4096 * sizeof(v4f)) != hipSuccess || hipMalloc(&out, blocks * 256 * sizeof(float)) != hipSuccess)
        return 1;
    (void)hipMemset(tab, 0, 4096 * sizeof(v4f));
    for (int ai = 1; ai < argc; ++ai) {
        const uint32_t L = (uint32_t)atoi(argv[ai]);
        hipEvent_t a, b;
        (void)hipEventCreate(&a);
        (void)hipEventCreate(&b);
        hipLaunchKernelGGL(chase, dim3(blocks), dim3(256), 0, 0, tab, out, iters, L);
        (void)hipEventRecord(a);
        hipLaunchKernelGGL(chase, dim3(blocks), dim3(256), 0, 0, tab, out, iters, L);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, a, b);
        printf("lines %2u: %.3f ms, %.2f ns per wave-load per CU\n", L, ms, ms * 1e6 / ((double)blocks * 4 * iters / 256));
    }
    return 0;
}
