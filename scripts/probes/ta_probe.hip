// Microbenchmark: texture-address (TA) cycles of a divergent 16-B global load as a function of the
// active lanes.  Each lane walks a dependent chain of loads from a 16 KB table (L1-resident) at
// hashed addresses; only lanes < ACTIVE take part.  Run under rocprofv3 --pmc TA_TA_BUSY_sum
// TA_FLAT_READ_WAVEFRONTS_sum: TA cycles per load wave-instruction for ACTIVE = 64, 32, 16, 8.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

__global__ __launch_bounds__(256) void chase(const float4* __restrict__ tab, float* out, int iters, int active) {
    const int lane = threadIdx.x & 63;
    float acc = 0.0f;
    if (lane < active) {
        uint32_t i = (blockIdx.x * 256u + threadIdx.x) * 2654435761u;
        for (int k = 0; k < iters; ++k) {
            const float4 v = tab[(i >> 8) & 1023u];  // 1024 x 16 B = 16 KB
            acc += v.x;
            i = i * 1664525u + 1013904223u + __float_as_uint(v.y);
        }
    }
    out[blockIdx.x * 256 + threadIdx.x] = acc;
}

int main(int argc, char** argv) {
    const int active = argc > 1 ? atoi(argv[1]) : 64;
    const int blocks = 256 * 8, iters = 2000;
    float4* tab;
    float* out;
    if (hipMalloc(&tab, 1024 * sizeof(float4)) != hipSuccess || hipMalloc(&out, blocks * 256 * sizeof(float)) != hipSuccess) return 1;
    (void)hipMemset(tab, 0, 1024 * sizeof(float4));
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    hipLaunchKernelGGL(chase, dim3(blocks), dim3(256), 0, 0, tab, out, iters, active);
    (void)hipEventRecord(a);
    hipLaunchKernelGGL(chase, dim3(blocks), dim3(256), 0, 0, tab, out, iters, active);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    printf("active %d: %.3f ms, %.2f ns per wave-load per CU\n", active, ms, ms * 1e6 / ((double)blocks * 4 * iters / 256));
    return 0;
}
