// Which XCD / shader engine / CU a CU-mask bit of hipExtStreamCreateWithCUMask selects on this GPU:
// for a few single-bit masks (and a few multi-bit ones), launch 64 workgroups on a stream with that
// mask and record each workgroup's XCC_ID and HW_ID (SE, SH, CU) hardware registers (read only).
// Prints one line per mask: bit(s) -> the distinct (xcc, se, cu) the workgroups ran on.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <set>
#include <tuple>
#include <vector>

__global__ void where(uint32_t* out) {
    uint32_t xcc, hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    if (threadIdx.x == 0) {
        out[2 * blockIdx.x] = xcc;
        out[2 * blockIdx.x + 1] = hw;
    }
    // keep the workgroup resident a little so the dispatcher spreads them
    for (volatile int i = 0; i < 2000; ++i) {
    }
}

int main() {
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, 0) != hipSuccess) return 1;
    const int ncu = p.multiProcessorCount;
    std::printf("CUs %d\n", ncu);
    const int nwg = 64;
    uint32_t* d = nullptr;
    if (hipMalloc(&d, nwg * 2 * sizeof(uint32_t)) != hipSuccess) return 1;
    std::vector<std::vector<int>> masks;
    for (int b : {0, 1, 2, 3, 7, 8, 31, 32, 33, 64, 128, 224, 255}) masks.push_back({b});
    masks.push_back({0, 1, 2, 3, 4, 5, 6, 7});
    masks.push_back({0, 32, 64, 96, 128, 160, 192, 224});
    for (const auto& bits : masks) {
        std::vector<uint32_t> m((ncu + 31) / 32, 0u);
        for (int b : bits)
            if (b < ncu) m[b / 32] |= 1u << (b % 32);
        hipStream_t s;
        if (hipExtStreamCreateWithCUMask(&s, (uint32_t)m.size(), m.data()) != hipSuccess) return 2;
        hipLaunchKernelGGL(where, dim3(nwg), dim3(64), 0, s, d);
        std::vector<uint32_t> h(nwg * 2);
        if (hipMemcpyAsync(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost, s) != hipSuccess) return 3;
        if (hipStreamSynchronize(s) != hipSuccess) return 4;
        std::set<std::tuple<int, int, int, int>> seen;
        for (int i = 0; i < nwg; ++i) {
            const uint32_t hw = h[2 * i + 1];
            // gfx9 HW_ID: wave 3:0, simd 5:4, pipe 7:6, cu 11:8, sh 12, se 15:13
            seen.insert({(int)(h[2 * i] & 0xf), (int)((hw >> 13) & 7), (int)((hw >> 12) & 1), (int)((hw >> 8) & 0xf)});
        }
        std::printf("bits");
        for (int b : bits) std::printf(" %d", b);
        std::printf(" ->");
        for (auto& t : seen)
            std::printf(" (xcc %d se %d sh %d cu %d)", std::get<0>(t), std::get<1>(t), std::get<2>(t), std::get<3>(t));
        std::printf("\n");
        (void)hipStreamDestroy(s);
    }
    (void)hipFree(d);
    return 0;
}
