// rt_kernels.hip -- KernelEntry entry points for the pinned and devicelib math policies,
// the scene packing kernels and the host-side launch helpers.  The device code is
// rt_kernels_body.hpp; the shipped policy lives in rt_kernels_shipped.hip.
#include "rt_kernels_body.hpp"

#pragma clang fp contract(off)

namespace rtk {

// Entry points per math policy: the devicelib body fits 80 VGPRs with a small spill, and
// 6 waves per SIMD measured 7 % faster than the 4 its natural 113 VGPRs allow
// (profiles/r01/occupancy_ab.txt); the fp64-heavy pinned body stays at its natural budget.
// (LDS scenes 5 waves per SIMD, scenes read from HBM/L2 6, as for the shipped policy)
template <bool kStats, bool kBofs, int kMode>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(RT_STEP_DEVICELIB_WAVES, 8)))
void kernel_entry_step_devicelib_lds(KernelArgs a) {
    step_body<MathDeviceLib, true, kStats, kBofs, false, kMode>(a);
}
template <bool kStats, int kMode>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(RT_STEP_GLOBAL_WAVES, 8)))
void kernel_entry_step_devicelib_global(KernelArgs a) {
    step_body<MathDeviceLib, false, kStats, false, false, kMode>(a);
}
template <bool kStats, int kMode>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(RT_STEP_GOCT_WAVES, 8)))
void kernel_entry_step_devicelib_goct(KernelArgs a) {
    step_body<MathDeviceLib, true, kStats, false, true, kMode>(a);
}
// The pinned body on LDS scenes: 5 waves per SIMD (96 VGPRs, 80 B of spills) against the 4 its
// natural 116 VGPRs allow -- 4K Cornell 8 spp 1.044 -> 1.007 ms/frame (profiles/r06/pinned_ab.txt);
// the HBM/L2 walks keep their natural budget (1: no register cap)
#ifndef RT_STEP_PINNED_WAVES
#define RT_STEP_PINNED_WAVES 5
#endif
template <bool kLdsScene, bool kStats, bool kBofs, bool kGlobalOct, int kMode>
__global__ __launch_bounds__(256)
__attribute__((amdgpu_waves_per_eu(kLdsScene && !kGlobalOct ? RT_STEP_PINNED_WAVES : 1, 8)))
void kernel_entry_step_pinned(KernelArgs a) {
    step_body<MathPinned, kLdsScene, kStats, kBofs, kGlobalOct, kMode>(a);
}


// ---- scene packing (runs once per bound scene) -----------------------------------------------
__global__ void pack_shade(const rt_cl_triangle* __restrict__ in, float4* __restrict__ out, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const rt_cl_triangle& t = in[i];
    out[3 * i] = make_float4(t.v1.normal.x, t.v1.normal.y, t.v1.normal.z, __uint_as_float(t.mtlIndex));
    out[3 * i + 1] = make_float4(t.v2.normal.x, t.v2.normal.y, t.v2.normal.z, t.v3.normal.x);
    out[3 * i + 2] = make_float4(t.v3.normal.y, t.v3.normal.z, 0.0f, 0.0f);
}

__global__ void pack_mats(const rt_cl_material* __restrict__ in, float4* __restrict__ out, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    material_record<MathDeviceLib>(in[i], out + 4 * i);
}

__global__ void pack_tris(const rt_cl_triangle* __restrict__ in, float4* __restrict__ out, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const rt_float3 p1 = in[i].v1.position, p2 = in[i].v2.position, p3 = in[i].v3.position;
    // e1 = t2 - t1, e2 = t3 - t1 exactly as kernel_bvh.cl:109-110 computes them
    // 9 floats in a 48-B slot, packed so that a lane reads them with two 16-B and one 4-B
    // access (3 x 12-B reads cost twice the LDS cycles of 3 x 16-B ones)
    out[3 * i] = make_float4(p1.x, p1.y, p1.z, p2.x - p1.x);
    out[3 * i + 1] = make_float4(p2.y - p1.y, p2.z - p1.z, p3.x - p1.x, p3.y - p1.y);
    out[3 * i + 2] = make_float4(p3.z - p1.z, 0.0f, 0.0f, 0.0f);
}

}  // namespace rtk

// ---- host-side launch helpers ------------------------------------------------------------
namespace rtk {

// Kernel variants: [schedule][math][scene in LDS][stats].

template <class M, bool L, bool S, int kMode>
static KernelFn pick_step(bool bofs, bool goct) {
    if (M::kId == MathDeviceLib::kId) {
        if (!L) return goct ? kernel_entry_step_devicelib_goct<S, kMode> : kernel_entry_step_devicelib_global<S, kMode>;
        return bofs ? kernel_entry_step_devicelib_lds<S, true, kMode> : kernel_entry_step_devicelib_lds<S, false, kMode>;
    }
    if (!L) return goct ? kernel_entry_step_pinned<true, S, false, true, kMode> : kernel_entry_step_pinned<false, S, false, false, kMode>;
    return bofs ? kernel_entry_step_pinned<true, S, true, false, kMode> : kernel_entry_step_pinned<true, S, false, false, kMode>;
}
template <class M, bool L, bool S>
static KernelFn pick_sched(int sched, bool bofs, bool goct, bool fused) {
    if (sched == kSchedStep) {
        if constexpr (S || !RT_SPECIALIZE_FUSED)
            return pick_step<M, L, S, 0>(bofs, goct);
        else
            return fused ? pick_step<M, L, S, 1>(bofs, goct) : pick_step<M, L, S, 2>(bofs, goct);
    }
    return kernel_entry<M, L, S>;
}

// bofs: LDS node records with the B planes at kOctB (KernelArgs::octB == kOctB); goct: a scene
// too large for LDS walked through its octant records in HBM/L2 (step schedule); fused: a fused
// frames launch (KernelArgs::radBuf set)
static KernelFn pick(int sched, int math, bool lds, bool stats, bool bofs, bool goct, bool fused) {
    if (math == MathShipped::kId) return pick_shipped(sched, lds, stats, bofs, goct, fused);
    if (math == MathDeviceLib::kId) {
        if (lds) return stats ? pick_sched<MathDeviceLib, true, true>(sched, bofs, false, fused) : pick_sched<MathDeviceLib, true, false>(sched, bofs, false, fused);
        return stats ? pick_sched<MathDeviceLib, false, true>(sched, bofs, goct, fused) : pick_sched<MathDeviceLib, false, false>(sched, bofs, goct, fused);
    }
    if (lds) return stats ? pick_sched<MathPinned, true, true>(sched, bofs, false, fused) : pick_sched<MathPinned, true, false>(sched, bofs, false, fused);
    return stats ? pick_sched<MathPinned, false, true>(sched, bofs, goct, fused) : pick_sched<MathPinned, false, false>(sched, bofs, goct, fused);
}

hipError_t launch_kernel_entry(const KernelArgs& a, int sched, int math, bool lds, bool stats, unsigned grid,
                               size_t smem, hipStream_t st, bool goct) {
    KernelFn fn = pick(sched, math, lds, stats, lds && a.octB == kOctB, goct, a.radBuf != nullptr);
    hipLaunchKernelGGL(fn, dim3(grid), dim3(256), smem, st, a);
    return hipGetLastError();
}

template <class M>
__global__ __launch_bounds__(256) RT_ACCUM_OCC void accum_frames(KernelArgs a, const uint32_t* key) {
    accum_frames_body<M>(a, key);
}
template <class M>
__global__ void accum_key(KernelArgs a, uint32_t* key) {
    accum_key_body<M>(a, key);
}

hipError_t launch_accum_frames(const KernelArgs& a, int math, uint32_t* key, hipStream_t st) {
    if (math == MathShipped::kId) return launch_accum_frames_shipped(a, key, st);
    const dim3 grid((a.nTiles + kAccumWgWaves - 1u) / kAccumWgWaves);
    if (math == MathDeviceLib::kId) {
        hipLaunchKernelGGL(accum_key<MathDeviceLib>, dim3(1), dim3(64), 0, st, a, key);
        hipLaunchKernelGGL(accum_frames<MathDeviceLib>, grid, dim3(64 * kAccumWgWaves), 0, st, a, key);
    } else {
        hipLaunchKernelGGL(accum_key<MathPinned>, dim3(1), dim3(64), 0, st, a, key);
        hipLaunchKernelGGL(accum_frames<MathPinned>, grid, dim3(64 * kAccumWgWaves), 0, st, a, key);
    }
    return hipGetLastError();
}

int occupancy_kernel_entry(int sched, int math, bool lds, bool stats, bool bofs, size_t smem, bool goct, bool fused) {
    int blocks = 0;
    KernelFn fn = pick(sched, math, lds, stats, lds && bofs, goct, fused);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, fn, 256, smem) != hipSuccess) return 1;
    return blocks > 0 ? blocks : 1;
}

// ---- wavefront schedule ------------------------------------------------------------------------
static WfKernels pick_wf(int math, bool lds, bool stats, bool bofs, bool goct) {
    if (math == MathShipped::kId) return pick_wf_shipped(lds, stats, bofs, goct);
    if (math == MathDeviceLib::kId) return wf_pick<MathDeviceLib>(lds, stats, bofs, goct);
    return wf_pick<MathPinned>(lds, stats, bofs, goct);
}

hipError_t launch_wavefront(const KernelArgs& a, WfArgs w, float4* const q[2], uint32_t* const cnt[2], int math,
                            bool lds, bool stats, bool bofs, unsigned grid_e, size_t smem_e, unsigned grid_s,
                            hipStream_t st, bool goct) {
    const WfKernels kf = pick_wf(math, lds, stats, bofs, goct);
    for (int b = 0; b < a.lightBounces; ++b) {
        w.bounce = (uint32_t)b;
        w.inQ = q[b & 1];
        w.outQ = q[(b + 1) & 1];
        w.inCnt = cnt[b & 1];
        w.outCnt = cnt[(b + 1) & 1];
        hipLaunchKernelGGL(kf.extend, dim3(grid_e), dim3(kWfExtendThreads), smem_e, st, a, w);
        hipLaunchKernelGGL(kf.shade, dim3(grid_s), dim3(kWfShadeThreads), 0, st, a, w);
    }
    return hipGetLastError();
}

int occupancy_wf_extend(int math, bool lds, bool stats, bool bofs, size_t smem, bool goct) {
    int blocks = 0;
    const WfKernels kf = pick_wf(math, lds, stats, lds && bofs, goct);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, kf.extend, kWfExtendThreads, smem) != hipSuccess)
        return 1;
    return blocks > 0 ? blocks : 1;
}

int occupancy_wf_shade(int math, bool stats) {
    int blocks = 0;
    const WfKernels kf = pick_wf(math, false, stats, false, false);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, kf.shade, kWfShadeThreads, 0) != hipSuccess) return 1;
    return blocks > 0 ? blocks : 1;
}

// rtDiagPinnedMath: the pinned policy's builtins, element-wise (tests)
__global__ void pinned_math_kernel(int op, const float* __restrict__ a, const float* __restrict__ b,
                                   float* __restrict__ out, size_t n) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float x = a[i];
    float r;
    switch (op) {
        case 0: r = MathPinned::rcp(x); break;
        case 1: r = MathPinned::div(x, b[i]); break;
        case 2: r = MathPinned::sqrt(x); break;
        case 3: r = MathPinned::rsqrt(x); break;
        case 4: r = MathPinned::pow(x, b[i]); break;
        case 5: r = MathPinned::sin(x); break;
        default: r = MathPinned::cos(x); break;
    }
    out[i] = r;
}

hipError_t launch_pinned_math(int op, const float* a, const float* b, float* out, size_t n, hipStream_t st) {
    if (n) hipLaunchKernelGGL(pinned_math_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, op, a, b, out, n);
    return hipGetLastError();
}

hipError_t launch_pack(const rt_cl_triangle* tris, uint32_t n_tris, float4* pt, float4* ps,
                       const rt_cl_material* mats, uint32_t n_mats, float4* pm, hipStream_t st) {
    if (n_tris) hipLaunchKernelGGL(pack_tris, dim3((n_tris + 255) / 256), dim3(256), 0, st, tris, pt, n_tris);
    if (n_tris) hipLaunchKernelGGL(pack_shade, dim3((n_tris + 255) / 256), dim3(256), 0, st, tris, ps, n_tris);
    if (n_mats) hipLaunchKernelGGL(pack_mats, dim3((n_mats + 255) / 256), dim3(256), 0, st, mats, pm, n_mats);
    // the shipped policy's material records (2.5-ulp divisions) follow the IEEE ones
    if (n_mats) {
        hipError_t e = launch_pack_mats_shipped(mats, n_mats, pm + 4 * (size_t)n_mats, st);
        if (e != hipSuccess) return e;
    }
    return hipGetLastError();
}

}  // namespace rtk

