// rt_kernels_shipped.hip -- KernelEntry under the MathShipped policy: the reference kernel as
// the AMD OpenCL compiler builds it by default (clBuildProgram(" -I . "), CLutils.cpp:52-66).
//
// The policy spells out every reference `/` and sqrt as the backend's OpenCL-accuracy
// expansions (MathShipped::rcp/div/sqrt) and every fp-contract=on fusion as an fma at the
// reference's expression site (madd, rt_math.hpp).  This TU is also compiled with
// -fno-hip-fp32-correctly-rounded-divide-sqrt, so any division left to the compiler gets the
// same OpenCL accuracy instead of the HIP default.  Only MathShipped is instantiated here.
#include "rt_kernels_body.hpp"

#pragma clang fp contract(off)

namespace rtk {

// LDS-resident scenes run 5 waves per SIMD (VALU-bound); scenes read from HBM/L2 run 6 (load
// latency to hide: bunny proxy -2.4 %, profiles/r01/global_path_waves_ab.txt)
template <bool kStats, bool kBofs, int kMode>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(RT_STEP_DEVICELIB_WAVES, 8)))
void kernel_entry_step_shipped_lds(KernelArgs a) {
    step_body<MathShipped, true, kStats, kBofs, false, kMode>(a);
}
template <bool kStats, int kMode>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(RT_STEP_GLOBAL_WAVES, 8)))
void kernel_entry_step_shipped_global(KernelArgs a) {
    step_body<MathShipped, false, kStats, false, false, kMode>(a);
}
// octant records read from HBM/L2 (scenes too large for LDS): the LDS path's walk
template <bool kStats, int kMode>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(RT_STEP_GOCT_WAVES, 8)))
void kernel_entry_step_shipped_goct(KernelArgs a) {
    step_body<MathShipped, true, kStats, false, true, kMode>(a);
}

__global__ void pack_mats_shipped(const rt_cl_material* __restrict__ in, float4* __restrict__ out, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    material_record<MathShipped>(in[i], out + 4 * i);
}

template <bool L, bool S, int kMode>
static KernelFn pick_step_shipped(bool bofs, bool goct) {
    if (!L) return goct ? kernel_entry_step_shipped_goct<S, kMode> : kernel_entry_step_shipped_global<S, kMode>;
    return bofs ? kernel_entry_step_shipped_lds<S, true, kMode> : kernel_entry_step_shipped_lds<S, false, kMode>;
}
template <bool L, bool S>
static KernelFn pick_sched_shipped(int sched, bool bofs, bool goct, bool fused) {
    if (sched == kSchedStep) {
        if constexpr (S || !RT_SPECIALIZE_FUSED)
            return pick_step_shipped<L, S, 0>(bofs, goct);
        else
            return fused ? pick_step_shipped<L, S, 1>(bofs, goct) : pick_step_shipped<L, S, 2>(bofs, goct);
    }
    return kernel_entry<MathShipped, L, S>;
}

KernelFn pick_shipped(int sched, bool lds, bool stats, bool bofs, bool goct, bool fused) {
    if (lds)
        return stats ? pick_sched_shipped<true, true>(sched, bofs, false, fused)
                     : pick_sched_shipped<true, false>(sched, bofs, false, fused);
    return stats ? pick_sched_shipped<false, true>(sched, bofs, goct, fused)
                 : pick_sched_shipped<false, false>(sched, bofs, goct, fused);
}

__global__ __launch_bounds__(256) RT_ACCUM_OCC void accum_frames_shipped(KernelArgs a, const uint32_t* key) {
    accum_frames_body<MathShipped>(a, key);
}
__global__ void accum_key_shipped(KernelArgs a, uint32_t* key) {
    accum_key_body<MathShipped>(a, key);
}

hipError_t launch_accum_frames_shipped(const KernelArgs& a, uint32_t* key, hipStream_t st) {
    const dim3 grid((a.nTiles + kAccumWgWaves - 1u) / kAccumWgWaves);
    hipLaunchKernelGGL(accum_key_shipped, dim3(1), dim3(64), 0, st, a, key);
    hipLaunchKernelGGL(accum_frames_shipped, grid, dim3(64 * kAccumWgWaves), 0, st, a, key);
    return hipGetLastError();
}

WfKernels pick_wf_shipped(bool lds, bool stats, bool bofs, bool goct) {
    return wf_pick<MathShipped>(lds, stats, bofs, goct);
}

hipError_t launch_pack_mats_shipped(const rt_cl_material* mats, uint32_t n_mats, float4* pm, hipStream_t st) {
    hipLaunchKernelGGL(pack_mats_shipped, dim3((n_mats + 255) / 256), dim3(256), 0, st, mats, pm, n_mats);
    return hipGetLastError();
}

}  // namespace rtk
