// rt_kernels.hpp -- launch interface between the C ABI (rt_capi.cpp) and the kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/rt_cl_types.h"

namespace rtk {

// Everything KernelEntry's 14 arguments carry (kernel_bvh.cl:415-431), plus the packed
// scene, the work-item range of this launch and the optional extension outputs.
struct KernelArgs {
    float4* result;                     // slot 0: float3 per work-item, 16-byte stride
    const rt_cl_triangle* trisFull;     // slot 1 (normals, material index)
    const rt_cl_material* materials;    // slot 3
    const float4* packedTris;           // derived from slot 1: 3 x float4 per triangle
    const float4* octNodes;             // derived from slot 2: [node][octant] resolved records (LDS path)
    const float4* gNodes;               // derived from slot 2: 64-B node records (global path)
    const float4* shadeTris;            // derived from slot 1: {n1, mtlIndex}, {n2, n3.x}, {n3.yz} per triangle
    const float4* shadeMats;            // derived from slot 3: {diffuse, 1/(a+1)}, {specular, a^2/pi}, {emission, a^2-1}, {rough, a}
    uint32_t nNodes, nTris, nMats;
    uint32_t octStride;                 // LDS path: records per octant plane (nodes, END sentinel, odd pad)
    uint32_t octB;                      // LDS path: float4 offset of the B planes (8 * octStride, or kOctB)
    uint32_t octRecords;                // LDS path: float4s of node records (octB + 8 * octStride)
    uint32_t nTop;                      // global path: leading gNodes records staged in LDS
    uint32_t width, height;             // slots 4, 5
    uint32_t frameCount;                // slot 6 (slot 7, frameSeed, is unused by the reference)
    int32_t lightBounces, lightType;    // slots 8, 9
    float skyboxIntensity;              // slot 10
    float camPos[3], camFront[3], camUp[3];  // slots 11-13 (w ignored)
    // work decomposition: work-items [gidBegin, gidEnd), rows [rowBegin, rowEnd)
    uint64_t gidBegin, gidEnd;
    uint32_t rowBegin, rowCount, tilesX, nTiles;  // tiles: 16x16 (tile schedule) or 8x8 (regen)
    uint32_t* workCounter;              // persistent schedules: next chunk (zeroed per launch)
    uint32_t chunkPixels, tailChunk;    // pixels per chunk (multiples of 64: whole 8x8 tiles), bulk / tail
    uint32_t chunkSplit;                // bulk chunks cover pixels [0, chunkSplit) of the tile order
    uint32_t refillMin, shadeMin;       // step schedule batching thresholds (lanes)
    uint32_t stepWeightNode, stepWeightLeaf;  // step schedule: relative cost of node / triangle steps
    uint32_t bandPeriod, bandPhase;     // 8-row bands: this launch renders bands b % period == phase
    // extensions
    int32_t* hitIds;                    // primary hit primitive per work-item (-1 = miss)
    float* hitT;                        // primary isect.t per work-item
    unsigned long long* stats;          // [rays, node visits, triangle tests, hits, 4 phase-cycle sums]
    // rtEnqueueKernelFrames (step schedule): frames frameCount .. frameCount + nFrames - 1 in one
    // launch; radiance per (frame slot, gid) in radBuf[slot * radStride + gid] (null: one frame)
    float4* radBuf;
    // primary-miss flags: 1 = radiance (K_rad x3), not in radBuf.  flagTiles 0: one byte per
    // [slot * radStride + gid]; flagTiles 1 (the LDS walk's ray ring): one 64-bit word per
    // [slot * nTiles + tile], bit = pixel's lane in the tile, written once by the wave that
    // generated the tile's camera rays; every path not decided at its camera ray stores its
    // radiance.  flagTiles 2 (the HBM/L2 octant walk): no flags, every path stores it
    uint8_t* frameFlags;
    uint32_t flagTiles;
    uint32_t nFrames, radStride;
    uint32_t tileMajor;                 // fused: work items ordered (tile, frame) instead of (frame, tile)
    // per-frame launches (step schedule): sky-pixel shortcut key, chained launch to launch --
    // pfKeyIn = the value all-sky pixels hold if they followed the chain, pfKeyOut = this launch's
    const uint32_t* pfKeyIn;
    uint32_t* pfKeyOut;
    // (appended fields: the earlier ones keep their offsets)
    uint32_t* workCounterClear;         // per-frame step launches: the other counter slot, zeroed by this launch
    uint32_t tailBase;                  // first tail work item the tail counter hands out (next_chunk)
    uint32_t staticFirst;               // step schedule: waves start with their own tail chunk (no bulk region)
    // counter partitions (per-frame launches without a bulk region): nParts (a power of two) contiguous
    // ranges of partLen work items, each with its tail counter at workCounter[kPartStride * q + 1]
    uint32_t nParts, partLen;
};

constexpr int kSchedTiles = 0;  // one pixel per lane per 16x16 tile, all bounces in place
// (1: path regeneration and 3: a per-wave LDS path pool were measured slower than the step
// schedule and retired in round 3; DESIGN.md section 5 keeps their numbers)
constexpr int kSchedStep = 2;   // per-wave state machine: node / triangle steps, batched shading
constexpr int kSchedWavefront = 4;  // extend / shade launches per bounce over HBM ray queues
constexpr int kNumSched = 5;
// frames per fused launch (rtEnqueueKernelFrames splits longer runs)
constexpr uint32_t kMaxFusedFrames = 8;
// step schedule LDS per wave: the finish queue, 64 x {radiance, gid}
constexpr uint32_t kFinishWaveBytes = 64u * 16u;
// step schedule, LDS scenes: per-wave ring of camera rays generated a whole 8x8 tile at a time
// ({dir, seed}, {invDir, sign} (fused launches) + work-item id per slot)
constexpr uint32_t kRingSlots = 64;
constexpr uint32_t kRingWaveBytes = kRingSlots * 32u + kRingSlots * 4u;
constexpr uint32_t kRingWaveBytesPf = kRingSlots * 16u + kRingSlots * 4u;  // per-frame: no invDir
// step schedule: per workgroup, each wave's remaining chunk {next, end} (64-bit word per wave),
// from which its siblings take single tiles once the work counter is dry
constexpr uint32_t kStealBytes = 4u * 8u + 32u;  // (padded to whole float4s)
// END as a walk word that is neither a node (< 2^24) nor a leaf code (count << 24 | first, count
// 1..127): the step schedule's byte-address LDS walk and its octant walk over HBM/L2 (step_body)
constexpr uint32_t kEndWalk = 0xff000000u;
#ifndef RT_GOCT_END_WORD
#define RT_GOCT_END_WORD 1  // the HBM/L2 octant walk's END as kEndWalk (0: its sentinel's word, visited)
#endif

// LDS node records of trees with at most kOctBMaxStride records per plane keep their B planes at
// the fixed float4 offset kOctB, so a node step reads B with an immediate offset from A's address
constexpr uint32_t kOctBMaxStride = 64;
// counter partitions: words between two partitions' counters (1 KB), and the most partitions
constexpr uint32_t kPartStride = 256;
constexpr uint32_t kMaxParts = 8;
constexpr uint32_t kOctB = 8 * kOctBMaxStride;

using KernelFn = void (*)(KernelArgs);

// ---- wavefront schedule (rt_wavefront.hpp) ----------------------------------------------------
// Per bounce b: extend(b) walks the BVH for every queued ray, shade(b) shades every queued path
// and appends the continuations to the other queue.
struct WfArgs {
    const float4* inQ;        // bounce-b queue: 4 planes of `cap` float4:
                              //   {o.xyz, path}, {d.xyz, seed}, {beta.xyz, -}, {radiance.xyz, -}
    float4* outQ;             // bounce-(b+1) queue, same layout (written by shade)
    float2* hits;             // [cap] {t, primitive bits}: extend(b) -> shade(b)
    const uint32_t* inCnt;    // [G + 1]: entries per stream of inQ, [G] = their maximum
    uint32_t* outCnt;         // [G + 1]: the same for outQ
    uint32_t cap;             // entries per plane (nBlocks * 64)
    uint32_t G;               // streams
    uint32_t nBlocks;         // 64-entry blocks of the work-item space (nTiles * nFrames)
    uint32_t bounce;          // this launch's bounce index
    uint32_t refillMin;       // extend: take new rays once this many lanes are free
};
using WfKernelFn = void (*)(KernelArgs, WfArgs);
struct WfKernels {
    WfKernelFn extend, shade;
};
constexpr unsigned kWfExtendThreads = 512;  // extend workgroup: 8 waves (LDS scene staged once per 8)
constexpr unsigned kWfShadeThreads = 256;   // shade workgroup: one stream, 256 paths per round
constexpr int kWfMaxBounces = 64;            // longer bounce loops run the step schedule
constexpr uint32_t kWfRingBytes = 64u * 32u;  // extend: per-wave ray ring ({o, position}, {d, -})
// the launches of one wavefront render: for b < lightBounces, extend(b) then shade(b); queues and
// counts alternate between q[0]/q[1] and cnt[0]/cnt[1]
hipError_t launch_wavefront(const KernelArgs& a, WfArgs w, float4* const q[2], uint32_t* const cnt[2], int math,
                            bool lds, bool stats, bool bofs, unsigned grid_e, size_t smem_e, unsigned grid_s,
                            hipStream_t st, bool goct);
int occupancy_wf_extend(int math, bool lds, bool stats, bool bofs, size_t smem, bool goct);
int occupancy_wf_shade(int math, bool stats);
WfKernels pick_wf_shipped(bool lds, bool stats, bool bofs, bool goct);

// goct (step schedule, scene not in LDS): walk the octant records in HBM/L2 instead of the
// 64-B global node records
hipError_t launch_kernel_entry(const KernelArgs& a, int sched, int math, bool lds, bool stats, unsigned grid,
                               size_t smem, hipStream_t st, bool goct = false);
int occupancy_kernel_entry(int sched, int math, bool lds, bool stats, bool bofs, size_t smem, bool goct = false,
                           bool fused = true);
// accumulate the fused frames' radiances into the output (one pixel per lane)
// (`key`: 4 words of per-kernel state for the sky shortcut, zeroed once; accum_key_body)
hipError_t launch_accum_frames(const KernelArgs& a, int math, uint32_t* key, hipStream_t st);
hipError_t launch_accum_frames_shipped(const KernelArgs& a, uint32_t* key, hipStream_t st);
hipError_t launch_pinned_math(int op, const float* a, const float* b, float* out, size_t n, hipStream_t st);
hipError_t launch_pack(const rt_cl_triangle* tris, uint32_t n_tris, float4* pt, float4* ps,
                       const rt_cl_material* mats, uint32_t n_mats, float4* pm, hipStream_t st);

// rt_kernels_shipped.hip: the MathShipped instantiations (own TU: OpenCL-default / and sqrt)
KernelFn pick_shipped(int sched, bool lds, bool stats, bool bofs, bool goct, bool fused);
// the step schedule's entry points are specialised per launch kind (step_body kMode: 1 fused, 2
// per-frame); stats builds and RT_SPECIALIZE_FUSED 0 use the generic body (kMode 0)
#ifndef RT_SPECIALIZE_FUSED
#define RT_SPECIALIZE_FUSED 1
#endif
hipError_t launch_pack_mats_shipped(const rt_cl_material* mats, uint32_t n_mats, float4* pm, hipStream_t st);

}  // namespace rtk
