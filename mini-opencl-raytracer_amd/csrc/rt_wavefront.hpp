// rt_wavefront.hpp -- KernelEntry as a wavefront path tracer: separate extend
// (BVH traversal) and shade launches per bounce, with the paths between them in HBM ray queues.
// Included at the end of rt_kernels_body.hpp; instantiated per math policy by the two kernel TUs.
//
// The reference runs one work-item per pixel through its whole bounce loop
// (kernel_bvh.cl:349-384 inside KernelEntry :415-456), so lanes of a wave diverge in traversal
// length and in how many bounces their paths live.  Here one step renders the F fused frames in
// 2 x lightBounces launches:
//   extend(b) -- persistent waves pull the bounce-b rays from the queue (bounce 0: camera rays
//                generated from the work-item index, CreateRay :386-403) and walk the BVH; a lane
//                whose walk ends stores {t, primitive} and takes the next ray at once, so the
//                traversal runs on nearly full waves and needs only the traversal registers
//                (8 waves per SIMD, twice the step schedule's load-latency cover);
//   shade(b)  -- one lane per queued path: the bounce body after Intersect (:358-380, the same
//                shade_bounce as every schedule), then either the path's radiance into its frame
//                slot (miss, pdf break, or the last bounce) or its continuation appended to the
//                bounce-(b+1) queue.
// Per path the node visits, triangle tests, shading operations and RNG draws are the reference's,
// in its order, so radiance, hit IDs and counters equal the other schedules bit for bit; the
// fused accumulation launch (accum_frames) then applies kernel_bvh.cl:449-455 per frame.
//
// Queue layout (no atomics on the data path).  The work-item space is cut into 64-entry blocks
// (one 8x8 tile of one frame at bounce 0), and block B belongs to stream B % G (G ~ 8 per CU).
// A stream's entries live in blocks v, v + G, v + 2G, ... of each queue, packed from the front:
// entry k of stream v is at position (v + (k / 64) * G) * 64 + k % 64.  The shade launch gives
// each stream to one workgroup, which compacts the continuations of 256 paths at a time through
// an LDS prefix and appends them to the same stream of the next queue -- a stream never holds
// more paths than it did at bounce 0, so positions stay inside the queue, and stream counts
// replace a global queue tail.  Every stream samples the whole image (blocks G apart), so the
// streams stay balanced from bounce to bounce.  The extend launch walks 64-entry units
// (block j of stream v: unit j * G + v) statically over its waves.
#pragma once

namespace rtk {

// fused work item (block B = tile of one frame, lane w of its 8x8 pixels): the same (frame
// slot, pixel) order as the step schedule's fused launches (frame-major, or tile-major)
struct WorkItem {
    uint32_t x, row, gid, slot;
    bool valid;
};
__device__ __forceinline__ WorkItem wf_item(const KernelArgs& a, uint32_t B, uint32_t w) {
    WorkItem it;
    uint32_t tile = B;
    if (a.tileMajor) {
        it.slot = tile % a.nFrames;
        tile /= a.nFrames;
    } else {
        it.slot = tile / a.nTiles;
        tile -= it.slot * a.nTiles;
    }
    const uint32_t ty = tile / a.tilesX, tx = tile - ty * a.tilesX;
    it.x = tx * 8u + (w & 7u);
    it.row = a.rowBegin + (ty * a.bandPeriod + a.bandPhase) * 8u + (w >> 3);
    const uint64_t g64 = (uint64_t)it.row * a.width + it.x;
    it.gid = (uint32_t)g64;
    it.valid = it.x < a.width && it.row < a.rowBegin + a.rowCount && g64 >= a.gidBegin && g64 < a.gidEnd;
    return it;
}

__device__ __forceinline__ uint32_t wf_pos(uint32_t v, uint32_t k, uint32_t G) {
    return (v + (k >> 6) * G) * 64u + (k & 63u);
}

// ---- extend: BVH traversal only -----------------------------------------------------------------
// The step schedule's traversal (node steps / triangle steps in bursts, LDS octant records or
// global node records with the top of the tree in LDS) without its shading, refill or finish
// phases.  Per wave an LDS ring of 64 rays ({o, position}, {d, -}), filled one unit (64 queue
// entries, or one 8x8 tile of camera rays) at a time; free lanes take rays from it.
constexpr uint32_t kWfRingF4 = kWfRingBytes / 16u;  // float4 per wave

template <class M, bool kLdsScene, bool kStats, bool kBofs, bool kGlobalOct = false>
__device__ __forceinline__ void wf_extend_body(const KernelArgs& a, const WfArgs& w) {
    extern __shared__ __attribute__((aligned(16))) float4 smem[];
    const uint32_t tid = threadIdx.x, nthr = blockDim.x;
    SceneView sc;
    uint32_t scene_f4;
    if (kGlobalOct) {
        // octant records and triangles of a scene too large for LDS, read from HBM/L2
        sc = SceneView{nullptr, a.packedTris, a.octNodes, nullptr, nullptr};
        scene_f4 = 0;
    } else if (kLdsScene) {
        float4* lo = smem;
        float4* lt = lo + a.octRecords;
        for (uint32_t i = tid; i < a.octRecords; i += nthr) lo[i] = a.octNodes[i];
        for (uint32_t i = tid; i < 3 * a.nTris; i += nthr) lt[i] = a.packedTris[i];
        sc = SceneView{nullptr, lt, lo, nullptr, nullptr};
        scene_f4 = a.octRecords + 3u * a.nTris;
    } else {
        for (uint32_t i = tid; i < 4 * a.nTop; i += nthr) smem[i] = a.gNodes[i];
        sc = SceneView{a.gNodes, a.packedTris, smem, nullptr, nullptr};
        scene_f4 = 4u * a.nTop;
    }
    // the shade launch of this bounce takes the maximum of its stream counts here
    if (blockIdx.x == 0 && tid == 0) w.outCnt[w.G] = 0u;
    __syncthreads();

    const uint32_t lane = tid & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(blockIdx.x * (nthr >> 6) + (tid >> 6));
    const uint32_t nwaves = gridDim.x * (nthr >> 6);
    const bool first = w.bounce == 0u;
    const uint32_t n_units =
        first ? w.nBlocks : w.G * ((__builtin_amdgcn_readfirstlane(w.inCnt[w.G]) + 63u) >> 6);
    float4* ring = smem + scene_f4 + (tid >> 6) * kWfRingF4;
    const F3 camPos{a.camPos[0], a.camPos[1], a.camPos[2]};
    const F3 camFront{a.camFront[0], a.camFront[1], a.camFront[2]};
    const F3 camUp{a.camUp[0], a.camUp[1], a.camUp[2]};
    const float angle = M::tan(0.5f * (45.0f * 3.1415f / 180.0f));  // kernel_bvh.cl:392

    uint32_t unit = wave;            // wave-uniform: next unit of this wave
    uint32_t rc_head = 0, rc_n = 0;  // wave-uniform: ring entries [rc_head, rc_head + rc_n)
    bool exhausted = false;          // wave-uniform

    LaneStats st;
    Ray ray{};
    Traversal h{kMaxDist, -1, 0.0f, 0.0f};
    uint32_t pos = 0;
    // LDS path: walk word as in step_body (node < 2^24, leaf code, kNotWalking); global path:
    // state kIdle / kTrav / kLeaf / kShade (= walk finished) with cur, leaf_i, leaf_end
    uint32_t state = kIdle;
    uint32_t cur = kLdsScene ? kNotWalking : 0u;
    uint32_t leaf_i = 0u, leaf_end = 0u;

    for (;;) {
        // finished walks: {t, primitive} for the shade launch; the lane is free
        uint32_t n_trav, n_leaf;
        if (kLdsScene) {
            if (cur == a.nNodes) {
                w.hits[pos] = make_float2(h.t, __int_as_float(h.prim));
                cur = kNotWalking;
            }
            n_trav = popc_ballot(cur < kLeafMin);
            n_leaf = popc_ballot((int32_t)cur >= (int32_t)kLeafMin);
        } else {
            if (state == kShade) {
                w.hits[pos] = make_float2(h.t, __int_as_float(h.prim));
                state = kIdle;
            }
            n_trav = popc_ballot(state == kTrav);
            n_leaf = popc_ballot(state == kLeaf);
        }
        if (!exhausted && 64u - (n_trav + n_leaf) >= w.refillMin) {
            // ---- free lanes take rays from the ring; an empty ring loads the next unit ----------
            for (;;) {
                const bool idle = kLdsScene ? cur == kNotWalking : state == kIdle;
                const unsigned long long im = __ballot(idle);
                if (im == 0ull) break;
                if (rc_n == 0u) {
                    bool got = false;
                    while (!got && unit < n_units) {
                        const uint32_t u = unit;
                        unit += nwaves;
                        if (first) {
                            // one 8x8 tile of camera rays, out-of-range pixels compacted away
                            const WorkItem it = wf_item(a, u, lane);
                            const unsigned long long vm = __ballot(it.valid);
                            if (it.valid) {
                                uint32_t sd = it.gid + frame_hash(a.frameCount + it.slot);  // kernel_bvh.cl:445
                                const Ray cr = create_ray<M>(it.x, it.row, a.width, a.height, camPos, camFront, camUp,
                                                             angle, sd);
                                const uint32_t p = lane_rank(vm);
                                ring[2u * p] = make_float4(0.0f, 0.0f, 0.0f, __uint_as_float(u * 64u + lane));
                                ring[2u * p + 1u] = make_float4(cr.d.x, cr.d.y, cr.d.z, 0.0f);
                            }
                            rc_n = (uint32_t)__popcll(vm);
                        } else {
                            const uint32_t j = u / w.G, v = u - j * w.G;
                            const uint32_t c = __builtin_amdgcn_readfirstlane(w.inCnt[v]);
                            rc_n = c > j * 64u ? min(64u, c - j * 64u) : 0u;
                            if (lane < rc_n) {
                                const uint32_t p = (v + j * w.G) * 64u + lane;
                                const float4 r0 = w.inQ[p], r1 = w.inQ[w.cap + p];
                                ring[2u * lane] = make_float4(r0.x, r0.y, r0.z, __uint_as_float(p));
                                ring[2u * lane + 1u] = r1;
                            }
                        }
                        rc_head = 0;
                        got = rc_n != 0u;
                    }
                    if (!got) {
                        exhausted = true;
                        break;
                    }
                }
                const uint32_t rank = lane_rank(im);
                const uint32_t take = min((uint32_t)__popcll(im), rc_n);
                if (idle && rank < take) {
                    const float4 e0 = ring[2u * (rc_head + rank)], e1 = ring[2u * (rc_head + rank) + 1u];
                    pos = __float_as_uint(e0.w);
                    // the tail of InitRay (kernel_bvh.cl:42-55) on the stored unit direction
                    ray = ray_from_unit<M>(first ? camPos : F3{e0.x, e0.y, e0.z}, F3{e1.x, e1.y, e1.z});
                    h = Traversal{kMaxDist, -1, 0.0f, 0.0f};
                    cur = 0u;
                    state = kTrav;
                    if (kStats) ++st.rays;
                }
                rc_head += take;
                rc_n -= take;
            }
            if (kLdsScene) {
                n_trav = popc_ballot(cur < kLeafMin);
                n_leaf = popc_ballot((int32_t)cur >= (int32_t)kLeafMin);
            } else {
                n_trav = popc_ballot(state == kTrav);
                n_leaf = popc_ballot(state == kLeaf);
            }
        }
        if (n_trav + n_leaf == 0u) {
            if (exhausted) break;
            continue;
        }
        // ---- traversal steps (step_body's, kernel_bvh.cl:171-219 per lane) ---------------------
        const bool leaf_step = n_leaf * a.stepWeightNode > n_trav * a.stepWeightLeaf;
        constexpr int kNodeBurst = kLdsScene ? RT_NODE_BURST : RT_GNODE_BURST;
        constexpr int kTriBurst = kLdsScene ? RT_TRI_BURST : RT_GTRI_BURST;
        if (!leaf_step) {
#pragma unroll
            for (int rep = 0; rep < kNodeBurst; ++rep) {
                if (kLdsScene) {
                    if (cur < kLeafMin) {
                        if (kStats && cur != a.nNodes) ++st.visits;
                        cur = oct_step<kBofs>(sc, a, cur, ray, h.t, leaf_i);
                    }
                } else if (state == kTrav) {
                    if (kStats) ++st.visits;
                    uint32_t next, first_tri = 0, count = 0;
                    if (node_visit<false>(sc, a, cur, ray, h.t, next, first_tri, count)) {
                        state = kLeaf;
                        leaf_i = first_tri;
                        leaf_end = first_tri + count;
                    }
                    cur = next;
                    if (state == kTrav && next == kEnd) state = kShade;
                }
            }
        } else {
#pragma unroll
            for (int rep = 0; rep < kTriBurst; ++rep) {
                if (kLdsScene) {
                    if ((int32_t)cur >= (int32_t)kLeafMin) {
                        if (kStats) ++st.tests;
                        const uint32_t idx = cur & 0x00ffffffu;
                        ray_triangle<M, false>(sc.tris + 3 * idx, (int32_t)idx, ray, h);
                        cur += 1u - kLeafMin;
                        if (cur < kLeafMin) cur = leaf_i;
                    }
                } else if (state == kLeaf) {
                    if (kStats) ++st.tests;
                    ray_triangle<M, false>(sc.tris + 3 * (size_t)leaf_i, (int32_t)leaf_i, ray, h);
                    ++leaf_i;
                    if (leaf_i == leaf_end) state = cur == kEnd ? kShade : kTrav;
                }
            }
        }
    }
    if (kStats) flush_stats(a, st, (int)lane);
}

// ---- shade: one lane per queued path --------------------------------------------------------------
// Workgroup g shades streams g, g + gridDim.x, ...: 256 paths per round, continuations compacted
// through an LDS prefix over the workgroup's waves into the same stream of the next queue.
template <class M, bool kStats>
__device__ __forceinline__ void wf_shade_body(const KernelArgs& a, const WfArgs& w) {
    __shared__ uint32_t wsum[16];
    const SceneView sc{nullptr, a.packedTris, nullptr, a.shadeTris, a.shadeMats};
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6, nw = blockDim.x >> 6;
    const bool first = w.bounce == 0u;
    const bool last = w.bounce + 1u >= (uint32_t)a.lightBounces;
    // the radiance of a primary miss (kernel_bvh.cl:360, :383): flagged, not stored
    const float krad = M::max(madd<M>(1.0f, 0.5f * a.skyboxIntensity, 0.0f), 0.0f);
    const uint32_t hit_slot0 = (a.nFrames - 1u) * a.radStride;  // primary hits: the last frame's
    const F3 camPos{a.camPos[0], a.camPos[1], a.camPos[2]};
    const F3 camFront{a.camFront[0], a.camFront[1], a.camFront[2]};
    const F3 camUp{a.camUp[0], a.camUp[1], a.camUp[2]};
    const float angle = M::tan(0.5f * (45.0f * 3.1415f / 180.0f));  // kernel_bvh.cl:392
    LaneStats st;

    for (uint32_t v = blockIdx.x; v < w.G; v += gridDim.x) {
        const uint32_t n = first ? (w.nBlocks > v ? (w.nBlocks - v + w.G - 1u) / w.G : 0u) * 64u
                                 : __builtin_amdgcn_readfirstlane(w.inCnt[v]);
        uint32_t out_n = 0;  // workgroup-uniform
        for (uint32_t base = 0; base < n; base += blockDim.x) {
            const uint32_t k = base + tid;
            const uint32_t p = wf_pos(v, k, w.G);
            bool live = k < n;
            Ray ray{};
            F3 radiance = f3s(0.0f), beta = f3s(1.0f);
            uint32_t seed = 0, path = 0;
            if (live) {
                if (first) {
                    // the camera ray again (cheaper than a queue round trip): same seed, same ray
                    const WorkItem it = wf_item(a, p >> 6, p & 63u);
                    live = it.valid;
                    if (live) {
                        seed = it.gid + frame_hash(a.frameCount + it.slot);  // kernel_bvh.cl:445
                        ray = create_ray<M>(it.x, it.row, a.width, a.height, camPos, camFront, camUp, angle, seed);
                        path = it.gid + it.slot * a.radStride;
                    }
                } else {
                    const float4 r0 = w.inQ[p], r1 = w.inQ[w.cap + p];
                    const float4 p0 = w.inQ[2u * w.cap + p], p1 = w.inQ[3u * w.cap + p];
                    ray.o = F3{r0.x, r0.y, r0.z};
                    ray.d = F3{r1.x, r1.y, r1.z};
                    path = __float_as_uint(r0.w);
                    seed = __float_as_uint(r1.w);
                    beta = F3{p0.x, p0.y, p0.z};
                    radiance = F3{p1.x, p1.y, p1.z};
                }
            }
            bool more = false;
            if (live) {
                const float2 hh = w.hits[p];
                const Traversal hit{hh.x, __float_as_int(hh.y), 0.0f, 0.0f};
                if (first && a.hitIds && path >= hit_slot0) {  // primary hit outputs (extension)
                    a.hitIds[path - hit_slot0] = hit.prim;
                    a.hitT[path - hit_slot0] = hit.t;
                }
                more = shade_bounce<M, kStats>(with_uv<M>(sc, hit, ray), ray, radiance, beta, seed, sc, a, st);
                if (!more || last) {
                    // the path ends: Render's max(radiance, 0) into its frame slot (accum_frames)
                    more = false;
                    radiance = F3{M::max(radiance.x, 0.0f), M::max(radiance.y, 0.0f), M::max(radiance.z, 0.0f)};
                    const bool skyv = __float_as_uint(radiance.x) == __float_as_uint(krad) &&
                                      __float_as_uint(radiance.y) == __float_as_uint(krad) &&
                                      __float_as_uint(radiance.z) == __float_as_uint(krad);
                    if (!skyv) a.radBuf[path] = make_float4(radiance.x, radiance.y, radiance.z, 0.0f);
                    a.frameFlags[path] = skyv ? 1u : 0u;
                }
            }
            // append the continuations to stream v of the next queue (workgroup prefix)
            const unsigned long long m = __ballot(more);
            if (lane == 0u) wsum[wv] = (uint32_t)__popcll(m);
            __syncthreads();
            uint32_t off = out_n, tot = 0;
            for (uint32_t i = 0; i < nw; ++i) {
                const uint32_t c = wsum[i];
                off += i < wv ? c : 0u;
                tot += c;
            }
            __syncthreads();
            if (more) {
                const uint32_t q = wf_pos(v, off + lane_rank(m), w.G);
                w.outQ[q] = make_float4(ray.o.x, ray.o.y, ray.o.z, __uint_as_float(path));
                w.outQ[w.cap + q] = make_float4(ray.d.x, ray.d.y, ray.d.z, __uint_as_float(seed));
                w.outQ[2u * w.cap + q] = make_float4(beta.x, beta.y, beta.z, 0.0f);
                w.outQ[3u * w.cap + q] = make_float4(radiance.x, radiance.y, radiance.z, 0.0f);
            }
            out_n += tot;
        }
        if (!last && tid == 0u) {
            w.outCnt[v] = out_n;
            atomicMax(&w.outCnt[w.G], out_n);
        }
    }
    if (kStats) flush_stats(a, st, (int)lane);
}

// entry points (instantiated per math policy by the TU that owns it: rt_kernels.hip for pinned and
// devicelib, rt_kernels_shipped.hip for shipped).  The extend kernel keeps only traversal state:
// 8 waves per SIMD (64 VGPRs), eight per workgroup so the staged scene is shared by eight.
#ifndef RT_WF_EXTEND_WAVES
#define RT_WF_EXTEND_WAVES 8
#endif
template <class M, bool kLdsScene, bool kStats, bool kBofs, bool kGlobalOct = false>
__global__ __launch_bounds__(kWfExtendThreads) __attribute__((amdgpu_waves_per_eu(RT_WF_EXTEND_WAVES, 8)))
void wf_extend(KernelArgs a, WfArgs w) {
    wf_extend_body<M, kLdsScene, kStats, kBofs, kGlobalOct>(a, w);
}
template <class M, bool kStats>
__global__ __launch_bounds__(kWfShadeThreads) void wf_shade(KernelArgs a, WfArgs w) {
    wf_shade_body<M, kStats>(a, w);
}

template <class M, bool S>
WfKernels wf_pick_s(bool lds, bool bofs, bool goct) {
    WfKernelFn e = lds    ? (bofs ? wf_extend<M, true, S, true> : wf_extend<M, true, S, false>)
                   : goct ? wf_extend<M, true, S, false, true>
                          : wf_extend<M, false, S, false>;
    return WfKernels{e, wf_shade<M, S>};
}
template <class M>
WfKernels wf_pick(bool lds, bool stats, bool bofs, bool goct) {
    return stats ? wf_pick_s<M, true>(lds, bofs, goct) : wf_pick_s<M, false>(lds, bofs, goct);
}

}  // namespace rtk
