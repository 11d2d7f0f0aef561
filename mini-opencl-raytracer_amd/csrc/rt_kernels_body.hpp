// rt_kernels_body.hpp -- the hot path on gfx950 (device code, templated on the math policy): camera-ray generation, stack-based BVH
// traversal, Moller-Trumbore triangle test, BRDF bounce loop and gamma accumulation.
//
// Replaces KernelEntry (/root/reference/kernel_bvh.cl:415-456) and everything it calls.
// Written for CDNA4, not translated from the OpenCL source:
//   * one ray per lane of a wave64, persistent waves taking 8x8-pixel chunks from a global
//     counter; the step schedule (default) advances every lane by one BVH node or one
//     triangle per step and shades / refills / accumulates when enough lanes are ready;
//   * the scene is re-packed once per bound scene (rt_capi.cpp: prepare_scene, pack_*):
//     octant-resolved node records (two b128 LDS reads per visit), 48-B triangle records
//     {p1, e1, e2}, 48-B shading records and 64-B material records; staged in LDS when they
//     fit (Cornell), else read from HBM/L2 with the top of the tree staged in LDS;
//   * no traversal stack: the reference's stack walk (push the far child, pop on a miss
//     or after a leaf) is a depth-first order whose child order depends only on the
//     ray's octant, so it is replayed exactly with per-octant skip pointers (8 per
//     node, built on the host): node visits, triangle tests and their order are the
//     reference's, without LDS pushes/pops or the dependent pop latency;
//   * traversal keeps {t, primitive, u, v}; the hit record (position, shading
//     normal, material) is formed once after the walk from the last accepted triangle, which
//     yields the same values as the reference forming it at every accept;
//   * no MFMA: this is branchy, latency-bound traversal.
// Parity: every arithmetic step follows the reference's operation order with
// -ffp-contract=off (the shipped policy fuses exactly the reference's contraction sites, madd); transcendentals/dot/normalize come from the math policy
// (rt_math.hpp).  Hit IDs are indices into the BVH-ordered triangle array, as
// `isect.object - triangles` in the reference.
//
// Included by two translation units: rt_kernels.hip instantiates the pinned and devicelib
// policies, rt_kernels_shipped.hip the shipped policy (a TU of its own because its `/` and
// sqrt are the OpenCL default 2.5/3-ulp forms, a per-TU compiler setting).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/rt_cl_types.h"
#include "rt_kernels.hpp"
#include "rt_math.hpp"

#pragma clang fp contract(off)

// waves per SIMD of the step entry points (devicelib / shipped); occupancy A/B builds override it
#ifndef RT_STEP_DEVICELIB_WAVES
#define RT_STEP_DEVICELIB_WAVES 5
#endif
#ifndef RT_STEP_GLOBAL_WAVES
#define RT_STEP_GLOBAL_WAVES 6  // the same entry points for scenes read from HBM/L2
#endif
#ifndef RT_STEP_GOCT_WAVES
#define RT_STEP_GOCT_WAVES 5  // ... walking their octant records (5: no spills; 6 spills 23 VGPRs)
#endif

namespace rtk {

constexpr float kTwoPi = 6.28318530718f;    // kernel_bvh.cl:4
constexpr float kInvPi = 0.31830988618f;    // kernel_bvh.cl:5
constexpr float kMaxDist = 100000.0f;       // kernel_bvh.cl:7
constexpr float kHitEps = 1.0e-8f;          // kernel_bvh.cl:101


__device__ __forceinline__ F3 load3(const rt_float3& v) { return F3{v.x, v.y, v.z}; }

// ---- RNG: kernel_bvh.cl:57-71 (integer, bit-exact by construction) ---------------------
__device__ __forceinline__ uint32_t frame_hash(uint32_t x) { return 1103515245u * x + 12345u; }
__device__ __forceinline__ float next_rand(uint32_t& s) {
    uint32_t v = s;
    v ^= v >> 16;
    v *= 0x7feb352du;
    v ^= v >> 15;
    v *= 0x846ca68bu;
    v ^= v >> 16;
    s = v;
    // float(v) / float(0xffffffff) == float(v) / 2^32, an exact power-of-two scaling
    return (float)v * 0x1p-32f;
}

struct Ray {
    F3 o, d, inv;
    uint32_t sgn;  // bit i = invDir[i] < 0
};

// kernel_bvh.cl:42-55 after its normalize: invDir and sign of an already normalized direction
template <class M>
__device__ __forceinline__ Ray ray_from_unit(F3 o, F3 d) {
    Ray r;
    r.o = o;
    r.d = d;
    r.inv = F3{M::rcp(d.x), M::rcp(d.y), M::rcp(d.z)};
    r.sgn = (r.inv.x < 0.0f ? 1u : 0u) | (r.inv.y < 0.0f ? 2u : 0u) | (r.inv.z < 0.0f ? 4u : 0u);
    return r;
}

// kernel_bvh.cl:42-55
template <class M>
__device__ __forceinline__ Ray init_ray(F3 o, F3 d) {
    return ray_from_unit<M>(o, normalize<M>(d));
}

// kernel_bvh.cl:386-403
// (px, py) = (gid % W, gid / W), passed in by the callers that already know them.
template <class M>
__device__ __forceinline__ Ray create_ray(uint32_t px, uint32_t py, uint32_t W, uint32_t H, F3 pos, F3 front,
                                          F3 up, float angle, uint32_t& seed) {
    const float invW = M::rcp((float)W);
    const float invH = M::rcp((float)H);
    const float aspect = M::div((float)W, (float)H);
    float x = ((float)px + next_rand(seed)) - 0.5f;
    float y = ((float)py + next_rand(seed)) - 0.5f;
    x = ((2.0f * ((x + 0.5f) * invW) - 1.0f) * angle) * aspect;
    y = -(1.0f - 2.0f * ((y + 0.5f) * invH)) * angle;
    // (2*A - 1 and 1 - 2*B contract to the same bits: 2*A is exact)
    F3 dir = madd<M>(M::cross(front, up), x, up * y) + front;
    return init_ray<M>(pos, normalize<M>(dir));
}

// ---- scene access ------------------------------------------------------------------------
// Global (HBM/L2) scenes: packed node q0 = (bmin.x, bmin.y, bmin.z, bmax.x), q1 = (bmax.y,
// bmax.z, offset, meta), meta = nPrimitives | axis << 16, plus [node][octant] skip pointers.
// LDS scenes: octant-resolved records A[octant][node] = {near.xyz, far.x}, B[octant][node] =
// {far.yz, hit_next, miss_next} (rt_capi.cpp, build_oct_nodes).  Packed triangle: p1, e1, e2 (w unused).
struct SceneView {
    const float4* nodes;    // global path: 64-B node records (bounds, children, 8 skip pointers)
    const float4* tris;     // LDS or global
    const float4* onodes;   // LDS path: octant-resolved node records; global path: the LDS top
    const float4* stris;    // shading record per triangle: {n1, mtlIndex}, {n2, n3.x}, {n3.yz, -, -}
    const float4* smats;    // per material: {diffuse, 1/(alpha+1)}, {specular, alpha^2/pi}, {emission, alpha^2-1}, {roughness, alpha, -, -}
};

constexpr uint32_t kEnd = 0xffffffffu;  // "stack empty": traversal finished (global node records)
// Octant records (LDS scenes): hit_next is the near child (< 2^24) or a leaf code
// count << 24 | first (count 1..127); the walk's END is a sentinel record at index nNodes that
// every ray misses and whose successors are itself (rt_capi.cpp, build_oct_nodes).
constexpr uint32_t kLeafMin = 1u << 24;

// Scene into LDS once per workgroup (when it fits), else read in place.  kGlobalOct: the octant
// records, triangles and shading records of a scene too large for LDS, read from HBM/L2 by the
// LDS path's walk (same record formats, nothing staged).
template <bool kLdsScene, bool kGlobalOct = false>
__device__ __forceinline__ SceneView stage_scene(const KernelArgs& a) {
    extern __shared__ __attribute__((aligned(16))) float4 smem[];
    if (kGlobalOct) return SceneView{nullptr, a.packedTris, a.octNodes, a.shadeTris, a.shadeMats};
    if (kLdsScene) {
        const int tid = threadIdx.x;
        float4* lo = smem;
        float4* lt = lo + a.octRecords;
        float4* ls = lt + 3 * a.nTris;
        float4* lm = ls + 3 * a.nTris;
        for (uint32_t i = tid; i < a.octRecords; i += 256) lo[i] = a.octNodes[i];
        for (uint32_t i = tid; i < 3 * a.nTris; i += 256) lt[i] = a.packedTris[i];
        for (uint32_t i = tid; i < 3 * a.nTris; i += 256) ls[i] = a.shadeTris[i];
        for (uint32_t i = tid; i < 4 * a.nMats; i += 256) lm[i] = a.shadeMats[i];
        __syncthreads();
        return SceneView{nullptr, lt, lo, ls, lm};
    }
    // global scene: the top-of-tree node records into LDS, the rest read from HBM/L2
    const int tid = threadIdx.x;
    for (uint32_t i = tid; i < 4 * a.nTop; i += 256) smem[i] = a.gNodes[i];
    __syncthreads();
    return SceneView{a.gNodes, a.packedTris, smem, a.shadeTris, a.shadeMats};
}

// The step schedule's LDS walk (RT_WALK_ADDR): the octant records staged with their successor words
// turned into LDS byte addresses -- a node word becomes the byte address of the A record of the same
// octant, a leaf code count << 24 | first becomes count << 24 | the byte address of triangle `first`'s
// record, END (each octant's sentinel) kEndWalk, a word that is neither (a walk that reaches it leaves
// the node and triangle steps at once, and is ready to shade: no sentinel visits, no END test per
// decision).  A visit reads its records at the word itself and a triangle step at the leaf word's low
// bits: no address arithmetic on the dependent path (one VALU per node visit).  The dynamic LDS
// of these kernels starts at LDS address 0 (no static __shared__), so a byte address is a byte
// offset into smem.
#ifndef RT_WALK_ADDR
#define RT_WALK_ADDR 1
#endif
__device__ __forceinline__ uint32_t walk_word(uint32_t w, uint32_t octant, const KernelArgs& a) {
    if (w >= kLeafMin) return (w & 0xff000000u) | (a.octRecords * 16u + (w & 0x00ffffffu) * 48u);
    if (w >= a.nNodes) return kEndWalk;
    return (octant * a.octStride + w) * 16u;
}
__device__ __forceinline__ SceneView stage_scene_walk(const KernelArgs& a) {
    extern __shared__ __attribute__((aligned(16))) float4 smem[];
    const int tid = threadIdx.x;
    float4* lo = smem;
    float4* lt = lo + a.octRecords;
    float4* ls = lt + 3 * a.nTris;
    float4* lm = ls + 3 * a.nTris;
    for (uint32_t i = tid; i < a.octRecords; i += 256) {
        float4 r = a.octNodes[i];
        if (i >= a.octB && i < a.octB + 8u * a.octStride) {  // a B record: {far.yz, hit_next, miss_next}
            const uint32_t o = (i - a.octB) / a.octStride;
            r.z = __uint_as_float(walk_word(__float_as_uint(r.z), o, a));
            r.w = __uint_as_float(walk_word(__float_as_uint(r.w), o, a));
        }
        lo[i] = r;
    }
    for (uint32_t i = tid; i < 3 * a.nTris; i += 256) lt[i] = a.packedTris[i];
    for (uint32_t i = tid; i < 3 * a.nTris; i += 256) ls[i] = a.shadeTris[i];
    for (uint32_t i = tid; i < 4 * a.nMats; i += 256) lm[i] = a.shadeMats[i];
    __syncthreads();
    return SceneView{nullptr, lt, lo, ls, lm};
}

// LDS float4s of the scene (the finish queue / pool follow it)
template <bool kLdsScene, bool kGlobalOct = false>
__device__ __forceinline__ uint32_t lds_scene_f4(const KernelArgs& a) {
    return kGlobalOct ? 0u : kLdsScene ? a.octRecords + 6u * a.nTris + 4u * a.nMats : 4u * a.nTop;
}

struct Traversal {
    float t;
    int32_t prim;
    float u, v;
};

// kernel_bvh.cl:156-169 (RayBounds).  max/min here only feed comparisons, where the
// sign of a zero never matters and a NaN operand (0 * inf) must lose -- the fmax/fmin
// hardware forms give the reference result in both math modes.
__device__ __forceinline__ bool ray_bounds(const float4 q0, const float4 q1, const Ray& r,
                                           float t) {
    const float lox = q0.x, loy = q0.y, loz = q0.z, hix = q0.w, hiy = q1.x, hiz = q1.y;
    const float nx = (r.sgn & 1u) ? hix : lox, fx = (r.sgn & 1u) ? lox : hix;
    const float ny = (r.sgn & 2u) ? hiy : loy, fy = (r.sgn & 2u) ? loy : hiy;
    const float nz = (r.sgn & 4u) ? hiz : loz, fz = (r.sgn & 4u) ? loz : hiz;
    float t0 = __builtin_fmaxf(0.0f, (nx - r.o.x) * r.inv.x);
    float t1 = __builtin_fminf(t, (fx - r.o.x) * r.inv.x);
    t0 = __builtin_fmaxf(t0, (ny - r.o.y) * r.inv.y);
    t1 = __builtin_fminf(t1, (fy - r.o.y) * r.inv.y);
    t0 = __builtin_fmaxf(t0, (nz - r.o.z) * r.inv.z);
    t1 = __builtin_fminf(t1, (fz - r.o.z) * r.inv.z);
    return t1 >= t0;
}

// One node visit of kernel_bvh.cl:184-215: returns true when the ray enters a leaf (its
// triangles [first, first + count) are tested next); `next` is the node the walk continues
// at -- the near child of a passed interior node, else the octant's skip pointer.
template <bool kOct>
__device__ __forceinline__ bool node_visit(const SceneView& sc, const KernelArgs& a, uint32_t cur, const Ray& r,
                                           float t, uint32_t& next, uint32_t& first, uint32_t& count) {
    if (kOct) {
        const uint32_t i = __umul24(r.sgn, a.octStride) + cur;
        const float4 A = sc.onodes[i], B = sc.onodes[i + a.octB];
        float t0 = __builtin_fmaxf(0.0f, (A.x - r.o.x) * r.inv.x);
        float t1 = __builtin_fminf(t, (A.w - r.o.x) * r.inv.x);
        t0 = __builtin_fmaxf(t0, (A.y - r.o.y) * r.inv.y);
        t1 = __builtin_fminf(t1, (B.x - r.o.y) * r.inv.y);
        t0 = __builtin_fmaxf(t0, (A.z - r.o.z) * r.inv.z);
        t1 = __builtin_fminf(t1, (B.y - r.o.z) * r.inv.z);
        const uint32_t hn = __float_as_uint(B.z), mn = __float_as_uint(B.w);
        const bool hit = t1 >= t0;
        const bool leaf = hit && hn >= kLeafMin;
        next = (hit && !leaf) ? hn : mn;
        first = hn & 0x00ffffffu;
        count = hn >> 24;
        return leaf;
    }
    // global 64-B record; the first nTop records are read from their LDS copy (one flat load
    // serves both address spaces)
    const float4* nd = (cur < a.nTop ? sc.onodes : sc.nodes) + 4u * cur;
    const float4 q0 = nd[0];
    const float4 q1 = nd[1];
    next = reinterpret_cast<const uint32_t*>(nd + 2)[r.sgn];
    if (ray_bounds(q0, q1, r, t)) {
        const uint32_t c0 = __float_as_uint(q1.z), c1 = __float_as_uint(q1.w);
        const uint32_t axis = c1 >> 30;
        if (axis == 3u) {
            first = c0;
            count = c1 & 0x3fffffffu;
            return true;
        }
        next = ((r.sgn >> axis) & 1u) ? (c1 & 0x3fffffffu) : c0;
    }
    return false;
}

// LDS octant record visit returning the raw hit_next word on entering a leaf.
__device__ __forceinline__ bool oct_visit(const SceneView& sc, const KernelArgs& a, uint32_t cur, const Ray& r,
                                          float t, uint32_t& next, uint32_t& leaf_code) {
    const uint32_t i = __umul24(r.sgn, a.octStride) + cur;
    const float4 A = sc.onodes[i], B = sc.onodes[i + a.octB];
    float t0 = __builtin_fmaxf(0.0f, (A.x - r.o.x) * r.inv.x);
    float t1 = __builtin_fminf(t, (A.w - r.o.x) * r.inv.x);
    t0 = __builtin_fmaxf(t0, (A.y - r.o.y) * r.inv.y);
    t1 = __builtin_fminf(t1, (B.x - r.o.y) * r.inv.y);
    t0 = __builtin_fmaxf(t0, (A.z - r.o.z) * r.inv.z);
    t1 = __builtin_fminf(t1, (B.y - r.o.z) * r.inv.z);
    const uint32_t hn = __float_as_uint(B.z), mn = __float_as_uint(B.w);
    const bool hit = t1 >= t0;
    const bool leaf = hit && hn >= kLeafMin;
    next = (hit && !leaf) ? hn : mn;
    leaf_code = hn;
    return leaf;
}

// LDS walk with the walk word in `cur`: one node visit returning the next word --
// the near child (< 2^24) or the leaf code on a passed box, else the skip pointer -- with the
// skip pointer itself in `skip` (the continuation once a leaf's triangles are done).  One
// compare and one select on the visit's own result: no mask arithmetic between them.
template <bool kBofs>
__device__ __forceinline__ uint32_t oct_step(const SceneView& sc, const KernelArgs& a, uint32_t cur, const Ray& r,
                                             float t, uint32_t& skip) {
    const uint32_t i = __umul24(r.sgn, a.octStride) + cur;
    // kBofs (trees of <= kOctBMaxStride records per plane): the B record at a fixed offset, read
    // with an immediate offset from A's address -- no second address on the dependent path
    const float4 A = sc.onodes[i], B = sc.onodes[i + (kBofs ? kOctB : a.octB)];
    float t0 = __builtin_fmaxf(0.0f, (A.x - r.o.x) * r.inv.x);
    float t1 = __builtin_fminf(t, (A.w - r.o.x) * r.inv.x);
    t0 = __builtin_fmaxf(t0, (A.y - r.o.y) * r.inv.y);
    t1 = __builtin_fminf(t1, (B.x - r.o.y) * r.inv.y);
    t0 = __builtin_fmaxf(t0, (A.z - r.o.z) * r.inv.z);
    t1 = __builtin_fminf(t1, (B.y - r.o.z) * r.inv.z);
    skip = __float_as_uint(B.w);
    return t1 >= t0 ? __float_as_uint(B.z) : __float_as_uint(B.w);
}

// (De-duplicated loads -- one leader lane per distinct record loads it into LDS for the others --
// cut the address unit's busy share 0.835 -> 0.516 but cost 57 % more VALU and an LDS round trip
// per step: bunny proxy 1.24 -> 2.19 ms/frame, profiles/r06/goct_dedup_ab.txt; removed.)
// Scenes read from HBM/L2 (the octant walk over global records): a node or triangle step's loads
// are the work the vector-memory address unit is bound by (bunny proxy: `ta_busy` 0.91).  A step's
// ~40 walking lanes read only ~5 distinct records (camera rays of a tile and its frames walk
// together), and in 11 % of the steps all of them read the same one (profiles/r05/goct_coherence.txt):
// such a step reads it once through the scalar cache (s_load, no address-unit work): bunny proxy
// 1.357 -> 1.351 ms/frame, `TA_TA_BUSY` -5.4 % (profiles/r05/goct_scalar_ab.txt).  (The first active
// lane's record through the scalar cache in every step, the other lanes' by vector loads, cut the
// address unit's wavefronts by 10 % but put the scalar cache's latency on every step: +15 %.)
typedef float sv4f __attribute__((ext_vector_type(4)));
// records at an LDS byte address (the LDS walk's words; the pointer in LDS's own address space, so a
// ds_read at the address itself): a node's A / B record, a triangle's two 16-B reads and one 4-B read
__device__ __forceinline__ sv4f lds_v4_at(uint32_t byte_addr) {
    return *reinterpret_cast<__attribute__((address_space(3))) const sv4f*>((size_t)byte_addr);
}
__device__ __forceinline__ float lds_f32_at(uint32_t byte_addr) {
    return *reinterpret_cast<__attribute__((address_space(3))) const float*>((size_t)byte_addr);
}

// oct_step on byte-address walk words (stage_scene_walk): `cur` is the A record's LDS byte address
template <bool kBofs>
__device__ __forceinline__ uint32_t oct_step_w(const KernelArgs& a, uint32_t cur, const Ray& r, float t,
                                               uint32_t& skip) {
    const sv4f A = lds_v4_at(cur);
    const sv4f B = lds_v4_at(cur + 16u * (kBofs ? kOctB : a.octB));
    float t0 = __builtin_fmaxf(0.0f, (A.x - r.o.x) * r.inv.x);
    float t1 = __builtin_fminf(t, (A.w - r.o.x) * r.inv.x);
    t0 = __builtin_fmaxf(t0, (A.y - r.o.y) * r.inv.y);
    t1 = __builtin_fminf(t1, (B.x - r.o.y) * r.inv.y);
    t0 = __builtin_fmaxf(t0, (A.z - r.o.z) * r.inv.z);
    t1 = __builtin_fminf(t1, (B.y - r.o.z) * r.inv.z);
    skip = __float_as_uint(B.w);
    return t1 >= t0 ? __float_as_uint(B.z) : __float_as_uint(B.w);
}

typedef __attribute__((address_space(4))) const sv4f cv4f;
typedef __attribute__((address_space(4))) const float cf32;

template <bool kBofs>
__device__ __forceinline__ uint32_t oct_step_g(const SceneView& sc, const KernelArgs& a, uint32_t cur, const Ray& r,
                                               float t, uint32_t& skip) {
    const uint32_t i = __umul24(r.sgn, a.octStride) + cur;
    const uint32_t ob = kBofs ? kOctB : a.octB;
    const uint32_t i0 = __builtin_amdgcn_readfirstlane(i);
    const cv4f* cp = (const cv4f*)sc.onodes;
    sv4f A, B;
    if (__ballot(i != i0) == 0ull) {  // every walking lane at one record
        A = cp[i0];
        B = cp[i0 + ob];
    } else {
        A = *reinterpret_cast<const sv4f*>(sc.onodes + i);
        B = *reinterpret_cast<const sv4f*>(sc.onodes + i + ob);
    }
    float t0 = __builtin_fmaxf(0.0f, (A.x - r.o.x) * r.inv.x);
    float t1 = __builtin_fminf(t, (A.w - r.o.x) * r.inv.x);
    t0 = __builtin_fmaxf(t0, (A.y - r.o.y) * r.inv.y);
    t1 = __builtin_fminf(t1, (B.x - r.o.y) * r.inv.y);
    t0 = __builtin_fmaxf(t0, (A.z - r.o.z) * r.inv.z);
    t1 = __builtin_fminf(t1, (B.y - r.o.z) * r.inv.z);
    skip = __float_as_uint(B.w);
    return t1 >= t0 ? __float_as_uint(B.z) : __float_as_uint(B.w);
}

// kernel_bvh.cl:98-153 (RayTriangle), accept test only.  Branch-free: the reference's
// early returns (det, u, v) become one accept predicate (ray_triangle below).  The values computed are the
// ones the reference computes where it reaches them; the rest are discarded.  A wave
// tests ~25 lanes' triangles at once and nearly always has some lane past every early
// return, so the branches saved no arithmetic and cost exec-mask bookkeeping.
struct TriEval {
    float det, u, v, t;
};

template <class M>
__device__ __forceinline__ TriEval tri_eval_v(sv4f a, sv4f b, float c, const Ray& r) {
    const F3 p1{a.x, a.y, a.z}, e1{a.w, b.x, b.y}, e2{b.z, b.w, c};
    const F3 pvec = M::cross(r.d, e2);
    const float det = M::dot(e1, pvec);
    const float inv_det = M::rcp(det);
    const F3 tvec = r.o - p1;
    const float u = M::dot(tvec, pvec) * inv_det;
    const F3 qvec = M::cross(tvec, e1);
    const float v = M::dot(r.d, qvec) * inv_det;
    const float t = M::dot(e2, qvec) * inv_det;
    return TriEval{det, u, v, t};
}

template <class M>
__device__ __forceinline__ TriEval tri_eval(const float4* tri, const Ray& r) {
    // {p1.xyz, e1.x}, {e1.yz, e2.xy}, {e2.z}: two 16-B reads and one 4-B read (pack_tris)
    return tri_eval_v<M>(*reinterpret_cast<const sv4f*>(tri), *reinterpret_cast<const sv4f*>(tri + 1),
                         *reinterpret_cast<const float*>(tri + 2), r);
}

// the same on a scene read from HBM/L2 (oct_step_g): through the scalar cache when every testing
// lane is at one triangle
template <class M>
__device__ __forceinline__ TriEval tri_eval_g(const float4* tris, uint32_t idx, const Ray& r) {
    const uint32_t i0 = __builtin_amdgcn_readfirstlane(idx);
    const cv4f* cp = (const cv4f*)tris;
    sv4f va, vb;
    float vc;
    if (__ballot(idx != i0) == 0ull) {  // every testing lane at one triangle
        va = cp[3u * i0];
        vb = cp[3u * i0 + 1u];
        vc = *((cf32*)(tris + 3u * i0 + 2u));
    } else {
        va = *reinterpret_cast<const sv4f*>(tris + 3u * idx);
        vb = *reinterpret_cast<const sv4f*>(tris + 3u * idx + 1u);
        vc = *reinterpret_cast<const float*>(tris + 3u * idx + 2u);
    }
    return tri_eval_v<M>(va, vb, vc, r);
}

// kUV = false: keep only {t, primitive} during the walk (two fewer live registers); the
// barycentrics of the closest hit are re-evaluated at shading time (hit_uv) from the same
// triangle and ray, which reproduces the accepted values bit for bit.
template <bool kUV = true>
__device__ __forceinline__ void tri_accept(const TriEval& e, int32_t idx, Traversal& h) {
    // The reference's early returns (det < 1e-8, u < 0, u > 1, v < 0, u + v > 1; then t <
    // isect.t) in VALU arithmetic rather than a chain of mask operations: for operands that are
    // not NaN, x < y <=> x - y < 0 exactly (an IEEE difference of distinct floats is never
    // rounded to zero or across it; denormals are kept), and minNum skips NaN operands, which
    // the early returns let through as well ((det < 1e-8 || -det > 1e-8) == det < 1e-8).
    // Rejected when any test fails; otherwise accepted iff t < isect.t.
    const float rej = __builtin_fminf(__builtin_fminf(__builtin_fminf(e.det - kHitEps, e.u),
                                                      __builtin_fminf(1.0f - e.u, e.v)),
                                      1.0f - (e.u + e.v));
    const float closer = rej < 0.0f ? -1.0f : h.t - e.t;
    const bool ok = closer > 0.0f;
    if (ok) {
        h.t = e.t;
        h.prim = idx;
        if (kUV) {
            h.u = e.u;
            h.v = e.v;
        }
    }
}

template <class M, bool kUV = true>
__device__ __forceinline__ void ray_triangle(const float4* tri, int32_t idx, const Ray& r, Traversal& h) {
    tri_accept<kUV>(tri_eval<M>(tri, r), idx, h);
}

template <class M>
__device__ __forceinline__ Traversal with_uv(const SceneView& sc, const Traversal& h, const Ray& r) {
    const TriEval e = tri_eval<M>(sc.tris + 3 * (size_t)(h.prim < 0 ? 0 : h.prim), r);
    return Traversal{h.t, h.prim, e.u, e.v};
}

// kernel_bvh.cl:171-219 (Intersect), replayed with the per-octant skip pointers: visiting
// a node whose box is missed -- or finishing a leaf -- continues at skip[node][octant], the
// node the reference pops next; a passed interior node continues at its near child
// (the second child when sign[axis], kernel_bvh.cl:200-207).
template <class M, bool kOct, bool kStats>
__device__ __forceinline__ Traversal intersect(const SceneView& sc, const KernelArgs& a, const Ray& r,
                                               uint32_t& visits, uint32_t& tests) {
    Traversal h{kMaxDist, -1, 0.0f, 0.0f};
    uint32_t cur = 0;
    const uint32_t end = kOct ? a.nNodes : kEnd;
    while (cur != end) {
        if (kStats) ++visits;
        uint32_t next, first = 0, count = 0;
        if (node_visit<kOct>(sc, a, cur, r, h.t, next, first, count)) {
            for (uint32_t i = 0; i < count; ++i) {
                if (kStats) ++tests;
                ray_triangle<M>(sc.tris + 3 * (size_t)(first + i), (int32_t)(first + i), r, h);
            }
        }
        cur = next;
    }
    return h;
}

// ---- shading: kernel_bvh.cl:74-90, :221-347 ---------------------------------------------
template <class M>
__device__ __forceinline__ void onb(F3 n, F3& s, F3& t) {
    const F3 axis = pm_fabs(n.x) > 0.001f ? F3{0.0f, 1.0f, 0.0f} : F3{1.0f, 0.0f, 0.0f};
    t = normalize<M>(M::cross(axis, n));
    s = M::cross(n, t);
}

struct MatView {
    F3 diffuse, specular, emission;
    // GGX constants of the material, formed once per material by pack_mats with the
    // reference's operations (kernel_bvh.cl:229, :233, :283) from alpha = 2/roughness^2 - 2:
    // 1/(alpha + 1), alpha^2 * (1/pi), alpha^2 - 1
    float inv_a1, a2pi, a2m1;
};

// SampleBrdf (kernel_bvh.cl:294-302) with SampleSpecular (:271-292) and SampleDiffuse
// (:264-269).  G and F of SampleSpecular are dead in the reference and not evaluated.
//
// SampleGGX (:227-239) and SampleHemisphereCosine (:79-90) end in the same expression,
// normalize((s*cos(phi))*sinT + (t*sin(phi))*sinT + n*c), with c = cosTheta (GGX) or
// sqrt(1 - sinThetaSqr) (cosine).  The lane-specific scalars are drawn in a short branch
// and the expensive tail (frame, sin, cos, normalize) is executed once for both kinds of
// lanes -- each lane still performs exactly the reference's operations, in its order.
template <class M>
__device__ __forceinline__ F3 sample_brdf(F3 wo, F3& wi, float& pdf, F3 n, const MatView& m,
                                          uint32_t& seed) {
    const bool spec = next_rand(seed) > 0.5f;
    const float phi = kTwoPi * next_rand(seed);
    float sinT, c;
    if (spec) {
        (void)next_rand(seed);  // `xi`, drawn and unused (kernel_bvh.cl:230)
        const float r = next_rand(seed);
        c = M::pow(r, m.inv_a1);  // cosTheta = pow(r, 1 / (alpha + 1))
        sinT = M::sqrt(M::max(0.0f, madd<M>(-c, c, 1.0f)));
    } else {
        const float s2 = next_rand(seed);
        sinT = M::sqrt(s2);
        c = M::sqrt(1.0f - s2);
    }
    F3 s, t;
    onb<M>(n, s, t);
    float sphi, cphi;
    M::sincos(phi, sphi, cphi);
    const F3 pb = (t * sphi) * sinT;
    const F3 dir = normalize<M>(madd<M>(n, c, madd<M>(s * cphi, sinT, pb)));
    if (spec) {
        const F3 wh = dir;
        const float cosTheta = c;
        wi = madd<M>(wh, 2.0f * M::dot(wo, wh), -wo);  // reflect, :76
        if (M::dot(wi, n) * M::dot(wo, n) < 0.000001f) return f3s(0.0f);
        const float D = M::div(m.a2pi, M::pow2(madd<M>(cosTheta * cosTheta, m.a2m1, 1.0f)));
        pdf = M::div(D * cosTheta, 4.0f * M::max(M::dot(wo, wh), 0.0f));
        const float denom =
            madd<M>(4.0f * M::max(M::dot(wi, n), 0.0f), M::max(M::dot(wo, n), 0.0f), 0.001f);
        return m.specular * M::div(D, denom);
    }
    wi = dir;
    pdf = M::dot(wi, n) * kInvPi;
    return m.diffuse * kInvPi;
}

// kernel_bvh.cl:304-347
template <class M>
__device__ __forceinline__ float light_pixel(const Ray& r, float t, F3 normal, int lightType) {
    const F3 lightPosition{0.0f, -10.0f, 16.0f};
    const F3 lightDirection{-0.5f, 0.4f, -0.1f};
    float intensity = 1.0f, NdotL, attn = 1.0f;
    if (lightType <= 0) {
        NdotL = M::max(M::dot(normal, -lightDirection), 0.0f);
    } else {
        const F3 X = madd<M>(r.d, t, r.o);
        const F3 L = lightPosition - X;
        NdotL = M::max(M::dot(normal, L), 0.0f);
        if (lightType == 1) {
            intensity = 16.0f;
            const float falloff = 0.8f;
            const F3 eye = L - X;
            const float d = M::sqrt(M::dot(eye, eye));
            attn = (float)(1.0 / (double)(falloff * (d * d)));  // `1.0` is a double literal
        }
    }
    return (attn * intensity) * NdotL;
}

struct LaneStats {
    uint32_t rays = 0, visits = 0, tests = 0, hits = 0;
};

// The body of Render's bounce loop after Intersect (kernel_bvh.cl:358-380): radiance and
// beta updates, BRDF sample and the next ray.  Returns false where the reference breaks
// out of the loop (miss, or pdf <= 0 / NaN).
template <class M, bool kStats, bool kScalarRec = false>
__device__ __forceinline__ bool shade_bounce(const Traversal& h, Ray& ray, F3& radiance, F3& beta,
                                             uint32_t& seed, const SceneView& sc, const KernelArgs& a,
                                             LaneStats& st) {
    if (h.prim < 0) {
        radiance = madd<M>(beta, f3s(0.5f * a.skyboxIntensity), radiance);
        return false;
    }
    if (kStats) ++st.hits;
    // hit record of the last accepted triangle (kernel_bvh.cl:142-147), from the packed
    // shading records (bit copies of the normals, mtlIndex and material fields)
    typedef float v4f __attribute__((ext_vector_type(4)));
    typedef float v2f __attribute__((ext_vector_type(2)));
    const float4* rec = sc.stris + 3 * h.prim;
    v4f s1, s2;
    v2f s3;
    // (records in HBM/L2, kScalarRec: a round whose lanes all hit one triangle, or all use one
    // material, reads that record through the scalar cache -- oct_step_g; bunny proxy -0.3 %,
    // profiles/r05/goct_scalar_ab.txt)
    const uint32_t p0 = kScalarRec ? (uint32_t)__builtin_amdgcn_readfirstlane(h.prim) : 0u;
    if (kScalarRec && __ballot((uint32_t)h.prim != p0) == 0ull) {
        const cv4f* cp = (const cv4f*)(sc.stris + 3u * p0);
        s1 = cp[0];
        s2 = cp[1];
        s3 = *((__attribute__((address_space(4))) const v2f*)(sc.stris + 3u * p0 + 2u));
    } else {
        s1 = *reinterpret_cast<const v4f*>(rec);
        s2 = *reinterpret_cast<const v4f*>(rec + 1);
        s3 = *reinterpret_cast<const v2f*>(rec + 2);
    }
    const float w = (1.0f - h.u) - h.v;
    const F3 normal = normalize<M>(
        madd<M>(F3{s1.x, s1.y, s1.z}, w, madd<M>(F3{s2.x, s2.y, s2.z}, h.u, F3{s2.w, s3.x, s3.y} * h.v)));
    const F3 pos = madd<M>(ray.d, h.t, ray.o);
    const uint32_t mi = 4u * __float_as_uint(s1.w);
    v4f m0, m1, m2;
    const uint32_t mi0 = kScalarRec ? __builtin_amdgcn_readfirstlane(mi) : 0u;
    if (kScalarRec && __ballot(mi != mi0) == 0ull) {
        const cv4f* cp = (const cv4f*)(sc.smats + mi0);
        m0 = cp[0];
        m1 = cp[1];
        m2 = cp[2];
    } else {
        m0 = *reinterpret_cast<const v4f*>(sc.smats + mi);
        m1 = *reinterpret_cast<const v4f*>(sc.smats + mi + 1);
        m2 = *reinterpret_cast<const v4f*>(sc.smats + mi + 2);
    }
    MatView m{F3{m0.x, m0.y, m0.z}, F3{m1.x, m1.y, m1.z}, F3{m2.x, m2.y, m2.z}, m0.w, m1.w, m2.w};

    radiance = madd<M>(beta * m.emission, 50.0f, radiance);
    F3 wi = f3s(0.0f);
    float pdf = 0.0f;
    const F3 f = sample_brdf<M>(-ray.d, wi, pdf, normal, m, seed);
    if (pdf <= 0.0f || pdf != pdf) return false;
    const F3 fd = f * M::dot(wi, normal);
    const F3 mul{M::div(fd.x, pdf), M::div(fd.y, pdf), M::div(fd.z, pdf)};
    beta = beta * mul;
    const float lp = light_pixel<M>(ray, h.t, normal, a.lightType);
    radiance = madd<M>(f3s(lp) * m.diffuse, beta, radiance);
    ray = init_ray<M>(madd<M>(wi, 0.01f, pos), wi);
    return true;
}

// kernel_bvh.cl:349-384 (Render)
template <class M, bool kOct, bool kStats>
__device__ __forceinline__ F3 render(const SceneView& sc, Ray ray,
                                     uint32_t& seed, const KernelArgs& a,
                                     int32_t& prim_id, float& prim_t, LaneStats& st) {
    F3 radiance = f3s(0.0f), beta = f3s(1.0f);
    const uint32_t bounces = (uint32_t)a.lightBounces;
    for (uint32_t i = 0; i < bounces; ++i) {
        if (kStats) ++st.rays;
        const Traversal h = intersect<M, kOct, kStats>(sc, a, ray, st.visits, st.tests);
        if (i == 0) {
            prim_id = h.prim;
            prim_t = h.t;
        }
        if (!shade_bounce<M, kStats>(h, ray, radiance, beta, seed, sc, a, st)) break;
    }
    return F3{M::max(radiance.x, 0.0f), M::max(radiance.y, 0.0f), M::max(radiance.z, 0.0f)};
}

// kernel_bvh.cl:449-455: the stored value for radiance `rad` over the stored value `old`
// (frameCount 0: pow(rad, 0.45454545f), `old` unused; else the gamma accumulation).
template <class M>
__device__ __forceinline__ F3 gamma_out(uint32_t frameCount, F3 old, F3 rad) {
    if (frameCount == 0)
        return F3{M::pow(rad.x, 0.45454545f), M::pow(rad.y, 0.45454545f), M::pow(rad.z, 0.45454545f)};
    const float fm1 = (float)(frameCount - 1), fc = (float)frameCount;
    const F3 lin{M::pow(old.x, 2.2f), M::pow(old.y, 2.2f), M::pow(old.z, 2.2f)};
    const F3 num = madd<M>(lin, fm1, rad);
    const F3 acc{M::div(num.x, fc), M::div(num.y, fc), M::div(num.z, fc)};
    return F3{M::pow(acc.x, 0.454545f), M::pow(acc.y, 0.454545f), M::pow(acc.z, 0.454545f)};
}

// write (frameCount 0) or gamma-accumulate one work-item's result
template <class M>
__device__ __forceinline__ void finish_color(const KernelArgs& a, uint32_t gid, F3 rad) {
    F3 old = f3s(0.0f);
    if (a.frameCount != 0) {
        const float4 o = a.result[gid];
        old = F3{o.x, o.y, o.z};
    }
    const F3 out = gamma_out<M>(a.frameCount, old, rad);
    a.result[gid] = make_float4(out.x, out.y, out.z, 0.0f);
}

template <class M>
__device__ __forceinline__ void finish_pixel(const KernelArgs& a, uint32_t gid, F3 rad, int32_t pid,
                                             float pt) {
    finish_color<M>(a, gid, rad);
    if (a.hitIds) {
        a.hitIds[gid] = pid;
        a.hitT[gid] = pt;
    }
}

__device__ __forceinline__ unsigned long long wave_sum(uint32_t v) {
    unsigned long long x = v;
    for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, 64);
    return x;
}

__device__ __forceinline__ void flush_stats(const KernelArgs& a, const LaneStats& st, int lane) {
    const unsigned long long r = wave_sum(st.rays), v = wave_sum(st.visits), t = wave_sum(st.tests),
                             h = wave_sum(st.hits);
    if (lane == 0) {
        atomicAdd(&a.stats[0], r);
        atomicAdd(&a.stats[1], v);
        atomicAdd(&a.stats[2], t);
        atomicAdd(&a.stats[3], h);
    }
}

// ---- the kernel (tile schedule) ------------------------------------------------------------
template <class M, bool kLdsScene, bool kStats>
__global__ __launch_bounds__(256) void kernel_entry(KernelArgs a) {
    const int tid = threadIdx.x;
    const SceneView sc = stage_scene<kLdsScene>(a);

    const F3 camPos{a.camPos[0], a.camPos[1], a.camPos[2]};
    const F3 camFront{a.camFront[0], a.camFront[1], a.camFront[2]};
    const F3 camUp{a.camUp[0], a.camUp[1], a.camUp[2]};
    // tan(0.5f * (45.0f * 3.1415f / 180.0f)), kernel_bvh.cl:392
    const float angle = M::tan(0.5f * (45.0f * 3.1415f / 180.0f));
    const uint32_t fh = frame_hash(a.frameCount);

    const int wave = tid >> 6, lane = tid & 63;
    const uint32_t dx = (uint32_t)((wave & 1) * 8 + (lane & 7));
    const uint32_t dy = (uint32_t)((wave >> 1) * 8 + (lane >> 3));

    LaneStats st;
    for (uint32_t tile = blockIdx.x; tile < a.nTiles; tile += gridDim.x) {
        const uint32_t ty = tile / a.tilesX, tx = tile - ty * a.tilesX;
        const uint32_t x = tx * 16 + dx;
        const uint32_t row = a.rowBegin + ty * 16 + dy;
        const uint64_t g64 = (uint64_t)row * a.width + x;
        if (x >= a.width || g64 < a.gidBegin || g64 >= a.gidEnd) continue;
        const uint32_t gid = (uint32_t)g64;

        uint32_t seed = gid + fh;  // kernel_bvh.cl:445
        const Ray ray = create_ray<M>(x, row, a.width, a.height, camPos, camFront, camUp, angle, seed);
        int32_t pid = -1;
        float pt = 0.0f;
        const F3 rad = render<M, kLdsScene, kStats>(sc, ray, seed, a, pid, pt, st);
        finish_pixel<M>(a, gid, rad, pid, pt);
    }
    if (kStats) flush_stats(a, st, lane);
}

// Work distribution of the persistent schedules (guided self-scheduling): pixels are handed
// out in chunks of whole 8x8 tiles from two global counters -- chunks of a.chunkPixels over the
// first a.chunkSplit pixels, then chunks of a.tailChunk.  Large chunks keep the returning
// atomics per frame low (one counter saturates near 90 per microsecond on MI355X); small
// ones at the end keep the last waves from finishing alone.  Returns false when no work is left.
// fused frames' radiance slots: written once by the render, read once by the accumulation --
// streamed past the caches (nontemporal) where the render reads its scene through them (HBM/L2
// scene path: bunny proxy 1.425 -> 1.404 ms/frame, profiles/r02/nt_rad_ab.txt; the LDS path
// showed no gain for its stores)
typedef float rad_v4f __attribute__((ext_vector_type(4)));
template <bool kNt>
__device__ __forceinline__ void rad_store(float4* p, float x, float y, float z) {
    if (kNt)
        __builtin_nontemporal_store(rad_v4f{x, y, z, 0.0f}, reinterpret_cast<rad_v4f*>(p));
    else
        *p = make_float4(x, y, z, 0.0f);
}
__device__ __forceinline__ float4 rad_load(const float4* p) {
    const rad_v4f v = __builtin_nontemporal_load(reinterpret_cast<const rad_v4f*>(p));
    return make_float4(v.x, v.y, v.z, v.w);
}

// Tail chunks come from a.tailBase on: the end of the bulk region, or -- per-frame launches whose
// first chunks are handed out statically (a.staticFirst, rt_capi.cpp) -- past those chunks
// (kFusedOnly: bodies for fused launches only, which never start statically: the bulk region's end).
// Counter partitions (a.nParts > 1; per-frame launches without a bulk region, rt_capi.cpp): the work
// items split into nParts contiguous ranges, each with its own tail counter on its own 1-KB line, so
// the waves' grabs spread over nParts addresses instead of queueing on one; workgroup b's waves
// belong to partition b % nParts and take chunks there, statically first, then from its counter,
// then -- once it is dry -- from the other partitions' counters.  Partition q's range, the number of
// waves it starts statically and the first work item its counter hands out:
__device__ __forceinline__ void part_range(const KernelArgs& a, uint32_t q, uint32_t total, uint32_t& beg,
                                           uint32_t& end, uint32_t& cbase) {
    beg = min(q * a.partLen, total);
    end = min(beg + a.partLen, total);
    const uint32_t nw = gridDim.x > q ? 4u * ((gridDim.x - q + a.nParts - 1u) / a.nParts) : 0u;
    cbase = min(beg + nw * a.tailChunk, end);
}
__device__ __forceinline__ bool next_chunk_parts(const KernelArgs& a, uint32_t total, uint32_t lane,
                                                 uint32_t& base, uint32_t& len) {
    const uint32_t p0 = blockIdx.x & (a.nParts - 1u);
    for (uint32_t k = 0; k < a.nParts; ++k) {
        const uint32_t q = (p0 + k) & (a.nParts - 1u);
        uint32_t beg, end, cbase;
        part_range(a, q, total, beg, end, cbase);
        uint32_t* ctr = a.workCounter + kPartStride * q + 1u;
        uint32_t b = 0;
        if (k > 0) {
            // another partition: skip it when its counter is already past its end (a plain read; a
            // stale value is smaller, and only costs the atomic below)
            if (lane == 0) b = __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            b = __shfl(b, 0, 64);
            if (cbase + b >= end) continue;
        }
        if (lane == 0) b = atomicAdd(ctr, a.tailChunk);
        b = __shfl(b, 0, 64) + cbase;
        if (b < end) {
            base = b;
            len = min(a.tailChunk, end - b);
            return true;
        }
    }
    return false;
}

template <bool kFusedOnly>
__device__ __forceinline__ bool next_chunk(const KernelArgs& a, uint32_t total, uint32_t lane, uint32_t& base,
                                           uint32_t& len, bool& tail) {
    if (!kFusedOnly && a.nParts > 1u) return next_chunk_parts(a, total, lane, base, len);
    uint32_t b = 0;
    if (!tail) {
        if (lane == 0) b = atomicAdd(&a.workCounter[0], a.chunkPixels);
        b = __shfl(b, 0, 64);
        if (b < a.chunkSplit) {
            base = b;
            len = min(a.chunkPixels, a.chunkSplit - b);
            return true;
        }
        tail = true;  // this wave never asks the bulk counter again
    }
    if (lane == 0) b = atomicAdd(&a.workCounter[1], a.tailChunk);
    b = __shfl(b, 0, 64) + (kFusedOnly ? a.chunkSplit : a.tailBase);
    if (b >= total) return false;
    base = b;
    len = min(a.tailChunk, total - b);
    return true;
}

// ---- step schedule: a per-wave state machine ------------------------------------------------
// Every lane is in one of four states:
//   IDLE  -- no path; refilled (new pixel -> camera ray) when enough lanes are idle
//   TRAV  -- at BVH node `cur`: one RayBounds per step (kernel_bvh.cl:184-215)
//   LEAF  -- inside a passing leaf: ONE RayTriangle per step, in the leaf's order
//   SHADE -- traversal finished; shaded when enough lanes are ready (kernel_bvh.cl:358-380)
//   DONE  -- path finished; its pixel is accumulated (kernel_bvh.cl:449-455) together with
//            the refill, so that code also runs with many lanes
// Each step advances every TRAV/LEAF lane by one node or one triangle, so a wave no longer
// runs a 4-triangle leaf loop for the few lanes that happen to sit at a leaf, and the heavy
// per-bounce (shading) and per-path (accumulate + next camera ray) code runs with many lanes
// at once.  Per lane the sequence of node visits and triangle tests -- and therefore every
// t, hit and pixel -- is exactly the reference's.
constexpr uint32_t kIdle = 0, kTrav = 1, kLeaf = 2, kShade = 3, kDone = 4;
constexpr uint32_t kNotWalking = 0x80000000u;  // LDS path walk word outside TRAV
// (A speculative walk -- a lane passing a leaf walks on to the next leaf while its triangles wait
// -- was built and measured slower in round 4: 0.824 vs 0.767 ms/frame on the 4K Cornell
// headline; removed in round 5, its record is profiles/r04/spec_walk_ab.txt.)

__device__ __forceinline__ uint32_t lane_rank(unsigned long long m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// Finish queue: the gamma accumulation (kernel_bvh.cl:449-455, six pow per pixel) of
// finished paths runs 64 pixels at a time instead of with the few lanes whose paths
// happen to end in a refill round.  Pixels are independent and each is written once per
// launch, so the order of finishing does not matter.
constexpr uint32_t kFinishSlots = 64;
static_assert(kFinishWaveBytes == kFinishSlots * 16, "finish queue layout");

template <class M>
__device__ __forceinline__ void finish_queued(const KernelArgs& a, const float4* fq, uint32_t n, uint32_t lane) {
    if (lane < n) {
        const float4 e = fq[lane];
        finish_color<M>(a, __float_as_uint(e.w), F3{e.x, e.y, e.z});
    }
}
// steps of the chosen kind per scheduling decision (thresholds are re-checked after each
// burst): the per-step ballots and threshold tests cost about as much as a node visit
#ifndef RT_PRIO_SHADE
#define RT_PRIO_SHADE 1  // wave priority while shading, finishing and refilling (traversal steps run at 3)
#endif
#ifndef RT_NODE_BURST
#define RT_NODE_BURST 7  // LDS walk (6 before work stealing; 5 / 8 slower: profiles/r03/burst_sweep.txt)
#endif
// diagnostic (stats variant, scripts/timeline.py): wave start/end timeline instead of the
// lane-wait counters
#ifndef RT_TIMELINE
#define RT_TIMELINE 0
#endif
#ifndef RT_TIMELINE_DIV
#define RT_TIMELINE_DIV 1
#endif
#ifndef RT_TRI_BURST
#define RT_TRI_BURST 2
#endif
// (The step schedule keeps the accepted triangle's barycentrics during the walk rather than
// re-evaluating them at shading: same bits, 4K Cornell 0.777 -> 0.773, bunny proxy 1.376 -> 1.364
// ms/frame, profiles/r04/keep_uv_ab.txt.  Shading early once few lanes still walk lost 2.5 %,
// profiles/r04/early_shade_ab.txt: removed in round 5.)


// the same for scenes read from HBM/L2 (global path)
#ifndef RT_GNODE_BURST
#define RT_GNODE_BURST 6
#endif
#ifndef RT_GTRI_BURST
#define RT_GTRI_BURST RT_TRI_BURST
#endif
// ... and for the octant walk over HBM/L2: 5 under the pixel-major order (4: +1.1 %, 6: +0.6 %, 8: +1.0 %,
// 3: +4.6 %; profiles/r05/goct_bursts_weights.txt; round 2's tile-major walk tied 3-5)
#ifndef RT_ONODE_BURST
#define RT_ONODE_BURST 5
#endif
#ifndef RT_OTRI_BURST
#define RT_OTRI_BURST RT_TRI_BURST
#endif


__device__ __forceinline__ uint32_t popc_ballot(bool p) { return (uint32_t)__popcll(__ballot(p)); }

// ---- diagnostic: modelled LDS bank conflicts per read site (RT_LDS_CONFLICTS builds) ----------
// A wave64 LDS read is serviced in fixed lane groups, one LDS cycle per group when conflict-free;
// within a group identical addresses broadcast and every further distinct address on a busy bank
// adds a cycle (MI355X_MICROARCH.md, LDS).  ds_read_b128: 4 groups of 16 lanes, {0-3,12-15,
// 20-27}, {4-11,16-19,28-31} and the same +32; a lane's 16-B slot is (byte address / 16) mod 16.
// ds_read_b32: 2 groups of 32 lanes, bank (byte address / 4) mod 32.  scripts/lds_conflicts.py.
#ifndef RT_LDS_CONFLICTS
#define RT_LDS_CONFLICTS 0
#endif
// distinct keys among the active lanes (wave-uniform); the HBM/L2 walk's coherence counters
__device__ __noinline__ uint32_t distinct_keys(bool act, uint32_t key) {
    const uint32_t lane = threadIdx.x & 63u;
    const unsigned long long am = __ballot(act);
    bool first = act;
    for (uint32_t j = 0; j < 64u; ++j) {
        const uint32_t kj = __shfl(key, (int)j, 64);
        if (((am >> j) & 1ull) && j < lane && kj == key) first = false;
    }
    return (uint32_t)__popcll(__ballot(first));
}
__device__ __forceinline__ uint32_t lds_group(uint32_t l, bool b128) {
    if (!b128) return l >> 5;
    const uint32_t h = l & 31u;
    const bool g0 = h < 4u || (h >= 12u && h < 16u) || (h >= 20u && h < 28u);
    return (l >> 5) * 2u + (g0 ? 0u : 1u);
}
// (ideal, modelled) cycles of one read by the active lanes: `key` identifies the address, `bank`
// its slot (b128) or bank (b32); wave-uniform results
__device__ __noinline__ void lds_model(bool act, uint32_t key, uint32_t bank, bool b128, uint64_t& ideal,
                                       uint64_t& cycles) {
    const uint32_t lane = threadIdx.x & 63u, g = lds_group(lane, b128);
    const unsigned long long am = __ballot(act);
    bool first = act;
    for (uint32_t j = 0; j < 64u; ++j) {
        const uint32_t kj = __shfl(key, (int)j, 64);
        if (((am >> j) & 1ull) && j < lane && lds_group(j, b128) == g && kj == key) first = false;
    }
    const unsigned long long fm = __ballot(first);
    uint32_t cnt = 0;
    for (uint32_t j = 0; j < 64u; ++j) {
        const uint32_t bj = __shfl(bank, (int)j, 64);
        if (((fm >> j) & 1ull) && lds_group(j, b128) == g && bj == bank) ++cnt;
    }
    const uint32_t mine = first ? cnt : 0u;
    uint32_t gmax[4] = {0u, 0u, 0u, 0u};
    for (uint32_t j = 0; j < 64u; ++j) {
        const uint32_t v = __shfl(mine, (int)j, 64);
        const uint32_t gj = lds_group(j, b128);
        gmax[gj] = v > gmax[gj] ? v : gmax[gj];
    }
    for (uint32_t q = 0; q < (b128 ? 4u : 2u); ++q) {
        ideal += gmax[q] ? 1u : 0u;
        cycles += gmax[q];
    }
}

// The next 8x8 tile of work for the calling wave (wave-uniform; returns false when there is none).
// Work stealing within the workgroup: a wave's chunk from the work counter is a {next, end} range
// in LDS (steal[wave], one 64-bit word) it takes its tiles from one at a time; once the counter is
// dry, the wave takes single tiles from its siblings' ranges instead of ending while they still
// hold whole chunks.  64-bit LDS atomics hand out every tile exactly once, whoever takes it, so
// the results cannot change (seeds follow the work item, kernel_bvh.cl:445).  Emulated N = 8 rank
// step -4 %, per-frame 4K launches -5 % (profiles/r03/steal_ab.txt).
template <bool kFusedOnly>
__device__ __forceinline__ bool take_tile(const KernelArgs& a, unsigned long long* steal, uint32_t me, uint32_t lane,
                                          uint32_t total, uint32_t& chunk_base, uint32_t& chunk_len, bool& chunk_tail,
                                          bool& dry, uint32_t& unit) {
    if (!dry) {
        unsigned long long old = 0;
        if (lane == 0) old = atomicAdd(&steal[me], 64ull);
        old = __shfl(old, 0, 64);
        if ((uint32_t)old < (uint32_t)(old >> 32)) {
            unit = (uint32_t)old;
            return true;
        }
        if (next_chunk<kFusedOnly>(a, total, lane, chunk_base, chunk_len, chunk_tail)) {
            if (lane == 0)
                (void)atomicExch(&steal[me], ((unsigned long long)(chunk_base + chunk_len) << 32) |
                                                 (unsigned long long)(chunk_base + 64u));
            unit = chunk_base;
            return true;
        }
        dry = true;
    }
    for (uint32_t k = 1; k < 4u; ++k) {
        unsigned long long old = 0;
        if (lane == 0) old = atomicAdd(&steal[(me + k) & 3u], 64ull);
        old = __shfl(old, 0, 64);
        if ((uint32_t)old < (uint32_t)(old >> 32)) {
            unit = (uint32_t)old;
            return true;
        }
    }
    return false;
}

// kMode: 0 -- one body for both launch kinds (fused frames when a.radBuf is set); 1 -- fused
// launches only (rtEnqueueKernelFrames); 2 -- per-frame launches only.  The specialised bodies
// leave out the other kind's code (finish queue, sky key, frame slots), which otherwise holds
// registers in the hot loop (52 SGPRs spilled to VGPR lanes in the generic body).
template <class M, bool kLdsScene, bool kStats, bool kBofs = false, bool kGlobalOct = false, int kMode = 0>
__device__ __forceinline__ void step_body(const KernelArgs& a) {
    const int tid = threadIdx.x;
    // scenes read from HBM/L2: the render's waves issue ahead of co-resident accumulation waves
    // (second stream), which then only fill the slots the render leaves idle (bunny proxy -1.5 %;
    // profiles/r01/render_priority_ab.txt); traversal steps raise it further (below)
    if (!kLdsScene) __builtin_amdgcn_s_setprio(1);
    // frames fused into this launch (rtEnqueueKernelFrames): work item = (frame slot, pixel);
    // a finished path stores its radiance in radBuf[slot][gid] for accum_frames, and the lane's
    // `gid` register then holds slot * radStride + gid
    const bool fused = kMode == 1 ? true : kMode == 2 ? false : a.radBuf != nullptr;
    // the waves' remaining chunks (work stealing, take_tile): empty ranges before anyone looks
    unsigned long long* steal = nullptr;
    {
        extern __shared__ __attribute__((aligned(16))) float4 smem_s[];
        constexpr bool kRingLds = kLdsScene && !kGlobalOct;
        steal = reinterpret_cast<unsigned long long*>(
            smem_s + lds_scene_f4<kLdsScene, kGlobalOct>(a) + (fused ? 0u : 4u * kFinishSlots) +
            (kRingLds ? 4u * (fused ? kRingWaveBytes / 16u : kRingWaveBytesPf / 16u) : 0u));
        // published by stage_scene's barrier (or the one below).  a.staticFirst (launches without
        // a bulk region, rt_capi.cpp): each wave starts with its own tail chunk -- chunk (global wave
        // index) -- as its range, taken with no atomic: every resident wave asks for work at once
        // when a launch starts, and one address's returning atomics serialise at the L2
        // (1080p 2-bounce frames 0.282 -> 0.235 ms alone, profiles/r06/work_handout_ab.txt).  The
        // tail counter then hands out from past these chunks (a.tailBase): every work item is still
        // handed out exactly once.
        if (tid < 4) {
            unsigned long long r = 0ull;
            if (!fused && a.staticFirst) {
                const uint32_t tot = a.nTiles * 64u * (fused ? a.nFrames : 1u);
                uint32_t beg = 0, end = tot, wi = blockIdx.x * 4u + (uint32_t)tid;
                if (a.nParts > 1u) {  // counter partitions: the wave's index among its partition's
                    uint32_t cb;
                    part_range(a, blockIdx.x & (a.nParts - 1u), tot, beg, end, cb);
                    wi = (blockIdx.x / a.nParts) * 4u + (uint32_t)tid;
                }
                const uint32_t b0 = beg + wi * a.tailChunk;
                if (b0 < end) r = ((unsigned long long)min(b0 + a.tailChunk, end) << 32) | b0;
            }
            steal[tid] = r;
        }
    }
    // per-frame launches alternate between two counter slots: this launch zeroes the one the next
    // launch takes (same stream, so that launch sees it) instead of a clearing launch in front of
    // each render (rt_capi.cpp)
    // (every partition's words, whatever this launch uses: the next launch on that slot may use more)
    if (!fused && a.workCounterClear && blockIdx.x == 0 && (uint32_t)tid < 2u * kMaxParts)
        a.workCounterClear[kPartStride * ((uint32_t)tid >> 1) + ((uint32_t)tid & 1u)] = 0u;
    // the LDS walk on byte-address walk words (stage_scene_walk); kEndW the END word, rootW(sgn) the
    // root's word for a ray's octant
    constexpr bool kWalk = RT_WALK_ADDR && kLdsScene && !kGlobalOct;
    const SceneView sc = kWalk ? stage_scene_walk(a) : stage_scene<kLdsScene, kGlobalOct>(a);
    // END as a word that is neither a node nor a leaf (kEndWalk): the byte-address LDS walk and the octant
    // walk over HBM/L2 (whose END links the host writes so, a.nNodes = kEndWalk): a walk at END is
    // ready to shade, with no sentinel visits (no sentinel loads on the HBM/L2 walk) and no END test
    constexpr bool kEndWord = kWalk || (kGlobalOct && RT_GOCT_END_WORD);
    const uint32_t kEndW = kEndWord ? kEndWalk : a.nNodes;
    const uint32_t octStride16 = a.octStride * 16u;
    auto rootW = [&](uint32_t sgn) -> uint32_t { return kWalk ? __umul24(sgn, octStride16) : 0u; };
    if (kGlobalOct) __syncthreads();  // (stage_scene stages nothing for this walk)

    const F3 camPos{a.camPos[0], a.camPos[1], a.camPos[2]};
    const F3 camFront{a.camFront[0], a.camFront[1], a.camFront[2]};
    const F3 camUp{a.camUp[0], a.camUp[1], a.camUp[2]};
    const float angle = M::tan(0.5f * (45.0f * 3.1415f / 180.0f));  // kernel_bvh.cl:392
    const uint32_t bounces = (uint32_t)a.lightBounces;
    const uint32_t total = a.nTiles * 64u * (fused ? a.nFrames : 1u);
    // the radiance of a primary miss, max(1 * 0.5*skybox + 0, 0) per component (kernel_bvh.cl:360, :383)
    const float krad = M::max(madd<M>(1.0f, 0.5f * a.skyboxIntensity, 0.0f), 0.0f);
    // per-frame launches: a finished path with radiance (K_rad, K_rad, K_rad) over a stored value
    // of (K_old, K_old, K_old) gets gamma_out(frameCount, K_old, K_rad), computed once per wave
    // here -- the same operations on the same bits as finish_color -- instead of 6 pow in the
    // finish queue (56 % of the 16:9 Cornell view is sky).  Bit equality decides, so the key
    // chain (launch to launch, pfKeyIn -> pfKeyOut) only affects how often the shortcut applies.
    float k_old = 0.0f, k_out = 0.0f;
    if (!fused && a.pfKeyIn) {
        k_old = __uint_as_float(*a.pfKeyIn);
        // three equal components; wave-uniform, kept in scalar registers
        k_out = __uint_as_float(__builtin_amdgcn_readfirstlane(
            __float_as_uint(gamma_out<M>(a.frameCount, f3s(k_old), f3s(krad)).x)));
        if (blockIdx.x == 0 && tid == 0) *a.pfKeyOut = __float_as_uint(k_out);
    }
    const uint32_t rowEnd = a.rowBegin + a.rowCount;
    const int lane = tid & 63;
    const uint32_t kRefillMin = a.refillMin;  // finish + refill when this many lanes are free
    const uint32_t kShadeMin = a.shadeMin;    // shade when this many lanes are ready

    // per-wave finish queue in LDS (after the scene): {radiance, gid} of finished paths
    extern __shared__ __attribute__((aligned(16))) float4 smem[];
    float4* fq = smem + lds_scene_f4<kLdsScene, kGlobalOct>(a) + (uint32_t)(tid >> 6) * kFinishSlots;
    uint32_t fq_n = 0;  // wave-uniform
    // LDS scenes: per-wave ring of camera rays, generated one whole 8x8 tile (64 lanes) at a
    // time and handed to idle lanes at refill -- create_ray then runs on full waves instead of
    // on the few lanes a refill serves.  Same rays, same seeds, same pixel order.
    // (not for the octant walk over HBM/L2: bunny proxy 1.572 -> 1.536 ms/frame without it,
    // profiles/r02/goct/ring_ab_bunny.txt)
    constexpr bool kRing = kLdsScene && !kGlobalOct;
    // fused launches also keep {invDir, sign bits} (InitRay's tail, formed at fill) per slot;
    // per-frame launches re-form it at the pop (their finish queue leaves no LDS for it)
    float4* ring_d = smem + lds_scene_f4<kLdsScene, kGlobalOct>(a) + (fused ? 0u : 4u * kFinishSlots) +
                     (uint32_t)(tid >> 6) * (fused ? kRingWaveBytes / 16u : kRingWaveBytesPf / 16u);
    float4* ring_i = ring_d + kRingSlots;
    uint32_t* ring_g = reinterpret_cast<uint32_t*>(ring_d + (fused ? 2u : 1u) * kRingSlots);
    uint32_t rc_head = 0, rc_n = 0;  // wave-uniform: ring entries [rc_head, rc_head + rc_n)
    bool dry = false;                // wave-uniform: the work counter is exhausted

    LaneStats st;
    uint32_t state = kIdle;
    uint32_t gid = 0, seed = 0, bounce = 0;
    Ray ray{};
    F3 radiance = f3s(0.0f), beta = f3s(1.0f);
    Traversal h{kMaxDist, -1, 0.0f, 0.0f};
    // LDS path: `cur` is the walk word -- < 2^24 at node `cur`, count << 24 | first inside a
    // passed leaf (the triangle steps count it down), kNotWalking outside TRAV -- and `leaf_i`
    // the skip pointer a leaf continues at.  Global path: `cur` the node to visit or to continue
    // at after the leaf, `leaf_i` the leaf's next triangle.
    uint32_t cur = kLdsScene ? kNotWalking : 0u;
    uint32_t leaf_i = 0u, leaf_end = 0;
    // fused HBM/L2 octant walks without flags (a.flagTiles 2, the default there): every path
    // stores its radiance, primary misses included, and the accumulation reads every frame -- the
    // flag byte per path is gone (0.45 GB of 32-B partial-line writes per bunny launch)
    // (Per-tile flag words decided at refill measured 1 % slower there: the root visit at refill
    // costs load instructions outside the node bursts, profiles/r04/goct_flags.txt.)
    const bool kNoFlags = kGlobalOct && fused && a.flagTiles == 2u;
    // work: chunks of a.chunkPixels pixels (whole 8x8 tiles) from one global counter --
    // one returning atomic per chunk, so the counter stays far from its throughput limit
    uint32_t chunk_base = 0, chunk_len = 0;    // wave-uniform
    bool chunk_tail = a.chunkSplit == 0u;                     // wave-uniform: no bulk region
    bool exhausted = false;                    // wave-uniform
    uint32_t tile_unit = 0, tile_used = 64;    // wave-uniform (HBM/L2 scene paths: the current tile)
    // diagnostic phase timers (stats variant only): shader-clock cycles per phase, per wave
    uint64_t cyc_refill = 0, cyc_trav = 0, cyc_shade = 0;
    const uint64_t cyc_start = kStats ? __builtin_amdgcn_s_memtime() : 0;
#if RT_TIMELINE
    const uint64_t rt_start = __builtin_amdgcn_s_memrealtime();
    uint64_t rt_dry = 0;  // when this wave found the work counter dry
#endif
    // diagnostic lane-utilisation counters (wave-uniform): steps / rounds and lanes served
    [[maybe_unused]] uint64_t u_nsteps = 0, u_nlanes = 0, u_tsteps = 0, u_tlanes = 0, u_srounds = 0, u_slanes = 0,
             u_rrounds = 0, u_rlanes = 0, u_other = 0, u_shadew = 0, u_freew = 0, u_pad = 0;
    // RT_LDS_CONFLICTS: modelled (ideal, actual) LDS cycles per read site -- [0,1] a node visit's A
    // read (its B read has the same addresses + a constant: the same cycles), [2..5] the A read if
    // the octant planes had strides 43, 48 instead, [6,7] a triangle test's 16-B reads (each),
    // [8,9] its 4-B read of e2.z, [10,11] that read from a dense array of e2.z (a float per triangle)
    [[maybe_unused]] uint64_t lm[12] = {};

    for (;;) {
        // ---- finish + refill: accumulate finished paths, start new pixels ----------------------
        uint64_t tA = kStats ? __builtin_amdgcn_s_memtime() : 0;
        const uint32_t n_free = popc_ballot(state == kIdle || state == kDone);
        if (n_free == 64u || (!exhausted && n_free >= kRefillMin)) {
            if (kStats) {
                ++u_rrounds;
                u_rlanes += n_free;
            }
            // finished paths: the gamma accumulation through the finish queue, or (fused
            // frames) the radiance into its frame slot
            if (fused) {
                if (state == kDone) {
                    // a radiance of (K_rad, K_rad, K_rad) -- a primary miss -- is only flagged
                    const bool skyv = __float_as_uint(radiance.x) == __float_as_uint(krad) &&
                                      __float_as_uint(radiance.y) == __float_as_uint(krad) &&
                                      __float_as_uint(radiance.z) == __float_as_uint(krad);
                    // (ray ring: the tile's flags were written when it was generated -- a
                    // path that still ends as K_rad stores its radiance like any other, which
                    // the accumulation reads to the same bits)
                    if (!skyv || kRing || kNoFlags) rad_store<!kLdsScene || kGlobalOct>(a.radBuf + gid, radiance.x, radiance.y, radiance.z);
                    if (!kRing && !kNoFlags) a.frameFlags[gid] = skyv ? 1u : 0u;
                    state = kIdle;
                }
            }
            if (!fused && a.pfKeyIn && state == kDone &&
                __float_as_uint(radiance.x) == __float_as_uint(krad) &&
                __float_as_uint(radiance.y) == __float_as_uint(krad) &&
                __float_as_uint(radiance.z) == __float_as_uint(krad)) {
                bool chain = a.frameCount == 0u;  // frame 0 ignores the stored value
                if (!chain) {
                    const float4 o = a.result[gid];
                    chain = __float_as_uint(o.x) == __float_as_uint(k_old) &&
                            __float_as_uint(o.y) == __float_as_uint(k_old) &&
                            __float_as_uint(o.z) == __float_as_uint(k_old);
                }
                if (chain) {
                    a.result[gid] = make_float4(k_out, k_out, k_out, 0.0f);
                    state = kIdle;
                }
            }
            const unsigned long long done = __ballot(state == kDone);
            if (done != 0ull) {
                const uint32_t nd = (uint32_t)__popcll(done);
                const uint32_t rank = lane_rank(done);
                const uint32_t fit = kFinishSlots - fq_n;
                if (state == kDone) {
                    if (rank < fit) fq[fq_n + rank] = make_float4(radiance.x, radiance.y, radiance.z, __uint_as_float(gid));
                }
                if (nd >= fit) {
                    finish_queued<M>(a, fq, kFinishSlots, lane);
                    if (state == kDone && rank >= fit)
                        fq[rank - fit] = make_float4(radiance.x, radiance.y, radiance.z, __uint_as_float(gid));
                    fq_n = nd - fit;
                } else {
                    fq_n += nd;
                }
                if (state == kDone) state = kIdle;
            }
            while (kRing && !exhausted) {
                const unsigned long long idle = __ballot(state == kIdle);
                if (idle == 0ull) break;
                if (rc_n == 0u) {
                    uint32_t unit = 0;  // the tile's first work item in the work order (wave-uniform)
                    if (!take_tile<kMode == 1>(a, steal, (uint32_t)tid >> 6, (uint32_t)lane, total, chunk_base, chunk_len,
                                   chunk_tail, dry, unit)) {
                        exhausted = true;
#if RT_TIMELINE
                        rt_dry = __builtin_amdgcn_s_memrealtime();
#endif
                        break;
                    }
                    // one 8x8 tile, one work item per lane (chunks are whole tiles)
                    uint32_t tile = unit >> 6;  // wave-uniform
                    const uint32_t slot = fused ? tile / a.nTiles : 0u;  // frame-major (LDS scenes)
                    tile -= slot * a.nTiles;
                    const uint32_t ty = tile / a.tilesX, tx = tile - ty * a.tilesX;
                    const uint32_t x = tx * 8u + ((uint32_t)lane & 7u),
                                   row = a.rowBegin + (ty * a.bandPeriod + a.bandPhase) * 8u + ((uint32_t)lane >> 3);
                    const uint64_t g64 = (uint64_t)row * a.width + x;
                    const bool valid = x < a.width && row < rowEnd && g64 >= a.gidBegin && g64 < a.gidEnd;
                    bool keep = valid;
                    uint32_t sd = 0;
                    Ray cr{};
                    if (valid) {
                        sd = (uint32_t)g64 + frame_hash(a.frameCount + slot);  // kernel_bvh.cl:445
                        cr = create_ray<M>(x, row, a.width, a.height, camPos, camFront, camUp, angle, sd);
                        // fused launches: a camera ray that misses the root box ends its walk at
                        // the first visit -- Intersect finds nothing, the bounce body adds the sky
                        // and breaks (kernel_bvh.cl:358-361), Render returns max(radiance, 0)
                        // (:383) = K_rad: a flagged frame slot.  Decided here, on the whole tile at
                        // once, instead of through a traversal lane, a shading batch and a finish
                        // round (same visit, same bits, same counters; 4K Cornell 1.046 -> 1.013
                        // ms/frame, profiles/r02/sky_early_ab.txt)
                        // Per-frame launches with the sky key: such a pixel gets the key's
                        // gamma step when its stored value follows the chain (else it takes the
                        // ordinary path and the finish queue).
                        if (bounces > 0u && (fused || a.pfKeyIn)) {
                            uint32_t sk;
                            const uint32_t w0 = kWalk ? oct_step_w<kBofs>(a, rootW(cr.sgn), cr, kMaxDist, sk)
                                                      : oct_step<kBofs>(sc, a, 0u, cr, kMaxDist, sk);
                            if (w0 == kEndW) {
                                bool chain = fused || a.frameCount == 0u;
                                if (!chain) {
                                    const float4 o = a.result[(uint32_t)g64];
                                    chain = __float_as_uint(o.x) == __float_as_uint(k_old) &&
                                            __float_as_uint(o.y) == __float_as_uint(k_old) &&
                                            __float_as_uint(o.z) == __float_as_uint(k_old);
                                }
                                if (chain) {
                                    keep = false;
                                    if (kStats) {
                                        ++st.rays;
                                        ++st.visits;
                                    }
                                    if (a.hitIds && slot + 1u == a.nFrames) {
                                        a.hitIds[(uint32_t)g64] = -1;
                                        a.hitT[(uint32_t)g64] = kMaxDist;
                                    }
                                    if (!fused) a.result[(uint32_t)g64] = make_float4(k_out, k_out, k_out, 0.0f);
                                }
                            }
                        }
                    }
                    // fused: the tile's frame flags, all written here, at once, as one 64-bit
                    // word per (frame slot, tile) -- bit = lane, 1: decided as a primary miss
                    // above -- at [unit / 64] (frame-major order: slot * nTiles + tile).  A flag
                    // byte per path written at its end, then 8 flag bytes per tile row here, went
                    // out as partial lines: 4K Cornell writes 0.94 -> 0.81 -> 0.69 GB per launch
                    // (profiles/r03/write_traffic.txt)
                    const unsigned long long skym = __ballot(valid && !keep);
                    if (fused && lane == 0)
                        reinterpret_cast<unsigned long long*>(a.frameFlags)[unit >> 6] = skym;
                    const unsigned long long vm = __ballot(keep);
                    if (keep) {
                        const uint32_t pos = lane_rank(vm);
                        ring_d[pos] = make_float4(cr.d.x, cr.d.y, cr.d.z, __uint_as_float(sd));
                        if (fused) ring_i[pos] = make_float4(cr.inv.x, cr.inv.y, cr.inv.z, __uint_as_float(cr.sgn));
                        ring_g[pos] = (uint32_t)g64 + (fused ? slot * a.radStride : 0u);
                    }
                    rc_head = 0;
                    rc_n = (uint32_t)__popcll(vm);
                    continue;
                }
                const uint32_t rank = lane_rank(idle);
                const uint32_t take = min((uint32_t)__popcll(idle), rc_n);
                if (state == kIdle && rank < take) {
                    const float4 e = ring_d[rc_head + rank];
                    gid = ring_g[rc_head + rank];
                    seed = __float_as_uint(e.w);
                    if (fused) {
                        const float4 iv = ring_i[rc_head + rank];
                        ray.o = camPos;
                        ray.d = F3{e.x, e.y, e.z};
                        ray.inv = F3{iv.x, iv.y, iv.z};
                        ray.sgn = __float_as_uint(iv.w);
                    } else {
                        ray = ray_from_unit<M>(camPos, F3{e.x, e.y, e.z});
                    }
                    radiance = f3s(0.0f);
                    beta = f3s(1.0f);
                    bounce = 0;
                    if (bounces > 0u) {
                        state = kTrav;
                        h = Traversal{kMaxDist, -1, 0.0f, 0.0f};
                        cur = rootW(ray.sgn);
                        if (kStats) ++st.rays;
                    } else {
                        state = kDone;  // no bounce: radiance max(0, 0) = 0
                        const uint32_t slot = fused ? gid / a.radStride : 0u;
                        if (a.hitIds && slot + 1u == a.nFrames) {
                            a.hitIds[gid - slot * a.radStride] = -1;
                            a.hitT[gid - slot * a.radStride] = 0.0f;
                        }
                    }
                }
                rc_head += take;
                rc_n -= take;
            }
            while (!kRing && !exhausted) {
                const unsigned long long idle = __ballot(state == kIdle);
                if (idle == 0ull) break;
                // tile_unit: the current tile's first work item, tile_used of its 64 handed out
                if (tile_used >= 64u) {
                    if (!take_tile<kMode == 1>(a, steal, (uint32_t)tid >> 6, (uint32_t)lane, total, chunk_base, chunk_len,
                                   chunk_tail, dry, tile_unit)) {
                        exhausted = true;
                        break;
                    }
                    tile_used = 0;
                }
                const uint32_t used = tile_used, unit = tile_unit;
                const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(idle >> 32),
                                                                __builtin_amdgcn_mbcnt_lo((uint32_t)idle, 0u));
                const uint32_t take = min((uint32_t)__popcll(idle), 64u - used);  // within one 8x8 tile
                // fused work order: frame-major (all tiles of a frame, then the next: cheap sky
                // tiles and costly tiles mix in every wave), or -- large launches on scenes read
                // from HBM/L2 (a.tileMajor) -- tile-major, a tile's frames back to back for
                // coherent node and triangle fetches (profiles/r01/work_order_ab.txt)
                uint32_t tile = unit >> 6;  // wave-uniform (scalar division)
                uint32_t slot = 0, pblk = 0, lf = 0;
                // pixel-major (a.tileMajor 2; F = 2, 4 or 8 fused frames): a unit is 64 / F pixels of
                // a tile x the F frames -- work item w at frame w % F of the unit's pixel w / F -- so
                // a pixel's frames walk side by side in one wave
                const bool pxMajor = fused && a.tileMajor == 2u;
                if (pxMajor) {
                    lf = (uint32_t)__builtin_ctz(a.nFrames);
                    pblk = tile & (a.nFrames - 1u);
                    tile >>= lf;
                } else if (fused && a.tileMajor) {
                    slot = tile % a.nFrames;
                    tile /= a.nFrames;
                } else if (fused) {
                    slot = tile / a.nTiles;
                    tile -= slot * a.nTiles;
                }
                if (state == kIdle && rank < take) {
                    const uint32_t w = used + rank;  // chunks are whole 8x8 tiles
                    const uint32_t ty = tile / a.tilesX, tx = tile - ty * a.tilesX;
                    uint32_t pix = w;  // pixel in the tile
                    if (pxMajor) {
                        slot = w & (a.nFrames - 1u);
                        pix = (pblk << (6u - lf)) + (w >> lf);
                    }
                    const uint32_t x = tx * 8u + (pix & 7u),
                                   row = a.rowBegin + (ty * a.bandPeriod + a.bandPhase) * 8u + (pix >> 3);
                    const uint64_t g64 = (uint64_t)row * a.width + x;
                    if (x < a.width && row < rowEnd && g64 >= a.gidBegin && g64 < a.gidEnd) {
                        gid = (uint32_t)g64;
                        seed = gid + frame_hash(a.frameCount + slot);  // kernel_bvh.cl:445
                        ray = create_ray<M>(x, row, a.width, a.height, camPos, camFront, camUp, angle, seed);
                        const bool last_frame = slot + 1u == a.nFrames;
                        if (fused) gid += slot * a.radStride;
                        radiance = f3s(0.0f);
                        beta = f3s(1.0f);
                        bounce = 0;
                        if (bounces > 0u) {
                            state = kTrav;
                            h = Traversal{kMaxDist, -1, 0.0f, 0.0f};
                            cur = rootW(ray.sgn);
                            if (kStats) ++st.rays;
                        } else {
                            state = kDone;  // no bounce: radiance max(0, 0) = 0
                            if (a.hitIds && last_frame) {
                                a.hitIds[(uint32_t)g64] = -1;
                                a.hitT[(uint32_t)g64] = 0.0f;
                            }
                        }
                    }
                }
                tile_used += take;
            }
        }
        uint64_t tB = kStats ? __builtin_amdgcn_s_memtime() : 0;
        if (kStats) cyc_refill += tB - tA;
        {
            const uint32_t n_idle = popc_ballot(state == kIdle);
            if (n_idle == 64u) {
                if (exhausted) break;
                continue;
            }
        }

        // ---- traversal steps -----------------------------------------------------------------
        // wave priority by phase: traversal steps (short dependent LDS/VALU chains) issue ahead
        // of waves that shade or refill (long independent VALU runs), which fill the gaps
        // (profiles/r01/phase_priority_ab.txt)
        __builtin_amdgcn_s_setprio(3);
        // Each step is wave-uniform: either a node step (TRAV lanes visit one node) or a
        // triangle step (LEAF lanes test one triangle), chosen by which serves more lanes per
        // instruction (weights ~ the two bodies' VALU cost), so the wave never pays both
        // bodies for a mix of lanes.
        for (;;) {
            uint32_t n_trav, n_leaf;
            if (kLdsScene) {
                // a walk parked on the END sentinel has finished the reference's traversal
                // (kernel_bvh.cl:181-218, stack empty): it is ready to shade
                if (!kEndWord && cur == kEndW) {
                    state = kShade;
                    cur = kNotWalking;
                }
                n_trav = popc_ballot(cur < kLeafMin);
                n_leaf = popc_ballot((int32_t)cur >= (int32_t)kLeafMin);
            } else {
                n_trav = popc_ballot(state == kTrav);
                n_leaf = popc_ballot(state == kLeaf);
            }
            if (n_trav + n_leaf == 0u) break;
            // (the byte-address walk: a walk at END is ready to shade; its state is set at shading)
            if (popc_ballot(kEndWord ? cur == kEndWalk : state == kShade) >= kShadeMin) break;
            if (!exhausted && popc_ballot(state == kIdle || state == kDone) >= kRefillMin) break;
            const bool leaf_step = n_leaf * a.stepWeightNode > n_trav * a.stepWeightLeaf;
            if (kStats) {
                u_shadew += popc_ballot(kEndWord ? cur == kEndWalk : state == kShade);
                u_freew += popc_ballot(state == kIdle || state == kDone);
                u_other += leaf_step ? n_trav : n_leaf;
                if (leaf_step) {
                    ++u_tsteps;
                    u_tlanes += n_leaf;
                } else {
                    ++u_nsteps;
                    u_nlanes += n_trav;
                }
            }
            constexpr int kNodeBurst = kGlobalOct ? RT_ONODE_BURST : kLdsScene ? RT_NODE_BURST : RT_GNODE_BURST;
            constexpr int kTriBurst = kGlobalOct ? RT_OTRI_BURST : kLdsScene ? RT_TRI_BURST : RT_GTRI_BURST;
            if (!leaf_step) {
#pragma unroll
                for (int rep = 0; rep < kNodeBurst; ++rep) {
                    if (kLdsScene) {
                        // one node; a passed leaf leaves its code in `cur` (and the lane out of
                        // the node steps), a walk at END keeps visiting the sentinel (always
                        // missed, its own successor) until the next decision: no per-step
                        // end test, one compare and one select per visit
#if RT_LDS_CONFLICTS
                        if (kStats && !kGlobalOct) {
                            const bool act = cur < kLeafMin;
                            const uint32_t i = kWalk ? cur >> 4 : __umul24(ray.sgn, a.octStride) + cur;
                            lds_model(act, i, i & 15u, true, lm[0], lm[1]);
                            const uint32_t strides[2] = {43u, 48u};
                            for (int v = 0; v < 2; ++v) {
                                const uint32_t iv = ray.sgn * strides[v] + (kWalk ? (cur >> 4) - ray.sgn * a.octStride : cur);
                                lds_model(act, iv, iv & 15u, true, lm[2 + 2 * v], lm[3 + 2 * v]);
                            }
                        }
#endif
#if RT_LDS_CONFLICTS
                        // HBM/L2 octant walk: per node step, active lanes, distinct records, distinct
                        // 128-B lines, steps with one record ([0..3]), steps [8], with <= 2 and <= 4
                        // records [10, 11]; per triangle step [4..7], steps [9]
                        if (kStats && kGlobalOct) {
                            const bool act = cur < kLeafMin;
                            const uint32_t na = popc_ballot(act);
                            if (na) {
                                const uint32_t i = __umul24(ray.sgn, a.octStride) + cur;
                                const uint32_t dk = distinct_keys(act, i);
                                lm[0] += na;
                                lm[1] += dk;
                                lm[2] += distinct_keys(act, i >> 3);
                                lm[3] += dk == 1u;
                                lm[8] += 1u;
                                lm[10] += dk <= 2u;
                                lm[11] += dk <= 4u;
                            }
                        }
#endif
                        if (cur < kLeafMin) {
                            if (kStats && cur != kEndW) ++st.visits;
                            cur = kGlobalOct ? oct_step_g<kBofs>(sc, a, cur, ray, h.t, leaf_i)
                                  : kWalk    ? oct_step_w<kBofs>(a, cur, ray, h.t, leaf_i)
                                             : oct_step<kBofs>(sc, a, cur, ray, h.t, leaf_i);
                        }
                    } else if (state == kTrav) {
                        if (kStats) ++st.visits;
                        uint32_t next, first = 0, count = 0;
                        if (node_visit<false>(sc, a, cur, ray, h.t, next, first, count)) {
                            state = kLeaf;
                            leaf_i = first;
                            leaf_end = first + count;
                        }
                        cur = next;
                        if (state == kTrav && next == kEnd) state = kShade;
                    }
                }
            } else {
#pragma unroll
                for (int rep = 0; rep < kTriBurst; ++rep) {
                    if (kLdsScene) {
                        // one triangle of the leaf; after the last one the lane continues at
                        // the leaf's skip pointer
#if RT_LDS_CONFLICTS
                        if (kStats && !kGlobalOct) {
                            const bool act = (int32_t)cur >= (int32_t)kLeafMin;
                            const uint32_t t4 = kWalk ? (cur & 0x00ffffffu) >> 4 : a.octRecords + 3u * (cur & 0x00ffffffu);  // float4 index
                            lds_model(act, t4, t4 & 15u, true, lm[6], lm[7]);
                            lds_model(act, t4, (4u * (t4 + 2u)) & 31u, false, lm[8], lm[9]);
                            const uint32_t z = 4u * (a.octRecords + 6u * a.nTris + 4u * a.nMats) + (cur & 0x00ffffffu);
                            lds_model(act, t4, z & 31u, false, lm[10], lm[11]);
                        }
#endif
#if RT_LDS_CONFLICTS
                        if (kStats && kGlobalOct) {
                            const bool act = (int32_t)cur >= (int32_t)kLeafMin;
                            const uint32_t na = popc_ballot(act);
                            if (na) {
                                const uint32_t idx = cur & 0x00ffffffu;
                                const uint32_t dk = distinct_keys(act, idx);
                                lm[4] += na;
                                lm[5] += dk;
                                lm[6] += distinct_keys(act, (3u * idx) >> 3);
                                lm[7] += dk == 1u;
                                lm[9] += 1u;
                            }
                        }
#endif
                        if ((int32_t)cur >= (int32_t)kLeafMin) {
                            if (kStats) ++st.tests;
                            const uint32_t idx = cur & 0x00ffffffu;
                            if (kGlobalOct)
                                tri_accept(tri_eval_g<M>(sc.tris, idx, ray), (int32_t)idx, h);
                            else if (kWalk)  // idx: the record's byte address (h.prim too, until shading)
                                tri_accept(tri_eval_v<M>(lds_v4_at(idx), lds_v4_at(idx + 16u), lds_f32_at(idx + 32u), ray), (int32_t)idx, h);
                            else
                                ray_triangle<M>(sc.tris + 3 * idx, (int32_t)idx, ray, h);
                            cur += (kWalk ? 48u : 1u) - kLeafMin;
                            if (cur < kLeafMin) cur = leaf_i;
                        }
                    } else if (state == kLeaf) {
                        if (kStats) ++st.tests;
                        ray_triangle<M>(sc.tris + 3 * (size_t)leaf_i, (int32_t)leaf_i, ray, h);
                        ++leaf_i;
                        if (leaf_i == leaf_end) state = cur == kEnd ? kShade : kTrav;
                    }
                }
            }
        }

        // ---- shading ---------------------------------------------------------------------------
        __builtin_amdgcn_s_setprio(RT_PRIO_SHADE);
        uint64_t tC = kStats ? __builtin_amdgcn_s_memtime() : 0;
        if (kStats) {
            cyc_trav += tC - tB;
            const uint32_t ns = popc_ballot(kEndWord ? cur == kEndWalk : state == kShade);
            if (ns) {
                ++u_srounds;
                u_slanes += ns;
            }
        }
        if (kEndWord ? cur == kEndWalk : state == kShade) {
            if (kWalk && h.prim >= 0)  // the walk's byte address -> the triangle index, (addr - base) / 48
                h.prim = (int32_t)(__umulhi((uint32_t)h.prim - a.octRecords * 16u, 0xAAAAAAABu) >> 5);
            if (bounce == 0u && a.hitIds) {  // primary hit outputs (extension); fused: last frame's
                const uint32_t last = (a.nFrames - 1u) * a.radStride;
                if (!fused || gid >= last) {
                    a.hitIds[gid - (fused ? last : 0u)] = h.prim;
                    a.hitT[gid - (fused ? last : 0u)] = h.t;
                }
            }
            const bool more = shade_bounce<M, kStats, kGlobalOct>(h, ray, radiance, beta, seed, sc, a, st);
            ++bounce;
            if (!more || bounce >= bounces) {
                radiance = F3{M::max(radiance.x, 0.0f), M::max(radiance.y, 0.0f), M::max(radiance.z, 0.0f)};
                state = kDone;
                if (kLdsScene) cur = kNotWalking;
            } else {
                state = kTrav;
                h = Traversal{kMaxDist, -1, 0.0f, 0.0f};
                cur = rootW(ray.sgn);
                if (kStats) ++st.rays;
            }
        }
        if (kStats) cyc_shade += __builtin_amdgcn_s_memtime() - tC;
    }
    finish_queued<M>(a, fq, fq_n, lane);
    if (kStats) {
        flush_stats(a, st, lane);
        if (lane == 0) {
            atomicAdd(&a.stats[4], (unsigned long long)cyc_refill);
            atomicAdd(&a.stats[5], (unsigned long long)cyc_trav);
            atomicAdd(&a.stats[6], (unsigned long long)cyc_shade);
            atomicAdd(&a.stats[7], (unsigned long long)(__builtin_amdgcn_s_memtime() - cyc_start));
#if RT_LDS_CONFLICTS
            // (the lane-utilisation counters' words carry the model instead)
            for (int q = 0; q < 12; ++q) atomicAdd(&a.stats[8 + q], (unsigned long long)lm[q]);
#else
            atomicAdd(&a.stats[8], (unsigned long long)u_nsteps);
            atomicAdd(&a.stats[9], (unsigned long long)u_nlanes);
            atomicAdd(&a.stats[10], (unsigned long long)u_tsteps);
            atomicAdd(&a.stats[11], (unsigned long long)u_tlanes);
            atomicAdd(&a.stats[12], (unsigned long long)u_srounds);
            atomicAdd(&a.stats[13], (unsigned long long)u_slanes);
            atomicAdd(&a.stats[14], (unsigned long long)u_rrounds);
#if RT_TIMELINE
            // diagnostic timeline (100 MHz device clock; scripts/timeline.py): last wave start,
            // first wave start (complemented), last wave end, sum of wave ends, waves, and a
            // wave lifetime histogram (20 us bins) after the hit-id words (the caller sizes that
            // buffer W*H + 64)
            const uint64_t rt_end = __builtin_amdgcn_s_memrealtime();
            atomicMax(&a.stats[15], (unsigned long long)rt_start);
            atomicMax(&a.stats[16], (unsigned long long)~rt_start);
            atomicMax(&a.stats[17], (unsigned long long)rt_end);
            atomicAdd(&a.stats[18], (unsigned long long)rt_end);
            atomicAdd(&a.stats[19], 1ull);
            if (a.hitIds) {
                // lifetime (40 us bins), counter-dry time (40 us bins), end - dry (10 us bins); all
                // RT_TIMELINE_DIV times finer in builds for short launches
                constexpr uint64_t kBin = 4000ull / RT_TIMELINE_DIV, kBinTail = 1000ull / RT_TIMELINE_DIV;
                const uint32_t bin = min((uint32_t)((rt_end - rt_start) / kBin), 63u);
                atomicAdd(&a.hitIds[a.width * a.height + bin], 1);
                const uint64_t dry_at = rt_dry ? rt_dry : rt_end;
                atomicAdd(&a.hitIds[a.width * a.height + 64u + min((uint32_t)((dry_at - rt_start) / kBin), 63u)], 1);
                atomicAdd(&a.hitIds[a.width * a.height + 128u + min((uint32_t)((rt_end - dry_at) / kBinTail), 63u)], 1);
            }
#else
            atomicAdd(&a.stats[15], (unsigned long long)u_rlanes);
            atomicAdd(&a.stats[16], (unsigned long long)u_other);
            atomicAdd(&a.stats[17], (unsigned long long)u_shadew);
            atomicAdd(&a.stats[18], (unsigned long long)u_freew);
            atomicAdd(&a.stats[19], (unsigned long long)u_pad);
#endif
#endif  // RT_LDS_CONFLICTS
        }
    }
}

// rtEnqueueKernelFrames: the gamma accumulation (kernel_bvh.cl:449-455) of frames
// frameCount .. frameCount + nFrames - 1 in order, per pixel, from the radiances the fused step
// launch left in radBuf[slot][gid].  Same pixel set as the step launch (8x8 tiles of the rank's
// bands within the work range), same operations as nFrames per-frame launches.
//
// Sky pixels: a pixel whose every frame was a primary miss has radiance K_rad = max(1*0.5*sky
// + 0, 0) in every component of every frame (kernel_bvh.cl:358-362, :383); if it also held
// K_old, its result is one per-launch constant K_out = chain(K_old; K_rad x nFrames), computed
// once by accum_key (one lane, same policy and operations).  Those pixels are written
// directly; the others are accumulated in place, one 8x8 tile per wave (a per-wave LDS queue of
// several tiles' non-sky pixels, 64 at a time, measured no faster and was removed in round 5).
// The key never affects results, only how often the shortcut applies: K_old chains from the
// previous launch's K_out (the value all-sky pixels then hold).
// Key words: [0] valid, [1] K_rad bits, [2] K_old, [3] K_out.
// a pixel's frame flags (flagTiles 0: a byte per frame and work item)
__device__ __forceinline__ uint32_t load_flags(const KernelArgs& a, uint32_t gid) {
    uint32_t fl = 0;
#pragma unroll
    for (uint32_t s = 0; s < kMaxFusedFrames; ++s)
        if (s < a.nFrames) fl |= (uint32_t)a.frameFlags[(size_t)s * a.radStride + gid] << s;
    return fl;
}
// the same bits from the per-tile words (flagTiles): the tile's F words are wave-uniform loads
__device__ __forceinline__ uint32_t load_tile_flags(const KernelArgs& a, uint32_t tile, uint32_t lane) {
    const unsigned long long* w = reinterpret_cast<const unsigned long long*>(a.frameFlags) + tile;
    uint32_t fl = 0;
#pragma unroll 1
    for (uint32_t s = 0; s < a.nFrames; ++s) fl |= (uint32_t)((w[(size_t)s * a.nTiles] >> lane) & 1ull) << s;
    return fl;
}
// The gamma chain of a pixel's frames (kernel_bvh.cl:449-455 per frame, in order), each frame's
// radiance loaded when its step runs, the six pow of a step one after another (scheduling
// barriers between them): few registers, so the accumulation waves fit beside a running render
// grid (co-resident overlap, rt_capi.cpp).  Same values, same operations, same order.  The loop
// is not unrolled: a gamma step is ~6 ocml pow of ~120 instructions each, and an unrolled 8-frame
// chain made a 17k-instruction kernel whose waves missed the instruction cache.
template <class M>
__device__ __forceinline__ F3 gamma_out_serial(uint32_t frameCount, F3 old, F3 rad) {
    if (frameCount == 0) {
        F3 o;
        o.x = M::pow(rad.x, 0.45454545f);
        __builtin_amdgcn_sched_barrier(0);
        o.y = M::pow(rad.y, 0.45454545f);
        __builtin_amdgcn_sched_barrier(0);
        o.z = M::pow(rad.z, 0.45454545f);
        return o;
    }
    const float fm1 = (float)(frameCount - 1), fc = (float)frameCount;
    float c[3] = {old.x, old.y, old.z};
    const float r[3] = {rad.x, rad.y, rad.z};
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const float lin = M::pow(c[i], 2.2f);
        __builtin_amdgcn_sched_barrier(0);
        c[i] = M::pow(M::div(madd<M>(lin, fm1, r[i]), fc), 0.454545f);
        __builtin_amdgcn_sched_barrier(0);
    }
    return F3{c[0], c[1], c[2]};
}

template <class M>
__device__ __forceinline__ F3 accum_chain_lean(const KernelArgs& a, F3 v, uint32_t gid, uint32_t flags, float krad) {
#pragma unroll 1
    for (uint32_t s = 0; s < a.nFrames; ++s) {
        const float4 r = ((flags >> s) & 1u) ? make_float4(krad, krad, krad, 0.0f)
                                             : rad_load(a.radBuf + (size_t)s * a.radStride + gid);
        v = gamma_out_serial<M>(a.frameCount + s, v, F3{r.x, r.y, r.z});
    }
    return v;
}

// Flagless radiance sets (flagTiles 2) store a primary miss as (K_rad, K_rad, K_rad) like any other
// radiance: the sky shortcut's frame flags are read back from the frames themselves, all set only
// when every frame holds K_rad (a pixel whose old value is not K_old never asks; the first frame
// that is not K_rad ends the scan).  The chain would read the same bits, so the flags change which
// path writes K_out, never a value (1.364 vs 1.357 ms/frame on the bunny proxy without the scan,
// profiles/r04/noflag_skyscan_ab.txt).
__device__ __forceinline__ uint32_t scan_sky_frames(const KernelArgs& a, uint32_t gid, float krad) {
    const uint32_t k = __float_as_uint(krad);
#pragma unroll 1
    for (uint32_t s = 0; s < a.nFrames; ++s) {
        const float4 r = rad_load(a.radBuf + (size_t)s * a.radStride + gid);
        if (__float_as_uint(r.x) != k || __float_as_uint(r.y) != k || __float_as_uint(r.z) != k) return 0u;
    }
    return (1u << a.nFrames) - 1u;
}

template <class M>
__device__ __forceinline__ void accum_key_body(const KernelArgs& a, uint32_t* key) {
    if (threadIdx.x != 0) return;
    // the render this accumulation follows is done with its chunk counters: clear them for the
    // radiance set's next render (rt_capi.cpp launches it after this accumulation)
    if (a.workCounter) {
        a.workCounter[0] = 0u;
        a.workCounter[1] = 0u;
    }
    const float krad = M::max(madd<M>(1.0f, 0.5f * a.skyboxIntensity, 0.0f), 0.0f);
    const float kold = key[0] == 1u ? __uint_as_float(key[3]) : 0.0f;
    F3 v = f3s(kold);
    for (uint32_t s = 0; s < a.nFrames; ++s) v = gamma_out<M>(a.frameCount + s, v, f3s(krad));
    key[1] = __float_as_uint(krad);
    key[2] = __float_as_uint(kold);
    key[3] = __float_as_uint(v.x);  // three equal components: same inputs, same operations
    key[0] = 1u;
}

// a register cap that fits one accumulation wave per SIMD beside the render grid (5 waves of
// 96 VGPRs on the LDS path, 6 of 80 on the global path: 32 of 512 left)
#define RT_ACCUM_OCC __attribute__((amdgpu_num_vgpr(32)))
constexpr uint32_t kAccumWgWaves = 4;  // waves per accumulation workgroup, one 8x8 tile each

template <class M>
__device__ __forceinline__ void accum_frames_body(const KernelArgs& a, const uint32_t* key) {
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    const uint32_t kold = key[2], kout = key[3];
    const float krf = __uint_as_float(key[1]);
    const uint32_t tile = blockIdx.x * kAccumWgWaves + wv;
    if (tile >= a.nTiles) return;  // wave-uniform
    const uint32_t ty = tile / a.tilesX, tx = tile - ty * a.tilesX;
    const uint32_t x = tx * 8u + (lane & 7u), row = a.rowBegin + (ty * a.bandPeriod + a.bandPhase) * 8u + (lane >> 3);
    const uint64_t g64 = (uint64_t)row * a.width + x;
    const bool live = x < a.width && row < a.rowBegin + a.rowCount && g64 >= a.gidBegin && g64 < a.gidEnd;
    if (!live) return;
    const uint32_t gid = (uint32_t)g64;
    float4 o = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    if (a.frameCount != 0u) o = a.result[gid];
    const bool old_sky = a.frameCount == 0u ||
                         (__float_as_uint(o.x) == kold && __float_as_uint(o.y) == kold && __float_as_uint(o.z) == kold);
    const uint32_t fl = a.flagTiles == 1u ? load_tile_flags(a, tile, lane)
                        : a.flagTiles == 2u ? (old_sky ? scan_sky_frames(a, gid, krf) : 0u)
                                            : load_flags(a, gid);
    if (fl == (1u << a.nFrames) - 1u && old_sky) {
        const float v = __uint_as_float(kout);
        a.result[gid] = make_float4(v, v, v, 0.0f);
        return;
    }
    const F3 v = accum_chain_lean<M>(a, F3{o.x, o.y, o.z}, gid, fl, krf);
    a.result[gid] = make_float4(v.x, v.y, v.z, 0.0f);
}

// One packed material record (pack_mats, once per bound scene): the material fields plus the
// GGX constants the reference forms per sample (kernel_bvh.cl:229-231, :223-224, :275) with
// its operations: alpha = 2/roughness^2 - 2 (pow(r, 2.0f) == r*r), 1/(alpha + 1),
// alpha^2 * (1/pi), alpha^2 - 1, with the policy's division.
template <class M>
__device__ __forceinline__ void material_record(const rt_cl_material& m, float4* out) {
    const float alpha = M::div(2.0f, m.roughness * m.roughness) - 2.0f;
    const float a2 = alpha * alpha;
    // the shading step reads the first three 16-B words whole; the fourth is informational
    out[0] = make_float4(m.diffuse.x, m.diffuse.y, m.diffuse.z, M::rcp(alpha + 1.0f));
    out[1] = make_float4(m.specular.x, m.specular.y, m.specular.z, a2 * kInvPi);
    out[2] = make_float4(m.emission.x, m.emission.y, m.emission.z, a2 - 1.0f);
    out[3] = make_float4(m.roughness, alpha, 0.0f, 0.0f);
}

}  // namespace rtk

#include "rt_wavefront.hpp"
