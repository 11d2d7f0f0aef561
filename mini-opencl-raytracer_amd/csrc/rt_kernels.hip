// rt_kernels.hip -- the hot path on gfx950: camera-ray generation, stack-based BVH
// traversal, Moller-Trumbore triangle test, BRDF bounce loop and gamma accumulation.
//
// Replaces KernelEntry (/root/reference/kernel_bvh.cl:415-456) and everything it calls.
// Written for CDNA4, not translated from the OpenCL source:
//   * one ray per lane of a wave64; a 256-thread workgroup owns 16x16-pixel tiles
//     (each wave an 8x8 sub-tile, so neighbouring rays share traversal paths) and walks
//     them persistently (grid = resident workgroups), so the scene is staged into LDS
//     once per workgroup, not once per tile;
//   * BVH nodes are re-packed on the device into 32-byte records (two b128 LDS reads)
//     and triangles into 48-byte {p1, e1 = p2-p1, e2 = p3-p1} records (three b128
//     reads); both live in LDS when they fit (Cornell: 4.7 KB), else they are read from
//     HBM/L2 through the same code (global path);
//   * no traversal stack: the reference's stack walk (push the far child, pop on a miss
//     or after a leaf) is a depth-first order whose child order depends only on the
//     ray's octant, so it is replayed exactly with per-octant skip pointers (8 per
//     node, built on the host): node visits, triangle tests and their order are the
//     reference's, without LDS pushes/pops or the dependent pop latency;
//   * traversal keeps only {t, primitive, u, v}; the hit record (position, shading
//     normal, material) is formed once after the walk from the last accepted triangle,
//     which yields the same values as the reference forming it at every accept;
//   * no MFMA: this is branchy, latency-bound traversal.
// Parity: every arithmetic step follows the reference's operation order with
// -ffp-contract=off; transcendentals/dot/normalize come from the math policy
// (rt_math.hpp).  Hit IDs are indices into the BVH-ordered triangle array, as
// `isect.object - triangles` in the reference.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/rt_cl_types.h"
#include "rt_kernels.hpp"
#include "rt_math.hpp"

#pragma clang fp contract(off)

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

// kernel_bvh.cl:42-55
template <class M>
__device__ __forceinline__ Ray init_ray(F3 o, F3 d) {
    Ray r;
    d = normalize<M>(d);
    r.o = o;
    r.d = d;
    r.inv = F3{1.0f / d.x, 1.0f / d.y, 1.0f / d.z};
    r.sgn = (r.inv.x < 0.0f ? 1u : 0u) | (r.inv.y < 0.0f ? 2u : 0u) | (r.inv.z < 0.0f ? 4u : 0u);
    return r;
}

// kernel_bvh.cl:386-403
template <class M>
__device__ __forceinline__ Ray create_ray(uint32_t gid, uint32_t W, uint32_t H, F3 pos, F3 front,
                                          F3 up, float angle, uint32_t& seed) {
    const float invW = 1.0f / (float)W;
    const float invH = 1.0f / (float)H;
    const float aspect = (float)W / (float)H;
    float x = ((float)(gid % W) + next_rand(seed)) - 0.5f;
    float y = ((float)(gid / W) + next_rand(seed)) - 0.5f;
    x = ((2.0f * ((x + 0.5f) * invW) - 1.0f) * angle) * aspect;
    y = -(1.0f - 2.0f * ((y + 0.5f) * invH)) * angle;
    F3 dir = ((M::cross(front, up) * x) + (up * y)) + front;
    return init_ray<M>(pos, normalize<M>(dir));
}

// ---- scene access ------------------------------------------------------------------------
// Packed node: q0 = (bmin.x, bmin.y, bmin.z, bmax.x), q1 = (bmax.y, bmax.z, offset, meta),
// meta = nPrimitives | axis << 16.  Packed triangle: p1, e1, e2 (w unused).
struct SceneView {
    const float4* nodes;    // LDS or global
    const float4* tris;     // LDS or global
    const uint32_t* skips;  // [node][octant]: next node in this octant's DFS order after the subtree
};

constexpr uint32_t kEnd = 0xffffffffu;  // "stack empty": traversal finished

// Scene into LDS once per workgroup (when it fits), else read in place.
template <bool kLdsScene>
__device__ __forceinline__ SceneView stage_scene(const KernelArgs& a) {
    extern __shared__ __attribute__((aligned(16))) float4 smem[];
    if (kLdsScene) {
        const int tid = threadIdx.x;
        float4* ln = smem;
        float4* lt = smem + 2 * a.nNodes;
        float4* lk = lt + 3 * a.nTris;
        const float4* gk = reinterpret_cast<const float4*>(a.skips);
        for (uint32_t i = tid; i < 2 * a.nNodes; i += 256) ln[i] = a.packedNodes[i];
        for (uint32_t i = tid; i < 3 * a.nTris; i += 256) lt[i] = a.packedTris[i];
        for (uint32_t i = tid; i < 2 * a.nNodes; i += 256) lk[i] = gk[i];
        __syncthreads();
        return SceneView{ln, lt, reinterpret_cast<const uint32_t*>(lk)};
    }
    return SceneView{a.packedNodes, a.packedTris, a.skips};
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

// kernel_bvh.cl:98-153 (RayTriangle), accept test only.
template <class M>
__device__ __forceinline__ void ray_triangle(const float4* tri, int32_t idx, const Ray& r,
                                             Traversal& h) {
    const float4 a = tri[0], b = tri[1], c = tri[2];
    const F3 p1{a.x, a.y, a.z}, e1{b.x, b.y, b.z}, e2{c.x, c.y, c.z};
    const F3 pvec = M::cross(r.d, e2);
    const float det = M::dot(e1, pvec);
    if (det < kHitEps) return;  // == (det < 1e-8 || -det > 1e-8); NaN falls through
    const float inv_det = 1.0f / det;
    const F3 tvec = r.o - p1;
    const float u = M::dot(tvec, pvec) * inv_det;
    if (u < 0.0f || u > 1.0f) return;
    const F3 qvec = M::cross(tvec, e1);
    const float v = M::dot(r.d, qvec) * inv_det;
    if (v < 0.0f || u + v > 1.0f) return;
    const float t = M::dot(e2, qvec) * inv_det;
    if (t < h.t) {
        h.t = t;
        h.prim = idx;
        h.u = u;
        h.v = v;
    }
}

// kernel_bvh.cl:171-219 (Intersect), replayed with the per-octant skip pointers: visiting
// a node whose box is missed -- or finishing a leaf -- continues at skip[node][octant], the
// node the reference pops next; a passed interior node continues at its near child
// (the second child when sign[axis], kernel_bvh.cl:200-207).
template <class M, bool kStats>
__device__ __forceinline__ Traversal intersect(const SceneView& sc, const Ray& r, uint32_t& visits,
                                               uint32_t& tests) {
    Traversal h{kMaxDist, -1, 0.0f, 0.0f};
    uint32_t cur = 0;
    while (cur != kEnd) {
        const float4 q0 = sc.nodes[2 * cur];
        const float4 q1 = sc.nodes[2 * cur + 1];
        const uint32_t skip = sc.skips[8 * cur + r.sgn];
        if (kStats) ++visits;
        if (ray_bounds(q0, q1, r, h.t)) {
            const uint32_t off = __float_as_uint(q1.z);
            const uint32_t meta = __float_as_uint(q1.w);
            const uint32_t np = meta & 0xffffu;
            if (np > 0) {
                for (uint32_t i = 0; i < np; ++i) {
                    if (kStats) ++tests;
                    ray_triangle<M>(sc.tris + 3 * (size_t)(off + i), (int32_t)(off + i), r, h);
                }
                cur = skip;
            } else {
                cur = ((r.sgn >> (meta >> 16)) & 1u) ? off : cur + 1;
            }
        } else {
            cur = skip;
        }
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
    float roughness;
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
    float alpha = 0.0f, sinT, c;
    if (spec) {
        alpha = 2.0f / M::pow2(m.roughness) - 2.0f;
        (void)next_rand(seed);  // `xi`, drawn and unused (kernel_bvh.cl:230)
        const float r = next_rand(seed);
        c = M::pow(r, 1.0f / (alpha + 1.0f));  // cosTheta
        sinT = __builtin_sqrtf(M::max(0.0f, 1.0f - c * c));
    } else {
        const float s2 = next_rand(seed);
        sinT = __builtin_sqrtf(s2);
        c = __builtin_sqrtf(1.0f - s2);
    }
    F3 s, t;
    onb<M>(n, s, t);
    const F3 pa = (s * M::cos(phi)) * sinT;
    const F3 pb = (t * M::sin(phi)) * sinT;
    const F3 dir = normalize<M>((pa + pb) + n * c);
    if (spec) {
        const F3 wh = dir;
        const float cosTheta = c;
        wi = (-wo) + wh * (2.0f * M::dot(wo, wh));
        if (M::dot(wi, n) * M::dot(wo, n) < 0.000001f) return f3s(0.0f);
        const float a2 = alpha * alpha;
        const float D = (a2 * kInvPi) / M::pow2(cosTheta * cosTheta * (a2 - 1.0f) + 1.0f);
        pdf = (D * cosTheta) / (4.0f * M::max(M::dot(wo, wh), 0.0f));
        const float denom =
            (4.0f * M::max(M::dot(wi, n), 0.0f)) * M::max(M::dot(wo, n), 0.0f) + 0.001f;
        return m.specular * (D / denom);
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
        const F3 X = r.o + r.d * t;
        const F3 L = lightPosition - X;
        NdotL = M::max(M::dot(normal, L), 0.0f);
        if (lightType == 1) {
            intensity = 16.0f;
            const float falloff = 0.8f;
            const F3 eye = L - X;
            const float d = __builtin_sqrtf(M::dot(eye, eye));
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
template <class M, bool kStats>
__device__ __forceinline__ bool shade_bounce(const Traversal& h, Ray& ray, F3& radiance, F3& beta,
                                             uint32_t& seed, const rt_cl_triangle* __restrict__ tris_full,
                                             const rt_cl_material* __restrict__ mats, const KernelArgs& a,
                                             LaneStats& st) {
    if (h.prim < 0) {
        radiance = radiance + beta * f3s(0.5f * a.skyboxIntensity);
        return false;
    }
    if (kStats) ++st.hits;
    // hit record of the last accepted triangle (kernel_bvh.cl:142-147)
    const rt_cl_triangle& tri = tris_full[h.prim];
    const float w = (1.0f - h.u) - h.v;
    const F3 normal = normalize<M>((load3(tri.v2.normal) * h.u + load3(tri.v3.normal) * h.v) +
                                   load3(tri.v1.normal) * w);
    const F3 pos = ray.o + ray.d * h.t;
    const rt_cl_material& mm = mats[tri.mtlIndex];
    MatView m{load3(mm.diffuse), load3(mm.specular), load3(mm.emission), mm.roughness};

    radiance = radiance + (beta * m.emission) * 50.0f;
    F3 wi = f3s(0.0f);
    float pdf = 0.0f;
    const F3 f = sample_brdf<M>(-ray.d, wi, pdf, normal, m, seed);
    if (pdf <= 0.0f || pdf != pdf) return false;
    const F3 mul = (f * M::dot(wi, normal)) / pdf;
    beta = beta * mul;
    const float lp = light_pixel<M>(ray, h.t, normal, a.lightType);
    radiance = radiance + (f3s(lp) * m.diffuse) * beta;
    ray = init_ray<M>(pos + wi * 0.01f, wi);
    return true;
}

// kernel_bvh.cl:349-384 (Render)
template <class M, bool kStats>
__device__ __forceinline__ F3 render(const SceneView& sc, const rt_cl_triangle* __restrict__ tris_full,
                                     const rt_cl_material* __restrict__ mats, Ray ray,
                                     uint32_t& seed, const KernelArgs& a,
                                     int32_t& prim_id, float& prim_t, LaneStats& st) {
    F3 radiance = f3s(0.0f), beta = f3s(1.0f);
    const uint32_t bounces = (uint32_t)a.lightBounces;
    for (uint32_t i = 0; i < bounces; ++i) {
        if (kStats) ++st.rays;
        const Traversal h = intersect<M, kStats>(sc, ray, st.visits, st.tests);
        if (i == 0) {
            prim_id = h.prim;
            prim_t = h.t;
        }
        if (!shade_bounce<M, kStats>(h, ray, radiance, beta, seed, tris_full, mats, a, st)) break;
    }
    return F3{M::max(radiance.x, 0.0f), M::max(radiance.y, 0.0f), M::max(radiance.z, 0.0f)};
}

// kernel_bvh.cl:449-455: write (frameCount 0) or gamma-accumulate one work-item's result.
template <class M>
__device__ __forceinline__ void finish_pixel(const KernelArgs& a, uint32_t gid, F3 rad, int32_t pid,
                                             float pt) {
    F3 out;
    if (a.frameCount == 0) {
        out = F3{M::pow(rad.x, 0.45454545f), M::pow(rad.y, 0.45454545f), M::pow(rad.z, 0.45454545f)};
    } else {
        const float4 old = a.result[gid];
        const float fm1 = (float)(a.frameCount - 1), fc = (float)a.frameCount;
        const F3 lin{M::pow(old.x, 2.2f), M::pow(old.y, 2.2f), M::pow(old.z, 2.2f)};
        const F3 acc = ((lin * fm1) + rad) / fc;
        out = F3{M::pow(acc.x, 0.454545f), M::pow(acc.y, 0.454545f), M::pow(acc.z, 0.454545f)};
    }
    a.result[gid] = make_float4(out.x, out.y, out.z, 0.0f);
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
        const Ray ray = create_ray<M>(gid, a.width, a.height, camPos, camFront, camUp, angle, seed);
        int32_t pid = -1;
        float pt = 0.0f;
        const F3 rad = render<M, kStats>(sc, a.trisFull, a.materials, ray, seed, a, pid, pt, st);
        finish_pixel<M>(a, gid, rad, pid, pt);
    }
    if (kStats) flush_stats(a, st, lane);
}

// ---- path-regeneration schedule -------------------------------------------------------------
// Same per-pixel computation, different scheduling: every lane of a persistent wave carries
// one path; when a path ends (miss, pdf break, or lightBounces reached) the lane writes its
// pixel and immediately starts the next pixel, taken from the wave's current 64-pixel chunk
// (one 8x8 tile; one global atomic per chunk).  Lanes therefore stay busy across bounces
// instead of idling until the longest path of their tile ends.  Every pixel still runs the
// reference's exact sequence of operations with its own seed, so results are identical.
template <class M, bool kLdsScene, bool kStats>
__global__ __launch_bounds__(256) void kernel_entry_regen(KernelArgs a) {
    const int tid = threadIdx.x;
    const SceneView sc = stage_scene<kLdsScene>(a);

    const F3 camPos{a.camPos[0], a.camPos[1], a.camPos[2]};
    const F3 camFront{a.camFront[0], a.camFront[1], a.camFront[2]};
    const F3 camUp{a.camUp[0], a.camUp[1], a.camUp[2]};
    const float angle = M::tan(0.5f * (45.0f * 3.1415f / 180.0f));  // kernel_bvh.cl:392
    const uint32_t fh = frame_hash(a.frameCount);
    const uint32_t bounces = (uint32_t)a.lightBounces;
    const uint32_t total = a.nTiles * 64u;  // index space: 8x8-pixel tiles, tile-major
    const uint32_t rowEnd = a.rowBegin + a.rowCount;
    const int lane = tid & 63;

    LaneStats st;
    bool active = false;
    uint32_t gid = 0, seed = 0, bounce = 0;
    int32_t pid = -1;
    float pt = 0.0f;
    Ray ray{};
    F3 radiance = f3s(0.0f), beta = f3s(1.0f);
    uint32_t chunk_base = 0, chunk_used = 64;  // wave-uniform
    bool exhausted = false;                    // wave-uniform

    for (;;) {
        // ---- refill idle lanes from the wave's chunk --------------------------------------
        while (!exhausted) {
            const unsigned long long idle = __ballot(!active);
            if (idle == 0ull) break;
            if (chunk_used >= 64u) {
                uint32_t b = 0;
                if (lane == 0) b = atomicAdd(a.workCounter, 64u);
                b = __shfl(b, 0, 64);
                if (b >= total) {
                    exhausted = true;
                    break;
                }
                chunk_base = b;
                chunk_used = 0;
            }
            const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(idle >> 32),
                                                            __builtin_amdgcn_mbcnt_lo((uint32_t)idle, 0u));
            const uint32_t take = min((uint32_t)__popcll(idle), 64u - chunk_used);
            if (!active && rank < take) {
                const uint32_t idx = chunk_base + chunk_used + rank;
                const uint32_t tile = idx >> 6, w = idx & 63u;
                const uint32_t ty = tile / a.tilesX, tx = tile - ty * a.tilesX;
                const uint32_t x = tx * 8u + (w & 7u),
                                   row = a.rowBegin + (ty * a.bandPeriod + a.bandPhase) * 8u + (w >> 3);
                const uint64_t g64 = (uint64_t)row * a.width + x;
                if (x < a.width && row < rowEnd && g64 >= a.gidBegin && g64 < a.gidEnd) {
                    gid = (uint32_t)g64;
                    seed = gid + fh;  // kernel_bvh.cl:445
                    ray = create_ray<M>(gid, a.width, a.height, camPos, camFront, camUp, angle, seed);
                    radiance = f3s(0.0f);
                    beta = f3s(1.0f);
                    bounce = 0;
                    pid = -1;
                    pt = 0.0f;
                    if (bounces > 0u) {
                        active = true;
                    } else {
                        finish_pixel<M>(a, gid, f3s(0.0f), pid, pt);  // no bounce: radiance 0
                    }
                }
            }
            chunk_used += take;
        }
        if (__ballot(active) == 0ull) {
            if (exhausted) break;
            continue;
        }
        // ---- one bounce of every live path -------------------------------------------------
        if (active) {
            if (kStats) ++st.rays;
            const Traversal h = intersect<M, kStats>(sc, ray, st.visits, st.tests);
            if (bounce == 0u) {
                pid = h.prim;
                pt = h.t;
            }
            bool more = shade_bounce<M, kStats>(h, ray, radiance, beta, seed, a.trisFull, a.materials, a, st);
            ++bounce;
            if (!more || bounce >= bounces) {
                const F3 rad{M::max(radiance.x, 0.0f), M::max(radiance.y, 0.0f), M::max(radiance.z, 0.0f)};
                finish_pixel<M>(a, gid, rad, pid, pt);
                active = false;
            }
        }
    }
    if (kStats) flush_stats(a, st, lane);
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

__device__ __forceinline__ uint32_t popc_ballot(bool p) { return (uint32_t)__popcll(__ballot(p)); }

template <class M, bool kLdsScene, bool kStats>
__device__ __forceinline__ void step_body(const KernelArgs& a) {
    const int tid = threadIdx.x;
    const SceneView sc = stage_scene<kLdsScene>(a);

    const F3 camPos{a.camPos[0], a.camPos[1], a.camPos[2]};
    const F3 camFront{a.camFront[0], a.camFront[1], a.camFront[2]};
    const F3 camUp{a.camUp[0], a.camUp[1], a.camUp[2]};
    const float angle = M::tan(0.5f * (45.0f * 3.1415f / 180.0f));  // kernel_bvh.cl:392
    const uint32_t fh = frame_hash(a.frameCount);
    const uint32_t bounces = (uint32_t)a.lightBounces;
    const uint32_t total = a.nTiles * 64u;
    const uint32_t rowEnd = a.rowBegin + a.rowCount;
    const int lane = tid & 63;
    const uint32_t kRefillMin = a.refillMin;  // finish + refill when this many lanes are free
    const uint32_t kShadeMin = a.shadeMin;    // shade when this many lanes are ready

    LaneStats st;
    uint32_t state = kIdle;
    uint32_t gid = 0, seed = 0, bounce = 0;
    int32_t pid = -1;
    float pt = 0.0f;
    Ray ray{};
    F3 radiance = f3s(0.0f), beta = f3s(1.0f);
    Traversal h{kMaxDist, -1, 0.0f, 0.0f};
    uint32_t cur = 0;  // TRAV: node to visit; LEAF: node to continue at after the leaf
    uint32_t leaf_i = 0, leaf_end = 0;
    uint32_t chunk_base = 0, chunk_used = 64;  // wave-uniform
    bool exhausted = false;                    // wave-uniform
    // diagnostic phase timers (stats variant only): shader-clock cycles per phase, per wave
    uint64_t cyc_refill = 0, cyc_trav = 0, cyc_shade = 0;
    const uint64_t cyc_start = kStats ? __builtin_amdgcn_s_memtime() : 0;

    for (;;) {
        // ---- finish + refill: accumulate finished paths, start new pixels ----------------------
        uint64_t tA = kStats ? __builtin_amdgcn_s_memtime() : 0;
        const uint32_t n_free = popc_ballot(state == kIdle || state == kDone);
        if (n_free == 64u || (!exhausted && n_free >= kRefillMin)) {
            if (state == kDone) {
                finish_pixel<M>(a, gid, radiance, pid, pt);
                state = kIdle;
            }
            while (!exhausted) {
                const unsigned long long idle = __ballot(state == kIdle);
                if (idle == 0ull) break;
                if (chunk_used >= 64u) {
                    uint32_t b = 0;
                    if (lane == 0) b = atomicAdd(a.workCounter, 64u);
                    b = __shfl(b, 0, 64);
                    if (b >= total) {
                        exhausted = true;
                        break;
                    }
                    chunk_base = b;
                    chunk_used = 0;
                }
                const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(idle >> 32),
                                                                __builtin_amdgcn_mbcnt_lo((uint32_t)idle, 0u));
                const uint32_t take = min((uint32_t)__popcll(idle), 64u - chunk_used);
                if (state == kIdle && rank < take) {
                    const uint32_t idx = chunk_base + chunk_used + rank;
                    const uint32_t tile = idx >> 6, w = idx & 63u;
                    const uint32_t ty = tile / a.tilesX, tx = tile - ty * a.tilesX;
                    const uint32_t x = tx * 8u + (w & 7u),
                                   row = a.rowBegin + (ty * a.bandPeriod + a.bandPhase) * 8u + (w >> 3);
                    const uint64_t g64 = (uint64_t)row * a.width + x;
                    if (x < a.width && row < rowEnd && g64 >= a.gidBegin && g64 < a.gidEnd) {
                        gid = (uint32_t)g64;
                        seed = gid + fh;  // kernel_bvh.cl:445
                        ray = create_ray<M>(gid, a.width, a.height, camPos, camFront, camUp, angle, seed);
                        radiance = f3s(0.0f);
                        beta = f3s(1.0f);
                        bounce = 0;
                        pid = -1;
                        pt = 0.0f;
                        if (bounces > 0u) {
                            state = kTrav;
                            h = Traversal{kMaxDist, -1, 0.0f, 0.0f};
                            cur = 0;
                            if (kStats) ++st.rays;
                        } else {
                            state = kDone;  // no bounce: radiance max(0, 0) = 0
                        }
                    }
                }
                chunk_used += take;
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
        // Each step is wave-uniform: either a node step (TRAV lanes visit one node) or a
        // triangle step (LEAF lanes test one triangle), chosen by which serves more lanes per
        // instruction (weights ~ the two bodies' VALU cost), so the wave never pays both
        // bodies for a mix of lanes.
        for (;;) {
            const uint32_t n_trav = popc_ballot(state == kTrav);
            const uint32_t n_leaf = popc_ballot(state == kLeaf);
            if (n_trav + n_leaf == 0u) break;
            if (popc_ballot(state == kShade) >= kShadeMin) break;
            if (!exhausted && popc_ballot(state == kIdle || state == kDone) >= kRefillMin) break;
            const bool leaf_step = n_leaf * a.stepWeightNode > n_trav * a.stepWeightLeaf;
            if (!leaf_step) {
                if (state == kTrav) {
                    const float4 q0 = sc.nodes[2 * cur];
                    const float4 q1 = sc.nodes[2 * cur + 1];
                    const uint32_t skip = sc.skips[8 * cur + ray.sgn];
                    if (kStats) ++st.visits;
                    uint32_t next = skip;
                    if (ray_bounds(q0, q1, ray, h.t)) {
                        const uint32_t off = __float_as_uint(q1.z);
                        const uint32_t meta = __float_as_uint(q1.w);
                        const uint32_t np = meta & 0xffffu;
                        if (np > 0) {
                            state = kLeaf;
                            leaf_i = off;
                            leaf_end = off + np;
                        } else {
                            next = ((ray.sgn >> (meta >> 16)) & 1u) ? off : cur + 1;
                        }
                    }
                    cur = next;
                    if (state == kTrav && next == kEnd) state = kShade;
                }
            } else {
                if (state == kLeaf) {
                    if (kStats) ++st.tests;
                    ray_triangle<M>(sc.tris + 3 * (size_t)leaf_i, (int32_t)leaf_i, ray, h);
                    ++leaf_i;
                    if (leaf_i == leaf_end) state = cur == kEnd ? kShade : kTrav;
                }
            }
        }

        // ---- shading ---------------------------------------------------------------------------
        uint64_t tC = kStats ? __builtin_amdgcn_s_memtime() : 0;
        if (kStats) cyc_trav += tC - tB;
        if (state == kShade) {
            if (bounce == 0u) {
                pid = h.prim;
                pt = h.t;
            }
            const bool more = shade_bounce<M, kStats>(h, ray, radiance, beta, seed, a.trisFull, a.materials, a, st);
            ++bounce;
            if (!more || bounce >= bounces) {
                radiance = F3{M::max(radiance.x, 0.0f), M::max(radiance.y, 0.0f), M::max(radiance.z, 0.0f)};
                state = kDone;
            } else {
                state = kTrav;
                h = Traversal{kMaxDist, -1, 0.0f, 0.0f};
                cur = 0;
                if (kStats) ++st.rays;
            }
        }
        if (kStats) cyc_shade += __builtin_amdgcn_s_memtime() - tC;
    }
    if (kStats) {
        flush_stats(a, st, lane);
        if (lane == 0) {
            atomicAdd(&a.stats[4], (unsigned long long)cyc_refill);
            atomicAdd(&a.stats[5], (unsigned long long)cyc_trav);
            atomicAdd(&a.stats[6], (unsigned long long)cyc_shade);
            atomicAdd(&a.stats[7], (unsigned long long)(__builtin_amdgcn_s_memtime() - cyc_start));
        }
    }
}

// Entry points per math policy: the devicelib body fits 80 VGPRs with a small spill, and
// 6 waves per SIMD measured 7 % faster than the 4 its natural 113 VGPRs allow
// (profiles/r01/occupancy_ab.txt); the fp64-heavy pinned body stays at its natural budget.
#ifndef RT_STEP_DEVICELIB_WAVES
#define RT_STEP_DEVICELIB_WAVES 6
#endif
template <bool kLdsScene, bool kStats>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(RT_STEP_DEVICELIB_WAVES, 8)))
void kernel_entry_step_devicelib(KernelArgs a) {
    step_body<MathDeviceLib, kLdsScene, kStats>(a);
}
#ifdef RT_STEP_PINNED_WAVES
#define RT_STEP_PINNED_OCC __attribute__((amdgpu_waves_per_eu(RT_STEP_PINNED_WAVES, 8)))
#else
#define RT_STEP_PINNED_OCC
#endif
template <bool kLdsScene, bool kStats>
__global__ __launch_bounds__(256) RT_STEP_PINNED_OCC void kernel_entry_step_pinned(KernelArgs a) {
    step_body<MathPinned, kLdsScene, kStats>(a);
}

// ---- scene packing (runs once per bound scene) -----------------------------------------------
__global__ void pack_nodes(const rt_cl_bvh_node* __restrict__ in, float4* __restrict__ out, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const rt_cl_bvh_node nd = in[i];
    const uint32_t meta = (uint32_t)nd.nPrimitives | ((uint32_t)(nd.nPrimitives ? 0 : nd.axis) << 16);
    out[2 * i] = make_float4(nd.bounds.pmin.x, nd.bounds.pmin.y, nd.bounds.pmin.z, nd.bounds.pmax.x);
    out[2 * i + 1] = make_float4(nd.bounds.pmax.y, nd.bounds.pmax.z, __uint_as_float(nd.offset),
                                 __uint_as_float(meta));
}

__global__ void pack_tris(const rt_cl_triangle* __restrict__ in, float4* __restrict__ out, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const rt_float3 p1 = in[i].v1.position, p2 = in[i].v2.position, p3 = in[i].v3.position;
    // e1 = t2 - t1, e2 = t3 - t1 exactly as kernel_bvh.cl:109-110 computes them
    out[3 * i] = make_float4(p1.x, p1.y, p1.z, 0.0f);
    out[3 * i + 1] = make_float4(p2.x - p1.x, p2.y - p1.y, p2.z - p1.z, 0.0f);
    out[3 * i + 2] = make_float4(p3.x - p1.x, p3.y - p1.y, p3.z - p1.z, 0.0f);
}

}  // namespace rtk

// ---- host-side launch helpers ------------------------------------------------------------
namespace rtk {

// Kernel variants: [schedule][math][scene in LDS][stats].
using KernelFn = void (*)(KernelArgs);

template <class M, bool L, bool S>
static KernelFn pick_sched(int sched) {
    if (sched == kSchedStep) {
        if (M::kId == MathDeviceLib::kId) return kernel_entry_step_devicelib<L, S>;
        return kernel_entry_step_pinned<L, S>;
    }
    return sched == kSchedRegen ? kernel_entry_regen<M, L, S> : kernel_entry<M, L, S>;
}

static KernelFn pick(int sched, int math, bool lds, bool stats) {
    if (math == MathDeviceLib::kId) {
        if (lds) return stats ? pick_sched<MathDeviceLib, true, true>(sched) : pick_sched<MathDeviceLib, true, false>(sched);
        return stats ? pick_sched<MathDeviceLib, false, true>(sched) : pick_sched<MathDeviceLib, false, false>(sched);
    }
    if (lds) return stats ? pick_sched<MathPinned, true, true>(sched) : pick_sched<MathPinned, true, false>(sched);
    return stats ? pick_sched<MathPinned, false, true>(sched) : pick_sched<MathPinned, false, false>(sched);
}

hipError_t launch_kernel_entry(const KernelArgs& a, int sched, int math, bool lds, bool stats, unsigned grid,
                               size_t smem, hipStream_t st) {
    KernelFn fn = pick(sched, math, lds, stats);
    hipLaunchKernelGGL(fn, dim3(grid), dim3(256), smem, st, a);
    return hipGetLastError();
}

int occupancy_kernel_entry(int sched, int math, bool lds, bool stats, size_t smem) {
    int blocks = 0;
    KernelFn fn = pick(sched, math, lds, stats);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, fn, 256, smem) != hipSuccess) return 1;
    return blocks > 0 ? blocks : 1;
}

hipError_t launch_pack(const rt_cl_bvh_node* nodes, uint32_t n_nodes, float4* pn,
                       const rt_cl_triangle* tris, uint32_t n_tris, float4* pt, hipStream_t st) {
    if (n_nodes) hipLaunchKernelGGL(pack_nodes, dim3((n_nodes + 255) / 256), dim3(256), 0, st, nodes, pn, n_nodes);
    if (n_tris) hipLaunchKernelGGL(pack_tris, dim3((n_tris + 255) / 256), dim3(256), 0, st, tris, pt, n_tris);
    return hipGetLastError();
}

}  // namespace rtk
