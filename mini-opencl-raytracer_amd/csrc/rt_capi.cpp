// rt_capi.cpp -- the C ABI of include/rt_hip.h over the HIP runtime.
//
// Objects mirror the reference's OpenCL objects one to one:
//   rt_context = cl::Context + in-order cl::CommandQueue (CLutils.cpp:9-35) -> one HIP
//                device + one non-blocking HIP stream;
//   rt_mem     = cl::Buffer (CLBVHnode.cpp:215-236, CLRaytracer.cpp:132-135) -> hipMalloc
//                allocation (+ a host shadow of what the host last wrote, used to
//                validate scene arrays before any kernel reads them);
//   rt_kernel  = cl::Kernel "KernelEntry" (CLutils.cpp:52-77) -> the argument slots and
//                the derived packed scene the HIP kernels read.
// Safety: the node/triangle/material arrays are validated on the host before the first
// launch that uses them (child indices strictly increasing, leaf ranges inside the
// triangle array, material indices in range, depth <= 64), so a malformed scene is an
// error code, never an out-of-bounds or non-terminating GPU walk.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <limits>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <vector>

#include "../../include/rt_cl_types.h"
#include "../../include/rt_hip.h"
#include "rt_bvh.hpp"
#include "rt_internal.hpp"
#include "rt_kernels.hpp"

namespace {

constexpr uint64_t kKnownFlags =
    RT_MEM_READ_WRITE | RT_MEM_WRITE_ONLY | RT_MEM_READ_ONLY | RT_MEM_COPY_HOST_PTR;
constexpr int kStatWords = 20;                // rt_stats counters kept on the device
constexpr size_t kLdsBudget = 64 * 1024;       // per-workgroup LDS the scene path may use
#ifndef RT_TIMELINE
#define RT_TIMELINE 0
#endif
#ifndef RT_STATIC_FIRST
#define RT_STATIC_FIRST 1
#endif
// per-frame launches without a bulk region: tail counters on this many partitions (a power of two, <=
// rtk::kMaxParts; step_body next_chunk_parts) -- 1080p 2-bounce frames 0.172 -> 0.165 ms with 128-pixel
// tail chunks, which on one counter took 0.231 (profiles/r06/work_handout_ab.txt)
#ifndef RT_COUNTER_PARTS
#define RT_COUNTER_PARTS 8
#endif
#ifndef RT_PF_COUNTER_SLOTS
#define RT_PF_COUNTER_SLOTS 1
#endif
// tail chunks: sized so that every `RT_TAIL_SHARE_WAVES` waves get >= 2.5 of them (1: every wave; 4:
// every workgroup, whose waves split the last one by work stealing): fewer atomics on the tail
// counter for small launches (1080p 2-bounce frames 0.282 -> 0.218 ms alone; 4K launches already
// take the largest chunk, profiles/r06/work_handout_ab.txt)
#ifndef RT_TAIL_SHARE_WAVES
#define RT_TAIL_SHARE_WAVES 4
#endif
// diagnostic timeline builds (-DRT_TIMELINE=1, scripts/timeline.py) write three 64-bin histograms after
// the primary hit ids: such a build requires hit buffers that long
constexpr size_t kHitPad = RT_TIMELINE ? 192 : 0;

}  // namespace

using rti::map_hip;
using rti::qs;

struct rt_kernel_s {
    rt_context ctx = nullptr;
    bool set[RT_ARG_COUNT] = {};
    rt_mem bufs[4] = {};
    uint32_t u32[RT_ARG_COUNT] = {};  // slots 4..10 (raw 4-byte values)
    float f3[3][4] = {};              // slots 11..13
    int math = RT_MATH_SHIPPED;  // the reference as its host builds it (rt_hip.h)
    int sched = RT_SCHED_STEP;
    // step schedule thresholds (lanes), swept on MI355X: LDS scenes (camera-ray ring)
    // profiles/r01/threshold_sweep_ring.txt, shading at 48 since work stealing (44 -> 48: fused
    // -0.3 %, per-frame -0.5 %, profiles/r03/shade_threshold_sweep.txt); scenes read from HBM/L2
    // keep 8 / 48
    uint32_t refill_min = 6, shade_min = 48;
    bool refill_min_set = false;  // RT_TUNE_REFILL_MIN given: also for small per-frame launches (below)
    // scenes read from HBM/L2: 0 = auto (64-B node records 8 / 48; octant records 16 / 48,
    // profiles/r02/goct_sweep.txt)
    uint32_t refill_min_g = 0, shade_min_g = 0;
    uint32_t w_node = 35, w_leaf = 55;         // step schedule: node / triangle step cost weights
    uint32_t w_node_g = 0, w_leaf_g = 0;       // ... on scenes read from HBM/L2 (0: auto)
    // pixels per work-counter fetch: bulk, and the cap of the launch-sized tail chunk (swept on
    // MI355X: profiles/r02/chunk_sweep.txt; 128 / 64 of round 1 left the counter at its atomic
    // throughput once sky tiles were decided at ring fill: 4K Cornell 1.01 -> 0.79 ms/frame)
    uint32_t chunk_pixels = 0, tail_chunk = 256;  // chunk_pixels 0: auto (512; 1024 pixel-major)
    uint32_t bulk_percent = 80;                // share of the frame handed out in bulk chunks
    uint32_t band_period = 1, band_phase = 0;  // 8-row band interleave (multi-GPU sharding)
    uint32_t* work_counter = nullptr;  // persistent schedules' chunk counters: [4] per render stream
    uint32_t* accum_key = nullptr;     // sky-shortcut keys: [0..3] fused frames, [4..5] per-frame (zeroed once)
    int pf_parity = 0;                 // per-frame key slot read by the next launch
    int pf_ctr = 0;                    // per-frame chunk-counter slot of the next launch (RT_PF_COUNTER_SLOTS)
    int tile_major = -1;               // fused work order: -1 auto, 0 frame-major, 1 tile-major, 2 pixel-major
    int pf_sky = 1;                    // per-frame sky shortcut: 0 off, 1 large launches, 2 always
    int pf_defer = 2;                  // per-frame step launches through radiance slots + accumulation
                                       // (0 never, 1 always, 2 while the previous one still runs)
    uint32_t pf_defer_min = 4u << 20;  // ... (2) from this many work items per launch
    uint32_t pf_batch = rtk::kMaxFusedFrames;  // RT_TUNE_PERFRAME_BATCH: frames coalesced per launch
    int max_blocks = 0;                // persistent grid: workgroups per CU (0 = as many as fit)
    int global_oct = 1;                // scenes not in LDS: walk octant records in HBM/L2 (step;
                                       // bunny proxy 1.80 -> 1.58 ms/frame, profiles/r02/goct_sweep.txt)
    // wavefront schedule: ray queues (two sets of 4 float4 planes), hit records, stream counts
    // (refill at 32 free lanes: bunny proxy 2.62 -> 2.45 ms/frame, profiles/r02/wavefront/sweep_bunny.txt)
    uint32_t wf_refill_min = 32, wf_streams_per_cu = 0, wf_top_limit = 256;  // streams 0: auto
    int wf_shade_occ[3][2] = {};       // [math][stats] -> shade workgroups per CU (0 = unknown)
    float4* wf_q[2] = {};
    float2* wf_hits = nullptr;
    size_t wf_cap = 0;                 // entries per plane
    uint32_t* wf_cnt = nullptr;        // 2 x (G + 1) words
    size_t wf_cnt_cap = 0;             // words
    uint64_t range_first = 0, range_last = 0;
    bool comm_sharded = false;  // bands set by rtCommShardKernel: the gather's plan needs the whole frame
    rt_mem hit_ids = nullptr, hit_t = nullptr;
    bool stats = false, timing = false, force_global = false;
    unsigned long long* dstats = nullptr;  // device counters [4]
    uint64_t launches = 0;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> pending_events;  // KernelEntry launches
    std::vector<std::pair<hipEvent_t, hipEvent_t>> pending_accum;   // fused frames' accumulation
    std::vector<hipEvent_t> event_pool;
    double kernel_ms = 0.0, accum_ms = 0.0;
    // render period (rt_stats.render_period_ms): ends of consecutive timed renders
    hipEvent_t first_end = nullptr;
    double period_span_ms = 0.0;
    uint64_t period_intervals = 0;
    // fused frames: radiance and primary-miss flag per (frame slot, work-item), two sets used
    // alternately so a render can run while the previous launch's accumulation reads the other
    float4* rad_buf[RT_RAD_SETS] = {};
    uint8_t* frame_flags[RT_RAD_SETS] = {};
    size_t rad_buf_cap[RT_RAD_SETS] = {};  // float4 slots
    size_t flag_cap[RT_RAD_SETS] = {};     // frame-flag bytes
    hipEvent_t rad_free[RT_RAD_SETS] = {};  // recorded on astream after the accumulation reading the set
    bool rad_busy[RT_RAD_SETS] = {};
    int rad_set = 0;
    hipEvent_t render_done = nullptr;  // recorded on the main stream after a fused render
    uint64_t pf_waits = ~0ull;         // ctx->host_waits at the previous per-frame step launch
    // derived packed scene
    rt_mem packed_for_tris = nullptr, packed_for_nodes = nullptr, checked_mats = nullptr;
    uint64_t packed_tris_gen = ~0ull, packed_nodes_gen = ~0ull, checked_mats_gen = ~0ull;
    float4* packed_tris = nullptr;
    float4* oct_nodes = nullptr;       // [node][octant] 2 x float4 (LDS-resident scenes)
    float4* goct_nodes = nullptr;      // regrouped octant records for the HBM/L2 walk (RT_GOCT_GROUP)
    size_t goct_nodes_cap = 0;
    uint32_t goct_b = 0;               // their B planes' float4 offset
    float4* shade_tris = nullptr;      // compact shading records (normals + mtlIndex)
    float4* shade_mats = nullptr;      // compact materials
    size_t shade_tris_cap = 0, shade_mats_cap = 0;
    bool oct_ok = false;               // every leaf fits the records' inline {first, count}
    float4* g_nodes = nullptr;         // global-scene node records (64 B, top of the tree first)
    size_t g_nodes_cap = 0;
    uint32_t n_top = 0, top_limit = 384;  // nodes of g_nodes staged in LDS (global path; swept, profiles/r01/bunny_top_nodes_sweep_2.txt)
    size_t packed_tris_cap = 0, oct_nodes_cap = 0;
    uint32_t n_nodes = 0, n_tris = 0, n_mats = 0;
    int depth = 0;
    bool last_lds = false;
    // [sched][math][lds][stats][bofs or goct, + 2 for fused launches] -> blocks per CU (0 = unknown)
    int occ_cache[rtk::kNumSched][3][2][2][4] = {};
    size_t occ_smem[rtk::kNumSched][3][2][2][4] = {};
};

namespace {

int ensure_device(rt_context ctx) {
    if (!ctx) return RT_INVALID_CONTEXT;
    return map_hip(hipSetDevice(ctx->device));
}

// an error of an earlier coalesced launch (rti::flush_frames), else rc
int pending_error(rt_context ctx, int rc) {
    if (ctx && ctx->pend_error != RT_SUCCESS) {
        const int e = ctx->pend_error;
        ctx->pend_error = RT_SUCCESS;
        return e;
    }
    return rc;
}

// the context's coalesced frames, when they are `k`'s (a setting of k is about to change how
// they would launch)
void flush_kernel(rt_kernel k) {
    if (k && k->ctx && k->ctx->pend_k == k) (void)rti::flush_frames(k->ctx);
}

// the arguments a coalesced launch compares (FRAME_COUNT continues the run; FRAME_SEED is never
// read by KernelEntry, kernel_bvh.cl:415-456)
bool same_args(const rt_context ctx, const rt_kernel k) {
    for (int i = RT_ARG_WIDTH; i < RT_ARG_COUNT; ++i) {
        if (i == RT_ARG_FRAME_COUNT || i == RT_ARG_FRAME_SEED || i >= RT_ARG_CAMERA_POS) continue;
        if (ctx->pend_u32[i] != k->u32[i]) return false;
    }
    if (std::memcmp(ctx->pend_f3, k->f3, sizeof(k->f3)) != 0) return false;
    return std::memcmp(ctx->pend_bufs, k->bufs, sizeof(k->bufs)) == 0;
}


// Host view of a buffer's bytes (shadow, or a device read-back).
int host_bytes(rt_mem m, std::vector<uint8_t>& tmp, const uint8_t** out) {
    if (m->shadow_valid) {
        *out = m->shadow.data();
        return RT_SUCCESS;
    }
    tmp.resize(m->size);
    hipError_t e = hipMemcpyAsync(tmp.data(), m->dptr, m->size, hipMemcpyDeviceToHost, qs(m->ctx));
    if (e == hipSuccess) e = hipStreamSynchronize(qs(m->ctx));
    if (e != hipSuccess) return map_hip(e);
    *out = tmp.data();
    return RT_SUCCESS;
}

// Validate the flattened BVH (CLBVHnode.cpp:161-183 contract) and return its depth and its
// node count.  The tree is the prefix [0, end) of the array: in the depth-first layout (first
// child = parent + 1, second child after the first child's subtree) the root's subtree ends
// after the leaf its chain of second children reaches.  Nodes past `end` are never read -- by
// the reference's walk from node 0 either -- so a buffer may be larger than the tree it holds
// (rtBuildBVH writes `count` nodes into a buffer of 2n-1).  Within the tree every node is
// checked and each one but the root must have exactly one parent; since a parent's index is
// smaller than its children's, that makes every node reachable from node 0 and the
// skip-pointer walk a finite depth-first order (a child shared by two parents would make it
// loop).
int check_nodes(const rt_cl_bvh_node* nd, uint32_t n, uint32_t n_tris, int* depth_out, uint32_t* n_used) {
    if (n == 0) return RT_INVALID_MEM_OBJECT;
    uint32_t last = 0;  // the root's chain of second children (offsets strictly increase)
    while (nd[last].nPrimitives == 0) {
        if (nd[last].offset <= last || nd[last].offset >= n) return RT_INVALID_MEM_OBJECT;
        last = nd[last].offset;
    }
    n = last + 1;
    std::vector<int> depth(n, -1);
    std::vector<uint8_t> parents(n, 0);
    depth[0] = 0;
    int max_depth = 0;
    // children have larger indices than their parent, so one forward sweep sets depths
    for (uint32_t i = 0; i < n; ++i) {
        const rt_cl_bvh_node& x = nd[i];
        if (i > 0 && parents[i] != 1) return RT_INVALID_MEM_OBJECT;  // orphan: unreachable
        if (x.nPrimitives > 0) {
            if ((uint64_t)x.offset + x.nPrimitives > n_tris) return RT_INVALID_MEM_OBJECT;
            max_depth = std::max(max_depth, depth[i]);
        } else {
            if (x.axis > 2) return RT_INVALID_MEM_OBJECT;
            const uint64_t a = (uint64_t)i + 1, b = x.offset;
            if (a >= n || b >= n || b <= a) return RT_INVALID_MEM_OBJECT;
            if (parents[a]++ != 0 || parents[b]++ != 0) return RT_INVALID_MEM_OBJECT;  // shared child
            depth[a] = depth[i] + 1;
            depth[b] = depth[i] + 1;
        }
    }
    *depth_out = max_depth;
    *n_used = n;
    // The reference's 64-entry stack (kernel_bvh.cl:181) would overflow past depth 64; the
    // stackless walk here has no such limit, so deeper trees are rendered, not rejected.
    return RT_SUCCESS;
}

// Per-octant skip pointers (see rt_kernels.hip, intersect): for octant o (bit i = the ray
// direction's sign on axis i) the reference visits an interior node's second child first
// when bit axis(n) is set (kernel_bvh.cl:200-207).  skip[n][o] is the node the reference
// pops after finishing n's subtree: near child -> far child, far child -> skip of parent.
// Children have larger indices than their parent, so one forward sweep fills the table.
void build_skips(const rt_cl_bvh_node* nd, uint32_t n, std::vector<uint32_t>& skips) {
    skips.assign((size_t)n * 8, 0xffffffffu);
    for (uint32_t i = 0; i < n; ++i) {
        if (nd[i].nPrimitives > 0) continue;
        const uint32_t first = i + 1, second = nd[i].offset;
        for (uint32_t o = 0; o < 8; ++o) {
            const bool swap = (o >> nd[i].axis) & 1u;
            const uint32_t nearc = swap ? second : first, farc = swap ? first : second;
            skips[(size_t)nearc * 8 + o] = farc;
            skips[(size_t)farc * 8 + o] = skips[(size_t)i * 8 + o];
        }
    }
}

// Octant-resolved node records for LDS-resident scenes (stored as 16 planes of float4:
// A[octant][node], then B[octant][node], each plane n + 1 records): for node i and ray
// octant o,
//   A = {near.x, near.y, near.z, far.x}, B = {far.y, far.z, hit_next, miss_next}
// where near/far are the slab planes kernel_bvh.cl:156-169 selects by the ray's signs
// (bit-exact copies of pmin/pmax), miss_next = skip[i][o] and hit_next is the near child
// (interior, < 2^24) or the leaf code count << 24 | first (count 1..127).  The reference's
// "stack empty" is record n, a sentinel every ray misses (its near planes are +inf along the
// octant's direction, so t0 = +inf) whose successors are n itself: a finished walk parks
// there, and the kernel needs no end test per step.  A node step is two b128 reads, the slab
// arithmetic and two selects.  Returns false when a leaf does not fit (> 127 primitives or
// first + count > 2^24): such a scene is rendered from the global layout instead (LDS scenes
// are small, so this takes an unusual hand-made BVH).
constexpr uint32_t kLeafMin = 1u << 24;

// records per octant plane: the n nodes, the END sentinel, and one pad record when that count is
// even -- an odd plane stride (x 16 B) staggers the eight planes over the LDS banks, so lanes of
// different octants at the same node do not collide (an even stride of 40 put planes o and o+2
// on the same banks: +40 % bank-conflict cycles)
inline uint32_t oct_stride(uint32_t n) { return (n + 1) | 1u; }
// float4 offset of the B planes: rtk::kOctB for trees of at most kOctBMaxStride records per plane
// (a node step then reads B at an immediate offset from A), else right after the A planes
inline uint32_t oct_b(uint32_t n) {
    return oct_stride(n) <= rtk::kOctBMaxStride ? rtk::kOctB : 8u * oct_stride(n);
}
inline uint32_t oct_records(uint32_t n) { return oct_b(n) + 8u * oct_stride(n); }

bool build_oct_nodes(const rt_cl_bvh_node* nd, uint32_t n, const std::vector<uint32_t>& skips,
                     std::vector<uint32_t>& out) {
    const uint32_t stride = oct_stride(n), bofs = oct_b(n);
    out.assign((size_t)oct_records(n) * 4, 0u);
    bool ok = n < kLeafMin;
    auto bits = [](float f) {
        uint32_t u;
        std::memcpy(&u, &f, 4);
        return u;
    };
    const float inf = std::numeric_limits<float>::infinity();
    for (uint32_t i = 0; i <= n; ++i) {
        uint32_t leaf = 0;
        float lo[3], hi[3];
        if (i < n) {
            const rt_cl_bvh_node& x = nd[i];
            if (x.nPrimitives > 0) {
                if (x.nPrimitives <= 127 && (uint64_t)x.offset + x.nPrimitives <= kLeafMin)
                    leaf = ((uint32_t)x.nPrimitives << 24) | x.offset;
                else
                    ok = false;
            }
            lo[0] = x.bounds.pmin.x, lo[1] = x.bounds.pmin.y, lo[2] = x.bounds.pmin.z;
            hi[0] = x.bounds.pmax.x, hi[1] = x.bounds.pmax.y, hi[2] = x.bounds.pmax.z;
        } else {
            // END sentinel: near plane +inf (octant bit clear: near = pmin) or -inf (set: near =
            // pmax), i.e. lo = +inf, hi = -inf -- (near - o) * invDir = +inf on every axis
            for (int ax = 0; ax < 3; ++ax) lo[ax] = inf, hi[ax] = -inf;
        }
        for (uint32_t o = 0; o < 8; ++o) {
            // octant-major planes A[o][node], B[o][node] (16 B each): lanes visiting different
            // nodes in the same octant hit different LDS banks
            uint32_t* ra = &out[((size_t)o * stride + i) * 4];
            uint32_t* rb = &out[((size_t)bofs + (size_t)o * stride + i) * 4];
            float nr[3], fr[3];
            for (int ax = 0; ax < 3; ++ax) {
                const bool neg = (o >> ax) & 1u;
                nr[ax] = neg ? hi[ax] : lo[ax];
                fr[ax] = neg ? lo[ax] : hi[ax];
            }
            ra[0] = bits(nr[0]);
            ra[1] = bits(nr[1]);
            ra[2] = bits(nr[2]);
            ra[3] = bits(fr[0]);
            rb[0] = bits(fr[1]);
            rb[1] = bits(fr[2]);
            if (i == n) {
                rb[2] = rb[3] = n;
                continue;
            }
            const uint32_t skip = skips[(size_t)i * 8 + o];
            rb[2] = nd[i].nPrimitives > 0 ? leaf : (((o >> nd[i].axis) & 1u) ? nd[i].offset : i + 1);
            rb[3] = skip == 0xffffffffu ? n : skip;
        }
    }
    return ok;
}

#ifndef RT_GOCT_GROUP
#define RT_GOCT_GROUP 1  // node-major: bunny proxy fused 1.405 -> 1.393 ms/frame (profiles/r03/goct_layout_ab.txt)
#endif
// The same octant records regrouped for the walk over HBM/L2 (RT_GOCT_GROUP = G > 0): blocks of G
// consecutive nodes, each block laid out octant-major ([block][octant][G nodes], A planes then B
// planes), so G = 1 puts the eight octants' records of a node in one 128-B line (lanes of different
// octants at the same node -- every traversal starts at the root -- read one line, not eight) and
// larger G keeps neighbouring nodes of one octant together as the octant-major layout does.  Links
// are stored as walk words (block * 8G + node in block), so the kernel's index (octant x octStride
// + word) holds with octStride = G; END = rtk::kEndWalk, a word that is neither a node nor a leaf (a
// walk that reaches it leaves the node and triangle steps at once: no sentinel loads).
inline uint32_t goct_word(uint32_t i, uint32_t G) { return (i / G) * 8u * G + i % G; }
void build_oct_nodes_grouped(const std::vector<uint32_t>& oct, uint32_t n, uint32_t G, std::vector<uint32_t>& out,
                             uint32_t* b_ofs) {
    const uint32_t stride = oct_stride(n), bofs = oct_b(n);
    const uint32_t na = ((n + 1 + G - 1) / G) * 8u * G;  // A records, sentinel included, whole blocks
    *b_ofs = na;
    out.assign((size_t)2 * na * 4, 0u);
    for (uint32_t i = 0; i <= n; ++i)
        for (uint32_t o = 0; o < 8; ++o) {
            const uint32_t* ra = &oct[((size_t)o * stride + i) * 4];
            const uint32_t* rb = &oct[((size_t)bofs + (size_t)o * stride + i) * 4];
            const size_t at = (size_t)goct_word(i, G) + (size_t)o * G;
            uint32_t* wa = &out[at * 4];
            uint32_t* wb = &out[((size_t)na + at) * 4];
            for (int c = 0; c < 4; ++c) wa[c] = ra[c];
            wb[0] = rb[0];
            wb[1] = rb[1];
            wb[2] = rb[2] >= kLeafMin ? rb[2] : goct_word(rb[2], G);  // leaf code as it is, else the near child
            wb[3] = rb[3] >= n && RT_GOCT_END_WORD ? rtk::kEndWalk : goct_word(rb[3], G);  // END: the non-walk word
        }
}

template <class T>
int ensure_dev(T*& p, size_t& cap, size_t count) {
    if (cap >= count) return RT_SUCCESS;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    hipError_t e = hipMalloc(&p, count * sizeof(T));
    if (e != hipSuccess) return map_hip(e);
    cap = count;
    return RT_SUCCESS;
}

// Node records for scenes read from HBM/L2 (64 B = half a cache line, so one visit touches
// one line): q0 = {bmin.xyz, bmax.x}, q1 = {bmax.yz, c0, c1}, q2/q3 = skip[8].  Interior:
// c0 = first child, c1 = second child | axis << 30; leaf: c0 = first triangle,
// c1 = count | 3 << 30.  Children and skips are explicit, so the nodes can be renumbered:
// the first `top` nodes in breadth-first order (the top of the tree, visited by nearly every
// ray) come first and are staged in LDS; the rest keep their depth-first order.  The walk is
// the same tree and skip table, so visits, tests and results are unchanged.
void build_global_nodes(const rt_cl_bvh_node* nd, uint32_t n, const std::vector<uint32_t>& skips,
                        uint32_t top, std::vector<uint32_t>& out, uint32_t* n_top) {
    std::vector<uint32_t> order, newid(n, 0xffffffffu);
    order.reserve(n);
    std::vector<uint32_t> q = {0};
    for (size_t h = 0; h < q.size() && order.size() < top; ++h) {
        const uint32_t i = q[h];
        newid[i] = (uint32_t)order.size();
        order.push_back(i);
        if (nd[i].nPrimitives == 0) {
            q.push_back(i + 1);
            q.push_back(nd[i].offset);
        }
    }
    *n_top = (uint32_t)order.size();
    for (uint32_t i = 0; i < n; ++i)
        if (newid[i] == 0xffffffffu) {
            newid[i] = (uint32_t)order.size();
            order.push_back(i);
        }
    auto map = [&](uint32_t x) { return x == 0xffffffffu ? x : newid[x]; };
    auto bits = [](float f) {
        uint32_t u;
        std::memcpy(&u, &f, 4);
        return u;
    };
    out.assign((size_t)n * 16, 0u);
    for (uint32_t p = 0; p < n; ++p) {
        const uint32_t i = order[p];
        const rt_cl_bvh_node& x = nd[i];
        uint32_t* r = &out[(size_t)p * 16];
        r[0] = bits(x.bounds.pmin.x);
        r[1] = bits(x.bounds.pmin.y);
        r[2] = bits(x.bounds.pmin.z);
        r[3] = bits(x.bounds.pmax.x);
        r[4] = bits(x.bounds.pmax.y);
        r[5] = bits(x.bounds.pmax.z);
        if (x.nPrimitives > 0) {
            r[6] = x.offset;
            r[7] = (uint32_t)x.nPrimitives | (3u << 30);
        } else {
            r[6] = map(i + 1);
            r[7] = map(x.offset) | ((uint32_t)x.axis << 30);
        }
        for (int o = 0; o < 8; ++o) r[8 + o] = map(skips[(size_t)i * 8 + o]);
    }
}

int prepare_scene(rt_kernel k) {
    rt_mem tm = k->bufs[RT_ARG_BUFFER_SCENE], nm = k->bufs[RT_ARG_BUFFER_NODE],
           mm = k->bufs[RT_ARG_BUFFER_MATERIAL];
    if (tm->size < sizeof(rt_cl_triangle) || nm->size < sizeof(rt_cl_bvh_node) ||
        mm->size < sizeof(rt_cl_material))
        return RT_INVALID_MEM_OBJECT;
    const uint32_t nt = (uint32_t)(tm->size / sizeof(rt_cl_triangle));
    const uint32_t n_buf = (uint32_t)(nm->size / sizeof(rt_cl_bvh_node));
    const uint32_t nmat = (uint32_t)(mm->size / sizeof(rt_cl_material));
    const bool tris_stale = k->packed_for_tris != tm || k->packed_tris_gen != tm->generation;
    const bool nodes_stale = k->packed_for_nodes != nm || k->packed_nodes_gen != nm->generation;
    const bool mats_stale = k->checked_mats != mm || k->checked_mats_gen != mm->generation;
    if (!tris_stale && !nodes_stale && !mats_stale) return RT_SUCCESS;

    std::vector<uint8_t> tmp_t, tmp_n;
    const uint8_t *tb = nullptr, *nb = nullptr;
    int rc = host_bytes(tm, tmp_t, &tb);
    if (rc) return rc;
    rc = host_bytes(nm, tmp_n, &nb);
    if (rc) return rc;
    int depth = 0;
    uint32_t nn = 0;  // the tree's nodes: a prefix of the buffer
    rc = check_nodes(reinterpret_cast<const rt_cl_bvh_node*>(nb), n_buf, nt, &depth, &nn);
    if (rc) return rc;
    const rt_cl_triangle* tr = reinterpret_cast<const rt_cl_triangle*>(tb);
    for (uint32_t i = 0; i < nt; ++i)
        if (tr[i].mtlIndex >= nmat) return RT_INVALID_MEM_OBJECT;
    std::vector<uint32_t> skips;
    build_skips(reinterpret_cast<const rt_cl_bvh_node*>(nb), nn, skips);

    if (nn >= (1u << 30)) return RT_INVALID_MEM_OBJECT;  // node indices share a word with the axis
    std::vector<uint32_t> gn;
    uint32_t n_top = 0;
    build_global_nodes(reinterpret_cast<const rt_cl_bvh_node*>(nb), nn, skips, k->top_limit, gn, &n_top);
    rc = ensure_dev(k->g_nodes, k->g_nodes_cap, (size_t)nn * 4);
    if (rc) return rc;
    {
        hipError_t e = hipMemcpyAsync(k->g_nodes, gn.data(), gn.size() * sizeof(uint32_t), hipMemcpyHostToDevice,
                                      qs(k->ctx));
        if (e != hipSuccess) return map_hip(e);
    }
    std::vector<uint32_t> oct;
    const bool oct_ok = build_oct_nodes(reinterpret_cast<const rt_cl_bvh_node*>(nb), nn, skips, oct);
    rc = ensure_dev(k->oct_nodes, k->oct_nodes_cap, (size_t)oct_records(nn));
    if (rc) return rc;
    {
        hipError_t e = hipMemcpyAsync(k->oct_nodes, oct.data(), oct.size() * sizeof(uint32_t),
                                      hipMemcpyHostToDevice, qs(k->ctx));
        if (e == hipSuccess) e = hipStreamSynchronize(qs(k->ctx));
        if (e != hipSuccess) return map_hip(e);
    }
    k->goct_b = 0;
    if (RT_GOCT_GROUP && oct_ok && (uint64_t)(nn + RT_GOCT_GROUP) * 8u < kLeafMin) {
        std::vector<uint32_t> nm;
        build_oct_nodes_grouped(oct, nn, RT_GOCT_GROUP, nm, &k->goct_b);
        rc = ensure_dev(k->goct_nodes, k->goct_nodes_cap, nm.size() / 4);
        if (rc) return rc;
        hipError_t e = hipMemcpyAsync(k->goct_nodes, nm.data(), nm.size() * sizeof(uint32_t), hipMemcpyHostToDevice,
                                      qs(k->ctx));
        if (e == hipSuccess) e = hipStreamSynchronize(qs(k->ctx));
        if (e != hipSuccess) return map_hip(e);
    }
    if (k->packed_tris_cap < (size_t)nt) {
        if (k->packed_tris) (void)hipFree(k->packed_tris);
        k->packed_tris = nullptr;
        k->packed_tris_cap = 0;
        hipError_t e = hipMalloc(&k->packed_tris, (size_t)nt * 3 * sizeof(float4));
        if (e != hipSuccess) return map_hip(e);
        k->packed_tris_cap = nt;
    }
    rc = ensure_dev(k->shade_tris, k->shade_tris_cap, (size_t)nt * 3);
    if (rc) return rc;
    // two material tables: IEEE divisions (pinned, devicelib), then the shipped policy's
    rc = ensure_dev(k->shade_mats, k->shade_mats_cap, (size_t)nmat * 8);
    if (rc) return rc;
    hipError_t e = rtk::launch_pack(static_cast<const rt_cl_triangle*>(tm->dptr), nt, k->packed_tris,
                                    k->shade_tris, static_cast<const rt_cl_material*>(mm->dptr), nmat,
                                    k->shade_mats, qs(k->ctx));
    if (e != hipSuccess) return map_hip(e);
    k->n_nodes = nn;
    k->n_tris = nt;
    k->n_mats = nmat;
    k->depth = depth;
    k->oct_ok = oct_ok;
    k->n_top = n_top;
    k->packed_for_tris = tm;
    k->packed_tris_gen = tm->generation;
    k->packed_for_nodes = nm;
    k->packed_nodes_gen = nm->generation;
    k->checked_mats = mm;
    k->checked_mats_gen = mm->generation;
    return RT_SUCCESS;
}

hipEvent_t take_event(rt_kernel k) {
    if (!k->event_pool.empty()) {
        hipEvent_t e = k->event_pool.back();
        k->event_pool.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    return e;
}

static int drain_list(rt_kernel k, std::vector<std::pair<hipEvent_t, hipEvent_t>>& list, double& total,
                      bool renders) {
    for (auto& pr : list) {
        float ms = 0.0f;
        hipError_t e = hipEventSynchronize(pr.second);
        if (e == hipSuccess) e = hipEventElapsedTime(&ms, pr.first, pr.second);
        if (e != hipSuccess) return map_hip(e);
        total += ms;
        if (renders) {
            // render period: end of the first timed render to end of the latest one
            if (!k->first_end) {
                k->first_end = pr.second;
            } else {
                float span = 0.0f;
                e = hipEventElapsedTime(&span, k->first_end, pr.second);
                if (e != hipSuccess) return map_hip(e);
                k->period_span_ms = span;
                ++k->period_intervals;
                k->event_pool.push_back(pr.second);
            }
            k->event_pool.push_back(pr.first);
            continue;
        }
        k->event_pool.push_back(pr.first);
        k->event_pool.push_back(pr.second);
    }
    list.clear();
    return RT_SUCCESS;
}

int drain_events(rt_kernel k) {
    int rc = drain_list(k, k->pending_events, k->kernel_ms, true);
    if (rc) return rc;
    return drain_list(k, k->pending_accum, k->accum_ms, false);
}

void reset_period(rt_kernel k) {
    if (k->first_end) k->event_pool.push_back(k->first_end);
    k->first_end = nullptr;
    k->period_span_ms = 0.0;
    k->period_intervals = 0;
}

}  // namespace

extern "C" {

int rtCreateContext(int device_index, rt_context* out) {
    if (!out) return RT_INVALID_VALUE;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return RT_DEVICE_NOT_FOUND;
    if (device_index < 0 || device_index >= n) return RT_INVALID_DEVICE;
    hipError_t e = hipSetDevice(device_index);
    if (e != hipSuccess) return map_hip(e);
    rt_context c = new (std::nothrow) rt_context_s();
    if (!c) return RT_OUT_OF_HOST_MEMORY;
    c->device = device_index;
    e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->astream, hipStreamNonBlocking);
    for (hipStream_t& r : c->rstream)
        if (e == hipSuccess) e = hipStreamCreateWithFlags(&r, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->atail, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->mtail, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->gtail, hipEventDisableTiming);
    if (e != hipSuccess) {
        if (c->stream) (void)hipStreamDestroy(c->stream);
        if (c->astream) (void)hipStreamDestroy(c->astream);
        for (hipStream_t r : c->rstream)
            if (r) (void)hipStreamDestroy(r);
        delete c;
        return RT_INVALID_COMMAND_QUEUE;
    }
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device_index) == hipSuccess) {
        c->num_cus = prop.multiProcessorCount;
        // MI300-class parts: 8 XCDs, CU-mask bits interleaved across them
        // (scripts/probes/cu_mask_probe.hip, profiles/r04/cu_mask_probe.txt)
        if ((std::strncmp(prop.gcnArchName, "gfx94", 5) == 0 || std::strncmp(prop.gcnArchName, "gfx95", 5) == 0) &&
            c->num_cus % 8 == 0)
            c->n_xcd = 8;
    }
    if (c->num_cus <= 0) c->num_cus = 256;
    *out = c;
    return RT_SUCCESS;
}

int rtReleaseContext(rt_context ctx) {
    int rc = ensure_device(ctx);
    if (rc) return rc;
    (void)hipStreamSynchronize(qs(ctx));
    (void)hipStreamSynchronize(ctx->astream);
    (void)hipStreamDestroy(ctx->stream);
    (void)hipStreamDestroy(ctx->astream);
    for (hipStream_t r : ctx->rstream) {
        (void)hipStreamSynchronize(r);
        (void)hipStreamDestroy(r);
    }
    (void)hipEventDestroy(ctx->atail);
    (void)hipEventDestroy(ctx->mtail);
    (void)hipEventDestroy(ctx->gtail);
    delete ctx;
    return RT_SUCCESS;
}

int rtCreateBuffer(rt_context ctx, uint64_t flags, size_t size, const void* host_ptr, rt_mem* out) {
    if (!out) return RT_INVALID_VALUE;
    *out = nullptr;
    int rc = ensure_device(ctx);
    if (rc) return rc;
    if (flags & ~kKnownFlags) return RT_INVALID_VALUE;
    if (size == 0) return RT_INVALID_BUFFER_SIZE;
    const bool copy = (flags & RT_MEM_COPY_HOST_PTR) != 0;
    if (copy != (host_ptr != nullptr)) return RT_INVALID_HOST_PTR;
    rt_mem m = new (std::nothrow) rt_mem_s();
    if (!m) return RT_OUT_OF_HOST_MEMORY;
    m->ctx = ctx;
    m->size = size;
    m->flags = flags;
    hipError_t e = hipMalloc(&m->dptr, size);
    if (e != hipSuccess) {
        delete m;
        return map_hip(e);
    }
    if (copy) {
        try {
            m->shadow.assign(static_cast<const uint8_t*>(host_ptr),
                             static_cast<const uint8_t*>(host_ptr) + size);
        } catch (const std::bad_alloc&) {
            (void)hipFree(m->dptr);
            delete m;
            return RT_OUT_OF_HOST_MEMORY;
        }
        m->shadow_valid = true;
        e = hipMemcpyAsync(m->dptr, host_ptr, size, hipMemcpyHostToDevice, qs(ctx));
    } else {
        e = hipMemsetAsync(m->dptr, 0, size, qs(ctx));
    }
    if (e == hipSuccess) e = hipStreamSynchronize(qs(ctx));
    if (e != hipSuccess) {
        (void)hipFree(m->dptr);
        delete m;
        return map_hip(e);
    }
    *out = m;
    return RT_SUCCESS;
}

int rtReleaseBuffer(rt_mem m) {
    if (!m || m->released) return RT_INVALID_MEM_OBJECT;
    int rc = ensure_device(m->ctx);
    if (rc) return rc;
    (void)hipStreamSynchronize(qs(m->ctx));
    if (m->pins > 0) {  // a gather plan still writes into it: freed when the plan lets go
        m->released = true;
        return RT_SUCCESS;
    }
    (void)hipFree(m->dptr);
    delete m;
    return RT_SUCCESS;
}

int rtCreateKernel(rt_context ctx, const char* name, rt_kernel* out) {
    if (!out) return RT_INVALID_VALUE;
    *out = nullptr;
    int rc = ensure_device(ctx);
    if (rc) return rc;
    if (!name || std::strcmp(name, "KernelEntry") != 0) return RT_INVALID_KERNEL_NAME;
    rt_kernel k = new (std::nothrow) rt_kernel_s();
    if (!k) return RT_OUT_OF_HOST_MEMORY;
    k->ctx = ctx;
    hipError_t e = hipMalloc(&k->dstats, kStatWords * sizeof(unsigned long long));
    // fused radiance sets' counters (16 B each), then the two per-frame slots of kMaxParts counter
    // partitions kPartStride words apart
    const size_t wc_bytes = 16 * RT_RAD_SETS + 2 * sizeof(uint32_t) * rtk::kMaxParts * rtk::kPartStride;
    if (e == hipSuccess) e = hipMalloc(&k->work_counter, wc_bytes);
    if (e == hipSuccess) e = hipMemsetAsync(k->work_counter, 0, wc_bytes, qs(ctx));
    if (e == hipSuccess) e = hipMalloc(&k->accum_key, 32);
    if (e == hipSuccess) e = hipMemsetAsync(k->accum_key, 0, 32, qs(ctx));
    if (e == hipSuccess) e = hipMemsetAsync(k->dstats, 0, kStatWords * sizeof(unsigned long long), qs(ctx));
    if (e == hipSuccess) e = hipStreamSynchronize(qs(ctx));
    if (e != hipSuccess) {
        delete k;
        return map_hip(e);
    }
    *out = k;
    return RT_SUCCESS;
}

int rtReleaseKernel(rt_kernel k) {
    if (!k) return RT_INVALID_KERNEL;
    int rc = ensure_device(k->ctx);
    if (rc) return rc;
    flush_kernel(k);
    (void)hipStreamSynchronize(qs(k->ctx));
    for (auto* list : {&k->pending_events, &k->pending_accum})
        for (auto& pr : *list) {
            (void)hipEventDestroy(pr.first);
            (void)hipEventDestroy(pr.second);
        }
    (void)hipStreamSynchronize(k->ctx->astream);
    for (int i = 0; i < RT_RAD_SETS; ++i) {
        if (k->rad_buf[i]) (void)hipFree(k->rad_buf[i]);
        if (k->frame_flags[i]) (void)hipFree(k->frame_flags[i]);
        if (k->rad_free[i]) (void)hipEventDestroy(k->rad_free[i]);
    }
    if (k->render_done) (void)hipEventDestroy(k->render_done);
    if (k->first_end) (void)hipEventDestroy(k->first_end);
    for (hipEvent_t e : k->event_pool) (void)hipEventDestroy(e);
    for (float4* q : k->wf_q)
        if (q) (void)hipFree(q);
    if (k->wf_hits) (void)hipFree(k->wf_hits);
    if (k->wf_cnt) (void)hipFree(k->wf_cnt);
    if (k->packed_tris) (void)hipFree(k->packed_tris);
    if (k->oct_nodes) (void)hipFree(k->oct_nodes);
    if (k->goct_nodes) (void)hipFree(k->goct_nodes);
    if (k->g_nodes) (void)hipFree(k->g_nodes);
    if (k->shade_tris) (void)hipFree(k->shade_tris);
    if (k->shade_mats) (void)hipFree(k->shade_mats);
    if (k->dstats) (void)hipFree(k->dstats);
    if (k->work_counter) (void)hipFree(k->work_counter);
    if (k->accum_key) (void)hipFree(k->accum_key);
    delete k;
    return RT_SUCCESS;
}

int rtSetKernelArg(rt_kernel k, unsigned index, size_t size, const void* value) {
    if (!k) return RT_INVALID_KERNEL;
    if (index >= RT_ARG_COUNT) return RT_INVALID_ARG_INDEX;
    if (!value) return RT_INVALID_ARG_VALUE;
    if (index <= RT_ARG_BUFFER_MATERIAL) {
        if (size != sizeof(rt_mem)) return RT_INVALID_ARG_SIZE;
        rt_mem m = *static_cast<const rt_mem*>(value);
        if (!m || m->ctx != k->ctx) return RT_INVALID_MEM_OBJECT;
        k->bufs[index] = m;
    } else if (index <= RT_ARG_SKYBOX_INTENSITY) {
        if (size != 4) return RT_INVALID_ARG_SIZE;
        std::memcpy(&k->u32[index], value, 4);
    } else {
        if (size != 16) return RT_INVALID_ARG_SIZE;
        std::memcpy(k->f3[index - RT_ARG_CAMERA_POS], value, 16);
    }
    k->set[index] = true;
    return RT_SUCCESS;
}

static int enqueue(rt_context ctx, rt_kernel k, size_t global_work_size, uint32_t n_frames);


}  // extern "C"

void rti::unpin(rt_mem m) {
    if (--m->pins > 0 || !m->released) return;
    (void)hipFree(m->dptr);  // (the plan has synchronised the streams that wrote it)
    delete m;
}

int rti::flush_frames(rt_context ctx) {
    if (!ctx || !ctx->pend_k) return RT_SUCCESS;
    rt_kernel k = ctx->pend_k;
    ctx->pend_k = nullptr;  // (enqueue's own qs() calls find nothing pending)
    // launch with the arguments the frames were enqueued with, then give the kernel back its own
    uint32_t u32[RT_ARG_COUNT];
    float f3[3][4];
    rt_mem bufs[4];
    std::memcpy(u32, k->u32, sizeof(u32));
    std::memcpy(f3, k->f3, sizeof(f3));
    std::memcpy(bufs, k->bufs, sizeof(bufs));
    std::memcpy(k->u32, ctx->pend_u32, sizeof(u32));
    std::memcpy(k->f3, ctx->pend_f3, sizeof(f3));
    std::memcpy(k->bufs, ctx->pend_bufs, sizeof(bufs));
    std::memcpy(&k->u32[RT_ARG_FRAME_COUNT], &ctx->pend_f0, 4);
    const int rc = enqueue(ctx, k, ctx->pend_gws, ctx->pend_n);
    std::memcpy(k->u32, u32, sizeof(u32));
    std::memcpy(k->f3, f3, sizeof(f3));
    std::memcpy(k->bufs, bufs, sizeof(bufs));
    if (rc != RT_SUCCESS && ctx->pend_error == RT_SUCCESS) ctx->pend_error = rc;
    return rc;
}

extern "C" {

// Frame coalescing (RT_TUNE_PERFRAME_BATCH).  The reference's host issues one ExecuteKernel per
// frame (CLRaytracer.cpp:52-55); a host that queues frames without looking at them in between
// gets them as fused launches (rtEnqueueKernelFrames: bit-identical to the per-frame launches,
// test_fused_frames.py), one launch tail per run instead of one per frame.  The frame is checked
// here as a launch would check it, so argument and scene errors still come back from this call.
int rtEnqueueKernel(rt_context ctx, rt_kernel k, size_t global_work_size) {
    // (not once a stream or a device pointer of the context has been handed out: the host may then
    // synchronise behind the library's back, e.g. hipStreamSynchronize on the exposed stream, and
    // must find every frame it enqueued launched)
    const bool coalesce = ctx && k && k->ctx == ctx && k->pf_batch > 1 && k->sched == RT_SCHED_STEP && !k->stats &&
                          !k->timing && !ctx->mexposed && !ctx->dexposed;
    if (!coalesce) {
        if (ctx && ctx->pend_k) {
            const int rc = rti::flush_frames(ctx);
            if (rc) return pending_error(ctx, rc);
        }
        return enqueue(ctx, k, global_work_size, 1);
    }
    int rc = ensure_device(ctx);
    if (rc) return rc;
    for (int i = 0; i < RT_ARG_COUNT; ++i)
        if (!k->set[i]) return RT_INVALID_KERNEL_ARGS;
    if (global_work_size == 0 || global_work_size > 0xffffffffull) return RT_INVALID_GLOBAL_WORK_SIZE;
    uint32_t W, H, f;
    std::memcpy(&W, &k->u32[RT_ARG_WIDTH], 4);
    std::memcpy(&H, &k->u32[RT_ARG_HEIGHT], 4);
    std::memcpy(&f, &k->u32[RT_ARG_FRAME_COUNT], 4);
    if (W == 0 || H == 0) return RT_INVALID_KERNEL_ARGS;
    if (k->bufs[RT_ARG_BUFFER_OUT]->size < global_work_size * 16) return RT_INVALID_GLOBAL_WORK_SIZE;
    if (k->hit_ids && (k->hit_ids->size < (global_work_size + kHitPad) * 4 || k->hit_t->size < global_work_size * 4))
        return RT_INVALID_MEM_OBJECT;
    // an error of an earlier held launch is reported now, and this frame is not queued: the
    // caller retrying it starts a fresh run instead of accumulating it twice
    if (ctx->pend_error != RT_SUCCESS) return pending_error(ctx, RT_SUCCESS);
    if (ctx->pend_k == k && ctx->pend_gws == global_work_size && ctx->pend_n < k->pf_batch &&
        f == ctx->pend_f0 + ctx->pend_n && f != 0u && same_args(ctx, k)) {
        ++ctx->pend_n;  // the next frame of the run
        return RT_SUCCESS;
    }
    if (ctx->pend_k) {
        rc = rti::flush_frames(ctx);
        if (rc) return pending_error(ctx, rc);
    }
    rc = prepare_scene(k);  // (a malformed scene is refused now, not at the launch)
    if (rc) return rc;
    ctx->pend_k = k;
    ctx->pend_gws = global_work_size;
    ctx->pend_f0 = f;
    ctx->pend_n = 1;
    std::memcpy(ctx->pend_u32, k->u32, sizeof(k->u32));
    std::memcpy(ctx->pend_f3, k->f3, sizeof(k->f3));
    std::memcpy(ctx->pend_bufs, k->bufs, sizeof(k->bufs));
    return pending_error(ctx, RT_SUCCESS);
}

int rtEnqueueKernelFrames(rt_context ctx, rt_kernel k, size_t global_work_size, unsigned n_frames) {
    if (n_frames == 0) return RT_INVALID_VALUE;
    if (ctx && ctx->pend_k) {
        const int rc = rti::flush_frames(ctx);
        if (rc) return pending_error(ctx, rc);
    }
    if (n_frames == 1 || !k || (k->sched != RT_SCHED_STEP && k->sched != RT_SCHED_WAVEFRONT)) {
        // one launch per frame (the other schedules have no fused form): same results
        if (!k) return RT_INVALID_KERNEL;
        uint32_t f0;
        std::memcpy(&f0, &k->u32[RT_ARG_FRAME_COUNT], 4);
        int rc = RT_SUCCESS;
        for (unsigned i = 0; i < n_frames && rc == RT_SUCCESS; ++i) {
            const uint32_t f = f0 + i;
            std::memcpy(&k->u32[RT_ARG_FRAME_COUNT], &f, 4);
            rc = enqueue(ctx, k, global_work_size, 1);
        }
        std::memcpy(&k->u32[RT_ARG_FRAME_COUNT], &f0, 4);
        return rc;
    }
    // fused launches of at most kMaxFusedFrames frames each
    uint32_t f0;
    std::memcpy(&f0, &k->u32[RT_ARG_FRAME_COUNT], 4);
    int rc = RT_SUCCESS;
    for (unsigned done = 0; done < n_frames && rc == RT_SUCCESS;) {
        const unsigned n = std::min<unsigned>(n_frames - done, rtk::kMaxFusedFrames);
        const uint32_t f = f0 + done;
        std::memcpy(&k->u32[RT_ARG_FRAME_COUNT], &f, 4);
        rc = enqueue(ctx, k, global_work_size, n);
        done += n;
    }
    std::memcpy(&k->u32[RT_ARG_FRAME_COUNT], &f0, 4);
    return rc;
}

static int enqueue(rt_context ctx, rt_kernel k, size_t global_work_size, uint32_t n_frames) {
    int rc = ensure_device(ctx);
    if (rc) return rc;
    if (!k || k->ctx != ctx) return RT_INVALID_KERNEL;
    for (int i = 0; i < RT_ARG_COUNT; ++i)
        if (!k->set[i]) return RT_INVALID_KERNEL_ARGS;
    if (global_work_size == 0 || global_work_size > 0xffffffffull) return RT_INVALID_GLOBAL_WORK_SIZE;
    uint32_t W, H;
    std::memcpy(&W, &k->u32[RT_ARG_WIDTH], 4);
    std::memcpy(&H, &k->u32[RT_ARG_HEIGHT], 4);
    if (W == 0 || H == 0) return RT_INVALID_KERNEL_ARGS;
    rt_mem out = k->bufs[RT_ARG_BUFFER_OUT];
    if (out->size < global_work_size * 16) return RT_INVALID_GLOBAL_WORK_SIZE;
    if (k->hit_ids && (k->hit_ids->size < (global_work_size + kHitPad) * 4 || k->hit_t->size < global_work_size * 4))
        return RT_INVALID_MEM_OBJECT;
    rc = prepare_scene(k);
    if (rc) return rc;
    // the schedule this launch runs: the wavefront one needs a bounded bounce loop (two launches
    // per bounce), else the step schedule renders it (same bits)
    int32_t lb;
    std::memcpy(&lb, &k->u32[RT_ARG_LIGHT_BOUNCES], 4);
    const bool wf = k->sched == RT_SCHED_WAVEFRONT && lb >= 1 && lb <= rtk::kWfMaxBounces;
    const int si = wf ? rtk::kSchedWavefront : (k->sched == RT_SCHED_WAVEFRONT ? RT_SCHED_STEP : k->sched);
    // radiance per (frame slot, work-item) + the accumulation launch: fused frames, every wavefront
    // render, and (RT_TUNE_PERFRAME_DEFER) per-frame step launches -- then consecutive renders need
    // not wait for each other, only the accumulations are ordered
    // A loop that synchronises every frame -- the reference's RenderFrame: ExecuteKernel,
    // ReadBuffer, Finish -- gains nothing from it and pays the second launch, and so do small
    // frames; frames queued back to back gain (4K Cornell 1.11 -> 0.92 ms/frame).  So by default
    // (PERFRAME_DEFER 2) a large launch defers when the host has not waited on the context through
    // this API since the kernel's previous per-frame launch: the host is queueing, not waiting
    // (profiles/r03/perframe_defer_auto.txt).  "Queueing" = no host wait on the context (rtFinish,
    // a blocking read or write) since the previous per-frame launch: no GPU-side query, which
    // would itself cost the read-back loop (an event after every render: 3.63 -> 4.07 ms/frame).
    bool defer = false;
    if (n_frames == 1 && si == RT_SCHED_STEP && k->pf_defer) {
        defer = k->pf_defer == 1 ||
                (k->pf_defer == 2 && k->pf_waits == ctx->host_waits && global_work_size >= k->pf_defer_min &&
                 !ctx->mexposed && !ctx->dexposed);  // (a host that can synchronise outside the library)
        k->pf_waits = ctx->host_waits;
    }
    const bool fused = n_frames > 1 || wf || defer;
    // a launch that accumulates in-kernel read-modify-writes the output: after the pending
    // accumulations
    if (!fused) (void)qs(ctx);

    uint64_t g0 = std::min<uint64_t>(k->range_first, global_work_size);
    uint64_t g1 = k->range_last ? std::min<uint64_t>(k->range_last, global_work_size) : global_work_size;
    if (g1 <= g0) return RT_SUCCESS;  // nothing in range

    rtk::KernelArgs a;
    std::memset(&a, 0, sizeof(a));
    a.result = static_cast<float4*>(out->dptr);
    a.trisFull = static_cast<const rt_cl_triangle*>(k->bufs[RT_ARG_BUFFER_SCENE]->dptr);
    a.materials = static_cast<const rt_cl_material*>(k->bufs[RT_ARG_BUFFER_MATERIAL]->dptr);
    a.packedTris = k->packed_tris;
    a.octNodes = k->oct_nodes;
    a.gNodes = k->g_nodes;
    a.shadeTris = k->shade_tris;
    a.shadeMats = k->shade_mats + (k->math == RT_MATH_SHIPPED ? 4 * (size_t)k->n_mats : 0);
    a.nMats = k->n_mats;
    a.nNodes = k->n_nodes;
    a.octStride = oct_stride(k->n_nodes);
    a.octB = oct_b(k->n_nodes);
    a.octRecords = oct_records(k->n_nodes);
    a.nTris = k->n_tris;
    a.width = W;
    a.height = H;
    std::memcpy(&a.frameCount, &k->u32[RT_ARG_FRAME_COUNT], 4);
    std::memcpy(&a.lightBounces, &k->u32[RT_ARG_LIGHT_BOUNCES], 4);
    std::memcpy(&a.lightType, &k->u32[RT_ARG_LIGHT_TYPE], 4);
    std::memcpy(&a.skyboxIntensity, &k->u32[RT_ARG_SKYBOX_INTENSITY], 4);
    for (int i = 0; i < 3; ++i) {
        a.camPos[i] = k->f3[0][i];
        a.camFront[i] = k->f3[1][i];
        a.camUp[i] = k->f3[2][i];
    }
    a.gidBegin = g0;
    a.gidEnd = g1;
    const uint64_t row0 = g0 / W, row1 = (g1 + W - 1) / W;
    a.rowBegin = (uint32_t)row0;
    a.rowCount = (uint32_t)(row1 - row0);
    const uint32_t tile = si == RT_SCHED_TILES ? 16u : 8u;
    if (k->band_period > 1 && si == RT_SCHED_TILES) return RT_INVALID_OPERATION;
    a.tilesX = (W + tile - 1) / tile;
    uint64_t tilesY = (row1 - row0 + tile - 1) / tile;
    a.bandPeriod = k->band_period;
    a.bandPhase = k->band_phase;
    if (k->band_period > 1) {  // bands phase, phase + period, ... of the row window
        tilesY = tilesY > k->band_phase ? (tilesY - k->band_phase + k->band_period - 1) / k->band_period : 0;
        if (tilesY == 0) return RT_SUCCESS;
    }
    const uint64_t n_tiles = tilesY * a.tilesX;
    if (n_tiles * 64 > 0xfff00000ull) return RT_INVALID_GLOBAL_WORK_SIZE;
    a.nTiles = (uint32_t)n_tiles;
    // per-frame launches: their own counters (two slots in turn with RT_PF_COUNTER_SLOTS, below)
    a.workCounter = k->work_counter + 4 * RT_RAD_SETS;
    a.workCounterClear = nullptr;
    a.chunkPixels = k->chunk_pixels ? k->chunk_pixels : 512u;  // (the launch's order decides below)
    a.tailChunk = k->tail_chunk;
    a.refillMin = k->refill_min;
    a.shadeMin = k->shade_min;
    a.stepWeightNode = k->w_node;
    a.stepWeightLeaf = k->w_leaf;
    a.nFrames = n_frames;
    a.radStride = (uint32_t)g1;
    a.radBuf = nullptr;
    hipStream_t rstr = ctx->stream;  // the stream this launch's render goes to
    if (fused) {
        // fused frames: radiance slots indexed by global work-item id (the lane packs
        // slot * g1 + gid into 32 bits); tiles x frames work items
        // (work items stay below 2^32 - 2^20: the work-stealing ranges add a few tiles past
        // their end in 32-bit fields)
        if ((uint64_t)n_frames * g1 > 0xffffffffull || n_tiles * 64 * n_frames > 0xfff00000ull)
            return RT_INVALID_GLOBAL_WORK_SIZE;
        const size_t need = (size_t)n_frames * g1;
        // frame flags: a byte per (slot, work item), or a 64-bit word per (slot, tile) (flagTiles)
        const size_t fneed = std::max<size_t>(need, (size_t)n_frames * n_tiles * 8u);
        const int rs = ctx->overlap ? k->rad_set : 0;
        if (k->rad_buf_cap[rs] < need || k->flag_cap[rs] < fneed) {
            // the set may still be read by an accumulation in flight
            hipError_t me = hipStreamSynchronize(ctx->astream);
            if (me != hipSuccess) return map_hip(me);
            if (k->rad_buf[rs]) (void)hipFree(k->rad_buf[rs]);
            if (k->frame_flags[rs]) (void)hipFree(k->frame_flags[rs]);
            k->rad_buf[rs] = nullptr;
            k->frame_flags[rs] = nullptr;
            k->rad_buf_cap[rs] = 0;
            k->flag_cap[rs] = 0;
            me = hipMalloc(&k->rad_buf[rs], need * sizeof(float4));
            if (me == hipSuccess) me = hipMalloc(&k->frame_flags[rs], fneed);
            if (me == hipSuccess && !k->rad_free[rs])
                me = hipEventCreateWithFlags(&k->rad_free[rs], hipEventDisableTiming);
            if (me == hipSuccess && !k->render_done)
                me = hipEventCreateWithFlags(&k->render_done, hipEventDisableTiming);
            if (me != hipSuccess) return map_hip(me);
            k->rad_buf_cap[rs] = need;
            k->flag_cap[rs] = fneed;
        }
        if (ctx->overlap && !k->hit_ids && !wf) {
            // the set's own render stream, after everything queued on the main stream so far
            // (buffer writes, per-frame launches) but not after the previous step's render or
            // accumulation: it fills the CUs that render's draining waves free.  (With hit
            // buffers bound the renders stay in order on the main stream: each writes them.)
            rstr = ctx->rstream[ctx->rnext];
            ctx->rnext = (ctx->rnext + 1) % RT_RENDER_STREAMS;
            hipError_t me = rti::main_tail_wait(ctx, rstr);
            if (me != hipSuccess) return map_hip(me);
        }
        // the render writes the set: after the accumulation that last read it
        if (k->rad_busy[rs]) {
            hipError_t me = hipStreamWaitEvent(rstr, k->rad_free[rs], 0);
            if (me != hipSuccess) return map_hip(me);
            k->rad_busy[rs] = false;
        }
        a.radBuf = k->rad_buf[rs];
        a.frameFlags = k->frame_flags[rs];
        // one chunk counter per radiance set: renders of the two sets may run together
        a.workCounter = k->work_counter + 4 * rs;
    }
    // everything below (counter clear, timing events, the render; the accumulation when it is not
    // overlapped) goes to rstr: the main stream unless a render stream was taken above
    if (rstr == ctx->stream) ctx->mdirty = true;
    a.hitIds = k->hit_ids ? static_cast<int32_t*>(k->hit_ids->dptr) : nullptr;
    a.hitT = k->hit_t ? static_cast<float*>(k->hit_t->dptr) : nullptr;
    a.stats = k->dstats;

    // LDS: octant node records (8 x 32 B per node), triangles (48 B), shading records
    // (48 B per triangle, 64 B per material); no stack
    const size_t scene_bytes = (size_t)oct_records(k->n_nodes) * 16 + (size_t)k->n_tris * 96 + (size_t)k->n_mats * 64;
    const bool lds = !k->force_global && k->oct_ok && scene_bytes <= kLdsBudget;

    // scenes too large for LDS: the step schedule may walk the octant records in HBM/L2
    // (RT_TUNE_GLOBAL_OCT) instead of the 64-B global node records
    const bool goct = !lds && (wf || si == RT_SCHED_STEP) && k->oct_ok && k->global_oct;
    a.nTop = lds || goct ? 0u : k->n_top;  // global path: top-of-tree node records staged in LDS
    if (goct && RT_GOCT_GROUP && k->goct_nodes && k->goct_b) {
        // regrouped records, links as walk words (build_oct_nodes_grouped)
        a.octNodes = k->goct_nodes;
        a.octStride = RT_GOCT_GROUP;
        a.octB = k->goct_b;
        a.octRecords = 2u * a.octB;
        a.nNodes = RT_GOCT_END_WORD ? rtk::kEndWalk : goct_word(k->n_nodes, RT_GOCT_GROUP);  // the END word
    }
    // (octant walk: refill at 32 free lanes under the pixel-major order, 16 before: -0.5 %,
    // profiles/r05/goct_bursts_weights.txt)
    a.refillMin = lds ? k->refill_min : k->refill_min_g ? k->refill_min_g : goct ? 32u : 8u;
    a.shadeMin = lds ? k->shade_min : k->shade_min_g ? k->shade_min_g : 48u;
    if (!lds) {
        // scenes in HBM/L2: a node step's loads cost more against a triangle step's than in LDS
        // (octant walk under the pixel-major order: 65 / 55 -- 35: +1.0 %, 45: +0.4 %, 80-130 the same;
        // profiles/r05/goct_bursts_weights.txt)
        a.stepWeightNode = k->w_node_g ? k->w_node_g : goct ? 65u : k->w_node;
        a.stepWeightLeaf = k->w_leaf_g ? k->w_leaf_g : k->w_leaf;
    }
    if (wf) a.nTop = std::min(a.nTop, k->wf_top_limit);
    const size_t smem =
        wf ? (lds ? ((size_t)a.octRecords + 3 * (size_t)k->n_tris) * 16 : (size_t)a.nTop * 64) +
                 (rtk::kWfExtendThreads / 64) * rtk::kWfRingBytes
           : (lds ? scene_bytes : (size_t)a.nTop * 64) +
                 (si == RT_SCHED_STEP && !fused ? 4 * rtk::kFinishWaveBytes : 0) +
                 (si == RT_SCHED_STEP && lds ? 4 * (fused ? rtk::kRingWaveBytes : rtk::kRingWaveBytesPf) : 0) +
                 (si == RT_SCHED_STEP ? rtk::kStealBytes : 0);
    k->last_lds = lds;
    // the step schedule's ray ring (LDS scenes) writes each tile's frame flags as one word at ring
    // fill; the other fused renders write a byte per path at its end
    a.flagTiles = fused && !wf && si == RT_SCHED_STEP && lds ? 1u : fused && !wf && si == RT_SCHED_STEP && goct ? 2u : 0u;

    const int mi = k->math;
    const bool bofs = lds && a.octB == rtk::kOctB;
    const int var = (bofs || goct ? 1 : 0) + (a.radBuf ? 2 : 0);  // occupancy cache: the variant slot
    int& occ = k->occ_cache[si][mi][lds][k->stats][var];
    if (occ == 0 || k->occ_smem[si][mi][lds][k->stats][var] != smem) {
        occ = wf ? rtk::occupancy_wf_extend(k->math, lds, k->stats, bofs, smem, goct)
                 : rtk::occupancy_kernel_entry(si, k->math, lds, k->stats, bofs, smem, goct, a.radBuf != nullptr);
        k->occ_smem[si][mi][lds][k->stats][var] = smem;
    }
    uint64_t grid = (uint64_t)(k->max_blocks ? std::min(occ, k->max_blocks) : occ) * (uint64_t)ctx->num_cus;
    // tiles: one workgroup per 16x16 tile at most; persistent schedules: one 8x8 tile per wave
    // (wavefront extend: 8 waves per workgroup)
    grid = std::min<uint64_t>(grid, si == RT_SCHED_TILES ? n_tiles
                                    : wf                 ? (n_tiles * n_frames + 7) / 8
                                                         : (n_tiles * n_frames + 3) / 4);
    if (grid == 0) grid = 1;
    {
        // bulk chunks only when every resident wave gets at least two of them; a small frame
        // (512x512: ~40 pixels per wave) is handed out 64 pixels at a time
        const uint64_t tot = (uint64_t)a.nTiles * 64u * n_frames, waves = grid * 4u;
        // fused work order (step_body) on the HBM/L2 scene path: pixel-major when F is a power of two
        // -- a pixel's frames side by side in a wave, so a step's lanes read fewer records: bunny
        // proxy 1.352 -> 1.282 ms/frame, emulated N = 8 rank 1.637 -> 1.535 ms
        // (profiles/r05/pixel_major_ab.txt); else tile-major for large launches (a tile's frames back
        // to back: -1.4 %, profiles/r01/work_order_ab.txt) and frame-major for small ones (tile-major
        // bunches a costly tile's frames into the tail); LDS scenes frame-major (the ray ring)
        // (the pixel-major order is the step schedule's: the wavefront extend launches keep the
        // big / frame-major rule their order was measured with, profiles/r02/wavefront/)
        const bool pow2 = (n_frames == 2 || n_frames == 4 || n_frames == 8) && si == RT_SCHED_STEP;
        const bool big = !lds && tot >= 4096u * waves;
        a.tileMajor = n_frames < 2 ? 0u
                      : k->tile_major == 2 ? (!lds && pow2 ? 2u : 1u)
                      : k->tile_major == 1 ? 1u
                      : k->tile_major == 0 ? 0u
                      : !lds && pow2       ? 2u
                      : big                ? 1u
                                           : 0u;
        // the bulk share stops where the tail would hold less than two bulk chunks per wave: a
        // bulk chunk (512 pixel-frames, ~0.25 ms of a wave's time at 4K) taken just before the
        // split otherwise outlasts the tail that should even the waves out -- small launches
        // (multi-GPU ranks: N = 8 renders 1/8 of the frame) get a larger tail (bulk 80 % -> ~37 %:
        // emulated N = 8 rank step, Cornell 1.112 -> 1.047 ms, bunny proxy 1.694 -> 1.629 ms;
        // profiles/r02/multigpu/n8_chunk_sweep_*.txt); full 4K launches keep 80 %
        // bulk chunks of 512 work items, 1024 in the pixel-major order (two whole tiles x 8 frames per
        // fetch: bunny proxy -0.8 %, profiles/r05/goct_bursts_weights.txt)
        const uint32_t chunk = k->chunk_pixels ? k->chunk_pixels : a.tileMajor == 2u ? 1024u : 512u;
        a.chunkPixels = chunk;
        uint64_t bulk = tot * k->bulk_percent / 100;
        const uint64_t reserve = 2u * waves * chunk;
        bulk = std::min<uint64_t>(bulk, tot > reserve ? tot - reserve : 0u);
        a.chunkSplit = tot >= 2u * waves * chunk ? (uint32_t)(bulk / chunk * chunk) : 0u;
        // tail chunks: the largest power-of-two multiple of 64 pixels, up to tail_chunk, that still
        // gives every wave >= 2.5 of them -- few atomics on the tail counter for large launches,
        // fine-grained balance for small ones (4K fused 256, 4K per-frame / 1080p / 512^2 fused 128,
        // 512^2 per-frame 64: profiles/r02/chunk_sweep.txt)
        // (with counter partitions -- per-frame launches without a bulk region, below -- the grabs no
        // longer queue on one address, and the finer per-wave rule balances better)
        const bool parts = RT_COUNTER_PARTS > 1 && RT_STATIC_FIRST && RT_PF_COUNTER_SLOTS && !fused &&
                           si == RT_SCHED_STEP && !wf && a.chunkSplit == 0u && grid >= RT_COUNTER_PARTS &&
                           tot >= 256u * waves;  // (512^2 frames, ~50 work items per wave: +5 % with them)
        const uint64_t share = (tot - a.chunkSplit) * (parts ? 1u : RT_TAIL_SHARE_WAVES) / waves;
        uint32_t tail = 64;
        while (tail * 2u <= k->tail_chunk && (uint64_t)tail * 2u * 5u <= share * 2u) tail *= 2u;
        a.tailChunk = tail;
        // RT_STATIC_FIRST: a per-frame launch without a bulk region starts every wave on its own tail chunk,
        // with no atomic (step_body), and the tail counter hands out from past those chunks.  (The
        // same for the bulk region of large launches was 3-5 % slower: the waves then stay in step
        // and meet again at the counter.)
        a.tailBase = a.chunkSplit;
        if (RT_STATIC_FIRST && !fused && si == RT_SCHED_STEP && !wf && a.chunkSplit == 0u) {
            a.staticFirst = 1u;
            a.tailBase = (uint32_t)std::min<uint64_t>(waves * tail, tot);
            // RT_COUNTER_PARTS: the tail counter split over that many partitions (with the per-frame
            // counter slots, whose layout holds them)
            if (parts) {
                a.nParts = RT_COUNTER_PARTS;
                a.partLen = (uint32_t)((tot / 64u + RT_COUNTER_PARTS - 1) / RT_COUNTER_PARTS * 64u);
            }
            // such launches (a 1080p frame: ~400 work items per wave) refill at 16 free lanes, not 6:
            // 1080p 2-bounce frames -2.8 % (4K fused launches lose 5 % at 16,
            // profiles/r06/work_handout_ab.txt)
            if (lds && !k->refill_min_set) a.refillMin = 16u;
        }
    }

    // per-frame sky shortcut (step_body): its key costs each wave one gamma step at launch
    // start, which pays off from ~256 pixels per wave (1080p -2.7 %, 4K) and not on small frames
    // (512^2; round 6: the threshold was 1k pixels per wave before the small-launch hand-out,
    // profiles/r06/work_handout_ab.txt)
    if (!fused && si == RT_SCHED_STEP &&
        (k->pf_sky == 2 || (k->pf_sky == 1 && g1 - g0 >= 256u * 4u * grid))) {
        a.pfKeyIn = k->accum_key + 4 + k->pf_parity;
        a.pfKeyOut = k->accum_key + 4 + (k->pf_parity ^ 1);
    }
    rtk::WfArgs wa{};
    float4* wq[2] = {};
    uint32_t* wcnt[2] = {};
    unsigned grid_s = 0;
    if (wf) {
        // queues for every (frame slot, work-item) of the launch, streams of 64-entry blocks
        const uint64_t blocks = n_tiles * n_frames;
        const size_t cap = (size_t)blocks * 64;
        // streams: by default one per shade workgroup the GPU holds at once, so the shade
        // launch is a single round of workgroups (no second, partly empty round)
        int& occ_s = k->wf_shade_occ[mi][k->stats];
        if (occ_s == 0) occ_s = rtk::occupancy_wf_shade(k->math, k->stats);
        const uint64_t per_cu = k->wf_streams_per_cu ? k->wf_streams_per_cu : (uint64_t)occ_s;
        const uint32_t G = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(blocks, (uint64_t)ctx->num_cus * per_cu));
        if (k->wf_cap < cap) {
            // earlier renders on this stream may still read them
            hipError_t me = hipStreamSynchronize(rstr);
            for (float4*& q : k->wf_q) {
                if (q) (void)hipFree(q);
                q = nullptr;
            }
            if (k->wf_hits) (void)hipFree(k->wf_hits);
            k->wf_hits = nullptr;
            k->wf_cap = 0;
            for (float4*& q : k->wf_q)
                if (me == hipSuccess) me = hipMalloc(&q, cap * 4 * sizeof(float4));
            if (me == hipSuccess) me = hipMalloc(&k->wf_hits, cap * sizeof(float2));
            if (me != hipSuccess) return map_hip(me);
            k->wf_cap = cap;
        }
        if (k->wf_cnt_cap < 2 * ((size_t)G + 1)) {
            hipError_t me = hipStreamSynchronize(rstr);
            if (k->wf_cnt) (void)hipFree(k->wf_cnt);
            k->wf_cnt = nullptr;
            k->wf_cnt_cap = 0;
            if (me == hipSuccess) me = hipMalloc(&k->wf_cnt, 2 * ((size_t)G + 1) * sizeof(uint32_t));
            if (me != hipSuccess) return map_hip(me);
            k->wf_cnt_cap = 2 * ((size_t)G + 1);
        }
        wq[0] = k->wf_q[0];
        wq[1] = k->wf_q[1];
        wcnt[0] = k->wf_cnt;
        wcnt[1] = k->wf_cnt + G + 1;
        wa.hits = k->wf_hits;
        wa.cap = (uint32_t)cap;
        wa.G = G;
        wa.nBlocks = (uint32_t)blocks;
        wa.refillMin = k->wf_refill_min;
        grid_s = G;  // one workgroup per stream
    }
    // the chunk counters start at zero: per-frame launches clear theirs here; a fused render's
    // (its radiance set's) were cleared by the accumulation that followed the set's previous render
    // (accum_key_body), which this render already waits for -- no clearing launch in front of it
#ifdef RT_DIAG_NO_ACCUM
    const bool clear_here = true;  // (diagnostic builds without the accumulation launch)
#else
    const bool clear_here = !fused;
#endif
    // RT_PF_COUNTER_SLOTS: a per-frame step launch takes one of two counter slots in turn and zeroes
    // the other for the next one (step_body), so no clearing launch sits between consecutive renders
    // (1080p: a 4-us fill and two ~6-us dispatch gaps in a ~0.28-ms frame)
    const bool pf_slots = RT_PF_COUNTER_SLOTS && !fused && si == RT_SCHED_STEP && !wf;
    if (pf_slots) {
        a.workCounter = k->work_counter + 4 * RT_RAD_SETS + k->pf_ctr * rtk::kMaxParts * rtk::kPartStride;
        a.workCounterClear = k->work_counter + 4 * RT_RAD_SETS + (k->pf_ctr ^ 1) * rtk::kMaxParts * rtk::kPartStride;
    } else if (si != RT_SCHED_TILES && !wf && clear_here) {
        hipError_t me = hipMemsetAsync(a.workCounter, 0, 16, rstr);
        if (me != hipSuccess) return map_hip(me);
    }
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    if (k->timing) {
        ev0 = take_event(k);
        ev1 = take_event(k);
        if (!ev0 || !ev1) return RT_OUT_OF_RESOURCES;
        (void)hipEventRecord(ev0, rstr);
    }
    hipError_t e = wf ? rtk::launch_wavefront(a, wa, wq, wcnt, k->math, lds, k->stats, bofs, (unsigned)grid, smem,
                                              grid_s, rstr, goct)
                      : rtk::launch_kernel_entry(a, si, k->math, lds, k->stats, (unsigned)grid, smem, rstr, goct);
    if (e != hipSuccess) return map_hip(e);
    if (k->timing) {
        (void)hipEventRecord(ev1, rstr);
        k->pending_events.emplace_back(ev0, ev1);
    }
    if (a.pfKeyIn) k->pf_parity ^= 1;
    if (pf_slots) k->pf_ctr ^= 1;
    if (fused) {
        // fused frames: the gamma accumulation of every frame, in order, per pixel -- on the
        // accumulation stream after this render, overlapping whatever the main stream runs next
        // (the next fused render uses the other radiance set); qs() joins it back
        hipStream_t as = ctx->stream;
        if (!ctx->overlap) ctx->mdirty = true;
        // The render left its chunk counters for this accumulation to clear (accum_key_body); if
        // the accumulation cannot be enqueued, clear them behind the render (same stream as the
        // set's next render), so that render does not start with spent counters and skip tiles.
        auto fail = [&](int rc) {
            (void)hipMemsetAsync(a.workCounter, 0, 16, rstr);
            return rc;
        };
        if (ctx->overlap) {
            as = ctx->astream;
            e = hipEventRecord(k->render_done, rstr);
            if (e == hipSuccess) e = hipStreamWaitEvent(as, k->render_done, 0);
            if (e != hipSuccess) return fail(map_hip(e));
        }
        hipEvent_t ea = nullptr, eb = nullptr;
        if (k->timing) {
            ea = take_event(k);
            eb = take_event(k);
            if (!ea || !eb) return fail(RT_OUT_OF_RESOURCES);
            (void)hipEventRecord(ea, as);
        }
        // (a root's gather copies of the previous image read `out`: the accumulation that rewrites
        // it comes after them)
        e = rti::out_read_wait(ctx, as);
        if (e != hipSuccess) return fail(map_hip(e));
#ifndef RT_DIAG_NO_ACCUM  // diagnostic A/B builds only (wrong images): the render without its accumulation
        e = rtk::launch_accum_frames(a, k->math, k->accum_key, as);
        if (e != hipSuccess) return fail(map_hip(e));
#endif
        if (k->timing) {
            (void)hipEventRecord(eb, as);
            k->pending_accum.emplace_back(ea, eb);
        }
        if (ctx->overlap) {
            const int rs = k->rad_set;
            e = hipEventRecord(k->rad_free[rs], as);
            if (e == hipSuccess) e = hipEventRecord(ctx->atail, as);
            if (e != hipSuccess) return map_hip(e);
            k->rad_busy[rs] = true;
            k->rad_set = (k->rad_set + 1) % RT_RAD_SETS;
            ctx->apending = true;
        }
    }
    if (k->pending_events.size() + k->pending_accum.size() > 4096) {
        rc = drain_events(k);
        if (rc) return rc;
    }
    ++k->launches;
    return RT_SUCCESS;
}

int rtBuildBVH(rt_context ctx, rt_mem tris, size_t n_tris, unsigned max_prims_in_node, rt_mem nodes,
               size_t* n_nodes) {
    return rtBuildBVHEx(ctx, tris, n_tris, max_prims_in_node, RT_BVH_PLOC, nodes, n_nodes);
}

int rtBuildBVHEx(rt_context ctx, rt_mem tris, size_t n_tris, unsigned max_prims_in_node, int method, rt_mem nodes,
                 size_t* n_nodes) {
    if (method != RT_BVH_LBVH && method != RT_BVH_PLOC) return RT_INVALID_VALUE;
    int rc = ensure_device(ctx);
    if (rc) return rc;
    if (ctx->pend_k) (void)rti::flush_frames(ctx);
    if (!tris || !nodes || tris->ctx != ctx || nodes->ctx != ctx) return RT_INVALID_MEM_OBJECT;
    if (!n_nodes || n_tris == 0 || n_tris >= (1u << 30)) return RT_INVALID_VALUE;
    if (tris->size < n_tris * sizeof(rt_cl_triangle)) return RT_INVALID_BUFFER_SIZE;
    if (nodes->size < (2 * n_tris - 1) * sizeof(rt_cl_bvh_node)) return RT_INVALID_BUFFER_SIZE;
    const uint32_t mp = std::max(1u, std::min(max_prims_in_node, 65535u));
    void* scratch = nullptr;
    const size_t scratch_size = rtb::scratch_bytes((uint32_t)n_tris);
    if (scratch_size == 0) return RT_OUT_OF_RESOURCES;  // rocPRIM could not size its temporaries
    hipError_t e = hipMalloc(&scratch, scratch_size);
    if (e != hipSuccess) return map_hip(e);
    uint32_t count = 0;
    e = rtb::build(static_cast<rt_cl_triangle*>(tris->dptr), (uint32_t)n_tris, mp,
                   static_cast<rt_cl_bvh_node*>(nodes->dptr), &count, scratch, qs(ctx), method);
    if (e == hipSuccess) e = hipStreamSynchronize(qs(ctx));
    (void)hipFree(scratch);
    if (e != hipSuccess) return map_hip(e);
    for (rt_mem m : {tris, nodes}) {  // device contents changed: host shadows are stale
        m->shadow_valid = false;
        ++m->generation;
    }
    *n_nodes = count;
    return RT_SUCCESS;
}

// the host waits for the context's queue
static hipError_t host_wait(rt_context ctx) {
    ++ctx->host_waits;
    return hipStreamSynchronize(qs(ctx));
}

int rtEnqueueReadBuffer(rt_context ctx, rt_mem m, int blocking, size_t offset, size_t size, void* dst) {
    int rc = ensure_device(ctx);
    if (rc) return rc;
    if (!m || m->ctx != ctx) return RT_INVALID_MEM_OBJECT;
    if (!dst || offset > m->size || size > m->size - offset) return RT_INVALID_VALUE;
    hipError_t e = hipMemcpyAsync(dst, static_cast<uint8_t*>(m->dptr) + offset, size,
                                  hipMemcpyDeviceToHost, qs(ctx));
    if (e == hipSuccess && blocking) e = host_wait(ctx);
    return pending_error(ctx, map_hip(e));
}

int rtEnqueueWriteBuffer(rt_context ctx, rt_mem m, int blocking, size_t offset, size_t size,
                         const void* src) {
    int rc = ensure_device(ctx);
    if (rc) return rc;
    if (!m || m->ctx != ctx) return RT_INVALID_MEM_OBJECT;
    if (!src || offset > m->size || size > m->size - offset) return RT_INVALID_VALUE;
    // coalesced frames launch first, reading (and packing) the scene as it was
    if (ctx->pend_k) (void)rti::flush_frames(ctx);
    if (m->shadow_valid) std::memcpy(m->shadow.data() + offset, src, size);
    ++m->generation;
    hipError_t e = hipMemcpyAsync(static_cast<uint8_t*>(m->dptr) + offset, src, size,
                                  hipMemcpyHostToDevice, qs(ctx));
    if (e == hipSuccess && blocking) e = host_wait(ctx);
    return pending_error(ctx, map_hip(e));
}

int rtEnqueueCopyBufferToPointer(rt_context ctx, rt_mem m, size_t offset, size_t size, void* dst) {
    int rc = ensure_device(ctx);
    if (rc) return rc;
    if (!m || m->ctx != ctx) return RT_INVALID_MEM_OBJECT;
    if (!dst || offset > m->size || size > m->size - offset) return RT_INVALID_VALUE;
    return map_hip(hipMemcpyAsync(dst, static_cast<uint8_t*>(m->dptr) + offset, size,
                                  hipMemcpyDeviceToDevice, qs(ctx)));
}

int rtFinish(rt_context ctx) {
    int rc = ensure_device(ctx);
    if (rc) return rc;
    return pending_error(ctx, map_hip(host_wait(ctx)));
}

int rtKernelSetMathMode(rt_kernel k, int mode) {
    if (!k) return RT_INVALID_KERNEL;
    flush_kernel(k);
    if (mode != RT_MATH_PINNED && mode != RT_MATH_DEVICELIB && mode != RT_MATH_SHIPPED) return RT_INVALID_VALUE;
    k->math = mode;
    return RT_SUCCESS;
}

int rtKernelSetSchedule(rt_kernel k, int sched) {
    if (!k) return RT_INVALID_KERNEL;
    flush_kernel(k);
    if (sched != RT_SCHED_TILES && sched != RT_SCHED_STEP &&
        sched != RT_SCHED_WAVEFRONT)
        return RT_INVALID_VALUE;
    k->sched = sched;
    return RT_SUCCESS;
}

int rtKernelSetRowInterleave(rt_kernel k, unsigned period, unsigned phase) {
    if (!k) return RT_INVALID_KERNEL;
    flush_kernel(k);
    if (period == 0 || phase >= period) return RT_INVALID_VALUE;
    k->band_period = period;
    k->band_phase = phase;
    k->comm_sharded = false;
    return RT_SUCCESS;
}

}  // extern "C"

// rtCommShardKernel: the gather's band plan counts bands from image row 0, the kernel from the
// first row of its work range -- so a comm-sharded kernel renders whole frames only
int rti::shard_kernel(rt_kernel k, unsigned period, unsigned phase) {
    flush_kernel(k);
    if (!k) return RT_INVALID_KERNEL;
    if (k->range_first != 0 || k->range_last != 0) return RT_INVALID_OPERATION;
    int rc = rtKernelSetRowInterleave(k, period, phase);
    if (rc == RT_SUCCESS) k->comm_sharded = true;
    return rc;
}

extern "C" {

int rtEnqueueCopyBufferRectToPointer(rt_context ctx, rt_mem src, size_t src_offset, size_t src_pitch,
                                     size_t width_bytes, size_t rows, void* dst, size_t dst_pitch) {
    int rc = ensure_device(ctx);
    if (rc) return rc;
    if (ctx->pend_k) (void)rti::flush_frames(ctx);
    if (!src || src->ctx != ctx || !dst) return RT_INVALID_MEM_OBJECT;
    if (rows == 0 || width_bytes == 0) return RT_SUCCESS;
    if (width_bytes > src_pitch || width_bytes > dst_pitch) return RT_INVALID_VALUE;
    if (src_offset + (rows - 1) * src_pitch + width_bytes > src->size) return RT_INVALID_VALUE;
    if (ctx->readback_on_astream && ctx->overlap) {
        // after every accumulation enqueued so far, before any later one (astream is in order),
        // and after everything already queued on the main stream (a per-frame launch writes
        // `out` there; a fused render's tail is the accumulation's own dependency, so waiting on
        // it costs the overlap nothing); later main-stream work that joins (qs) waits for the
        // copy too
        hipError_t e = rti::main_tail_wait(ctx, ctx->astream);
        // ... and after the gathers queued so far (their unpack writes a root's image; nothing
        // else on astream waits for it)
        if (e == hipSuccess) e = rti::gather_wait(ctx, ctx->astream);
        if (e == hipSuccess)
            e = hipMemcpy2DAsync(dst, dst_pitch, static_cast<uint8_t*>(src->dptr) + src_offset, src_pitch,
                                 width_bytes, rows, hipMemcpyDeviceToDevice, ctx->astream);
        if (e == hipSuccess) e = hipEventRecord(ctx->atail, ctx->astream);
        if (e == hipSuccess) ctx->apending = true;
        return map_hip(e);
    }
    return map_hip(hipMemcpy2DAsync(dst, dst_pitch, static_cast<uint8_t*>(src->dptr) + src_offset, src_pitch,
                                    width_bytes, rows, hipMemcpyDeviceToDevice, qs(ctx)));
}

int rtContextSetReadbackOnAccumStream(rt_context ctx, int enable) {
    int rc = ensure_device(ctx);
    if (rc) return rc;
    if (ctx->pend_k) (void)rti::flush_frames(ctx);
    ctx->readback_on_astream = enable != 0;
    return RT_SUCCESS;
}

int rtContextGetAccumStream(rt_context ctx, void** s) {
    if (!ctx) return RT_INVALID_CONTEXT;
    if (!s) return RT_INVALID_VALUE;
    if (!ctx->overlap) ctx->mexposed = true;  // the main stream leaves the library's view
    ctx->dexposed = true;  // the caller may synchronise with the stream outside the library
    if (ctx->pend_k) (void)rti::flush_frames(ctx);
    *s = ctx->overlap ? ctx->astream : qs(ctx);
    return RT_SUCCESS;
}

int rtEnqueueCopyPointerRectToBuffer(rt_context ctx, const void* src, size_t src_pitch, rt_mem dst,
                                     size_t dst_offset, size_t dst_pitch, size_t width_bytes, size_t rows) {
    int rc = ensure_device(ctx);
    if (rc) return rc;
    if (ctx->pend_k) (void)rti::flush_frames(ctx);
    if (!dst || dst->ctx != ctx || !src) return RT_INVALID_MEM_OBJECT;
    if (rows == 0 || width_bytes == 0) return RT_SUCCESS;
    if (width_bytes > src_pitch || width_bytes > dst_pitch) return RT_INVALID_VALUE;
    if (dst_offset + (rows - 1) * dst_pitch + width_bytes > dst->size) return RT_INVALID_VALUE;
    dst->shadow_valid = false;  // device contents change: a scene buffer is re-read and repacked
    ++dst->generation;
    return map_hip(hipMemcpy2DAsync(static_cast<uint8_t*>(dst->dptr) + dst_offset, dst_pitch, src, src_pitch,
                                    width_bytes, rows, hipMemcpyDeviceToDevice, qs(ctx)));
}

int rtKernelSetWorkRange(rt_kernel k, uint64_t first, uint64_t last) {
    if (!k) return RT_INVALID_KERNEL;
    flush_kernel(k);
    if (last != 0 && last < first) return RT_INVALID_VALUE;
    if (k->comm_sharded && (first != 0 || last != 0)) return RT_INVALID_OPERATION;
    k->range_first = first;
    k->range_last = last;
    return RT_SUCCESS;
}

int rtKernelSetHitBuffers(rt_kernel k, rt_mem ids, rt_mem t) {
    if (!k) return RT_INVALID_KERNEL;
    flush_kernel(k);
    if ((ids == nullptr) != (t == nullptr)) return RT_INVALID_MEM_OBJECT;
    if (ids && (ids->ctx != k->ctx || t->ctx != k->ctx)) return RT_INVALID_MEM_OBJECT;
    k->hit_ids = ids;
    k->hit_t = t;
    return RT_SUCCESS;
}

int rtKernelSetStats(rt_kernel k, int enable) {
    if (!k) return RT_INVALID_KERNEL;
    flush_kernel(k);
    k->stats = enable != 0;
    return RT_SUCCESS;
}

int rtKernelSetTiming(rt_kernel k, int enable) {
    if (!k) return RT_INVALID_KERNEL;
    flush_kernel(k);
    k->timing = enable != 0;
    return RT_SUCCESS;
}

int rtKernelGetStats(rt_kernel k, rt_stats* out) {
    if (!k || !out) return RT_INVALID_VALUE;
    flush_kernel(k);
    int rc = ensure_device(k->ctx);
    if (rc) return rc;
    unsigned long long h[kStatWords] = {};
    hipError_t e = hipMemcpyAsync(h, k->dstats, sizeof(h), hipMemcpyDeviceToHost, qs(k->ctx));
    if (e == hipSuccess) e = hipStreamSynchronize(qs(k->ctx));
    if (e != hipSuccess) return map_hip(e);
    rc = drain_events(k);
    if (rc) return rc;
    out->rays = h[0];
    out->node_visits = h[1];
    out->tri_tests = h[2];
    out->hits = h[3];
    out->cycles_refill = h[4];
    out->cycles_traverse = h[5];
    out->cycles_shade = h[6];
    out->cycles_total = h[7];
    for (int i = 0; i < 12; ++i) out->sched[i] = h[8 + i];
    out->launches = k->launches;
    out->kernel_ms = k->kernel_ms;
    out->accum_ms = k->accum_ms;
    out->render_period_ms = k->period_intervals ? k->period_span_ms / (double)k->period_intervals : 0.0;
    return RT_SUCCESS;
}

int rtKernelResetStats(rt_kernel k) {
    if (!k) return RT_INVALID_KERNEL;
    flush_kernel(k);
    int rc = ensure_device(k->ctx);
    if (rc) return rc;
    rc = drain_events(k);
    if (rc) return rc;
    k->launches = 0;
    k->kernel_ms = 0.0;
    k->accum_ms = 0.0;
    reset_period(k);
    hipError_t e = hipMemsetAsync(k->dstats, 0, kStatWords * sizeof(unsigned long long), qs(k->ctx));
    if (e == hipSuccess) e = hipStreamSynchronize(qs(k->ctx));
    return map_hip(e);
}

int rtKernelGetSceneInLDS(rt_kernel k, int* in_lds) {
    if (!k || !in_lds) return RT_INVALID_VALUE;
    *in_lds = k->last_lds ? 1 : 0;
    return RT_SUCCESS;
}

int rtKernelForceGlobalScene(rt_kernel k, int force) {
    if (!k) return RT_INVALID_KERNEL;
    flush_kernel(k);
    k->force_global = force != 0;
    return RT_SUCCESS;
}

int rtBufferGetDevicePointer(rt_mem m, void** dptr) {
    if (!m || !dptr) return RT_INVALID_VALUE;
    if (m->ctx && m->ctx->pend_k) (void)rti::flush_frames(m->ctx);  // the caller may touch the bytes
    // ... at any later time, after synchronising outside the library: no more frame coalescing
    if (m->ctx) m->ctx->dexposed = true;
    *dptr = m->dptr;
    return RT_SUCCESS;
}

int rtBufferGetSize(rt_mem m, size_t* size) {
    if (!m || !size) return RT_INVALID_VALUE;
    *size = m->size;
    return RT_SUCCESS;
}

int rtContextGetStream(rt_context ctx, void** s) {
    if (!ctx || !s) return RT_INVALID_VALUE;
    // the caller may enqueue there, or synchronise with it, without going through the library
    // (qs below also launches any coalesced frames; none are held back from now on)
    ctx->mexposed = true;
    *s = qs(ctx);
    return RT_SUCCESS;
}

}  // extern "C"


extern "C" {

int rtContextGetDevice(rt_context ctx, int* d) {
    if (!ctx || !d) return RT_INVALID_VALUE;
    *d = ctx->device;
    return RT_SUCCESS;
}

int rtValidateBVH(const void* nodes, size_t n_nodes, size_t n_tris, int* depth) {
    if (!nodes || n_nodes == 0 || n_nodes >= (1u << 30) || n_tris >= (1ull << 32)) return RT_INVALID_VALUE;
    int d = 0;
    uint32_t used = 0;
    int rc = check_nodes(static_cast<const rt_cl_bvh_node*>(nodes), (uint32_t)n_nodes, (uint32_t)n_tris, &d, &used);
    if (rc == RT_SUCCESS && depth) *depth = d;
    return rc;
}

int rtKernelSetTuning(rt_kernel k, int param, int value) {
    if (!k) return RT_INVALID_KERNEL;
    flush_kernel(k);
    auto in = [&](int lo, int hi) { return value >= lo && value <= hi; };
    switch (param) {
        case RT_TUNE_REFILL_MIN:
            if (!in(1, 64)) return RT_INVALID_VALUE;
            k->refill_min = (uint32_t)value;
            k->refill_min_set = true;
            break;
        case RT_TUNE_SHADE_MIN: if (!in(1, 64)) return RT_INVALID_VALUE; k->shade_min = (uint32_t)value; break;
        case RT_TUNE_REFILL_MIN_GLOBAL: if (!in(0, 64)) return RT_INVALID_VALUE; k->refill_min_g = (uint32_t)value; break;
        case RT_TUNE_SHADE_MIN_GLOBAL: if (!in(0, 64)) return RT_INVALID_VALUE; k->shade_min_g = (uint32_t)value; break;
        case RT_TUNE_STEP_WEIGHT_NODE: if (!in(1, 1000)) return RT_INVALID_VALUE; k->w_node = (uint32_t)value; break;
        case RT_TUNE_STEP_WEIGHT_LEAF: if (!in(1, 1000)) return RT_INVALID_VALUE; k->w_leaf = (uint32_t)value; break;
        case RT_TUNE_CHUNK_PIXELS:
            if (!in(0, 4096) || value % 64) return RT_INVALID_VALUE;  // (0: auto)
            k->chunk_pixels = (uint32_t)value;
            break;
        case RT_TUNE_TAIL_CHUNK:
            if (!in(64, 4096) || value % 64) return RT_INVALID_VALUE;
            k->tail_chunk = (uint32_t)value;
            break;
        case RT_TUNE_BULK_PERCENT: if (!in(0, 100)) return RT_INVALID_VALUE; k->bulk_percent = (uint32_t)value; break;
        case RT_TUNE_TOP_NODES: if (!in(0, 1024)) return RT_INVALID_VALUE; k->top_limit = (uint32_t)value; k->packed_nodes_gen = ~0ull; break;
        case RT_TUNE_TILE_MAJOR: if (!in(-1, 2)) return RT_INVALID_VALUE; k->tile_major = value; break;
        case RT_TUNE_MAX_BLOCKS: if (!in(0, 64)) return RT_INVALID_VALUE; k->max_blocks = value; break;
        case RT_TUNE_PERFRAME_SKY: if (!in(0, 2)) return RT_INVALID_VALUE; k->pf_sky = value; break;
        case RT_TUNE_WF_REFILL_MIN: if (!in(1, 64)) return RT_INVALID_VALUE; k->wf_refill_min = (uint32_t)value; break;
        case RT_TUNE_WF_STREAMS_PER_CU: if (!in(0, 64)) return RT_INVALID_VALUE; k->wf_streams_per_cu = (uint32_t)value; break;
        case RT_TUNE_WF_TOP_NODES: if (!in(0, 1024)) return RT_INVALID_VALUE; k->wf_top_limit = (uint32_t)value; break;
        case RT_TUNE_GLOBAL_OCT: if (!in(0, 1)) return RT_INVALID_VALUE; k->global_oct = value; break;
        case RT_TUNE_PERFRAME_DEFER: if (!in(0, 2)) return RT_INVALID_VALUE; k->pf_defer = value; break;
        case RT_TUNE_PERFRAME_DEFER_MIN: if (value < 0) return RT_INVALID_VALUE; k->pf_defer_min = (uint32_t)value; break;
        case RT_TUNE_PERFRAME_BATCH: if (!in(1, (int)rtk::kMaxFusedFrames)) return RT_INVALID_VALUE; k->pf_batch = (uint32_t)value; break;
        case RT_TUNE_STEP_WEIGHT_NODE_GLOBAL: if (!in(0, 1000)) return RT_INVALID_VALUE; k->w_node_g = (uint32_t)value; break;
        case RT_TUNE_STEP_WEIGHT_LEAF_GLOBAL: if (!in(0, 1000)) return RT_INVALID_VALUE; k->w_leaf_g = (uint32_t)value; break;
        default: return RT_INVALID_VALUE;
    }
    return RT_SUCCESS;
}

int rtKernelGetTuning(rt_kernel k, int param, int* value) {
    if (!k) return RT_INVALID_KERNEL;
    if (!value) return RT_INVALID_VALUE;
    switch (param) {
        case RT_TUNE_REFILL_MIN: *value = (int)k->refill_min; break;
        case RT_TUNE_SHADE_MIN: *value = (int)k->shade_min; break;
        case RT_TUNE_REFILL_MIN_GLOBAL: *value = (int)k->refill_min_g; break;
        case RT_TUNE_SHADE_MIN_GLOBAL: *value = (int)k->shade_min_g; break;
        case RT_TUNE_STEP_WEIGHT_NODE: *value = (int)k->w_node; break;
        case RT_TUNE_STEP_WEIGHT_LEAF: *value = (int)k->w_leaf; break;
        case RT_TUNE_CHUNK_PIXELS: *value = (int)k->chunk_pixels; break;
        case RT_TUNE_TAIL_CHUNK: *value = (int)k->tail_chunk; break;
        case RT_TUNE_BULK_PERCENT: *value = (int)k->bulk_percent; break;
        case RT_TUNE_TOP_NODES: *value = (int)k->top_limit; break;
        case RT_TUNE_TILE_MAJOR: *value = k->tile_major; break;
        case RT_TUNE_MAX_BLOCKS: *value = k->max_blocks; break;
        case RT_TUNE_PERFRAME_SKY: *value = k->pf_sky; break;
        case RT_TUNE_WF_REFILL_MIN: *value = (int)k->wf_refill_min; break;
        case RT_TUNE_WF_STREAMS_PER_CU: *value = (int)k->wf_streams_per_cu; break;
        case RT_TUNE_WF_TOP_NODES: *value = (int)k->wf_top_limit; break;
        case RT_TUNE_GLOBAL_OCT: *value = k->global_oct; break;
        case RT_TUNE_PERFRAME_DEFER: *value = k->pf_defer; break;
        case RT_TUNE_PERFRAME_DEFER_MIN: *value = (int)k->pf_defer_min; break;
        case RT_TUNE_PERFRAME_BATCH: *value = (int)k->pf_batch; break;
        case RT_TUNE_STEP_WEIGHT_NODE_GLOBAL: *value = (int)k->w_node_g; break;
        case RT_TUNE_STEP_WEIGHT_LEAF_GLOBAL: *value = (int)k->w_leaf_g; break;
        default: return RT_INVALID_VALUE;
    }
    return RT_SUCCESS;
}

int rtContextSetAccumOverlap(rt_context ctx, int enable) {
    int rc = ensure_device(ctx);
    if (rc) return rc;
    // switching modes: everything queued so far completes on the old arrangement first
    hipError_t e = hipStreamSynchronize(qs(ctx));
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->astream);
    if (e != hipSuccess) return map_hip(e);
    ctx->overlap = enable != 0;
    return RT_SUCCESS;
}

int rtDiagPinnedMath(int device_index, int op, const float* a, const float* b, float* out, size_t n) {
    if (op < RT_PINNED_OP_RCP || op > RT_PINNED_OP_COS || !a || !out) return RT_INVALID_VALUE;
    const bool two = op == RT_PINNED_OP_DIV || op == RT_PINNED_OP_POW;
    if (two && !b) return RT_INVALID_VALUE;
    if (n == 0) return RT_SUCCESS;
    if (n > ((size_t)1 << 28)) return RT_INVALID_BUFFER_SIZE;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count == 0) return RT_DEVICE_NOT_FOUND;
    if (device_index < 0 || device_index >= count) return RT_INVALID_DEVICE;
    hipError_t e = hipSetDevice(device_index);
    float* d = nullptr;
    const size_t bytes = n * sizeof(float);
    if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&d), 3 * bytes);
    if (e == hipSuccess) e = hipMemcpy(d, a, bytes, hipMemcpyHostToDevice);
    if (e == hipSuccess && two) e = hipMemcpy(d + n, b, bytes, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = rtk::launch_pinned_math(op, d, d + n, d + 2 * n, n, nullptr);
    if (e == hipSuccess) e = hipMemcpy(out, d + 2 * n, bytes, hipMemcpyDeviceToHost);
    if (d) (void)hipFree(d);
    return map_hip(e);
}

const char* rtGetBuildInfo(void) {
    return "librt_hip: KernelEntry for gfx950 (HIP), math modes pinned|devicelib|shipped, scene in LDS or HBM";
}

}  // extern "C"
