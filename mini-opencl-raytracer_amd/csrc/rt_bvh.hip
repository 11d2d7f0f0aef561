// rt_bvh.hip -- device-side BVH build.
//
// The reference builds its BVH on the host: pbrt-style SAH, then a depth-first flatten into
// CLLinearBVHNode[] (CLBVHnode.cpp:7-207); host/scene.cpp restates that exactly.  For large
// meshes this builds a linear BVH on the GPU instead and writes the SAME node contract
// (CLBVHnode.cpp:161-183): depth-first order, first child = parent + 1, `offset` = second
// child (interior) or first triangle (leaf), nPrimitives <= maxPrimitivesInNode for leaves,
// `axis` = the axis of the node's largest extent; triangles are permuted into leaf order.
// The hot-path kernels therefore render it unchanged.  The tree differs from the SAH tree,
// so hit IDs and the images' last bits may differ from a host-built scene wherever two
// triangles tie (the Cornell OBJ holds every face twice): parity is per geometry, and a
// render of the device-built tree is bit-exact with the oracle rendering the same arrays.
//
// Two topologies over the same Morton order (rtBuildBVHEx): PLOC (default, below: SAH-like trees
// by bottom-up clustering) or the linear BVH of Karras (2012).
//
// LBVH steps: centroid bounds (block reduction) -> 30-bit Morton codes -> rocPRIM radix sort
// (stable: equal codes keep triangle order) -> Karras (2012) binary radix tree over the
// sorted order, ties broken by position -> bottom-up bounds and output-subtree sizes
// (atomic arrival counters) -> every subtree with <= maxPrims triangles becomes one leaf
// (its triangles are contiguous in sorted order) -> depth-first index of each output node by
// walking to the root -> node records + triangle gather.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include "../../include/rt_cl_types.h"
#include "rt_bvh.hpp"

namespace rtb {

constexpr uint32_t kLeafFlag = 0x80000000u;

struct Box {
    float lo[3], hi[3];
};

__device__ inline float3 tri_centroid(const rt_cl_triangle& t) {
    return make_float3((t.v1.position.x + t.v2.position.x + t.v3.position.x) * (1.0f / 3.0f),
                       (t.v1.position.y + t.v2.position.y + t.v3.position.y) * (1.0f / 3.0f),
                       (t.v1.position.z + t.v2.position.z + t.v3.position.z) * (1.0f / 3.0f));
}

__device__ inline Box tri_box(const rt_cl_triangle& t) {
    Box b;
    b.lo[0] = fminf(fminf(t.v1.position.x, t.v2.position.x), t.v3.position.x);
    b.lo[1] = fminf(fminf(t.v1.position.y, t.v2.position.y), t.v3.position.y);
    b.lo[2] = fminf(fminf(t.v1.position.z, t.v2.position.z), t.v3.position.z);
    b.hi[0] = fmaxf(fmaxf(t.v1.position.x, t.v2.position.x), t.v3.position.x);
    b.hi[1] = fmaxf(fmaxf(t.v1.position.y, t.v2.position.y), t.v3.position.y);
    b.hi[2] = fmaxf(fmaxf(t.v1.position.z, t.v2.position.z), t.v3.position.z);
    return b;
}

// per-block centroid bounds, then one block folds the partials
__global__ void centroid_bounds(const rt_cl_triangle* __restrict__ tris, uint32_t n, float* __restrict__ part) {
    __shared__ float s[6][256];
    float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
        const float3 c = tri_centroid(tris[i]);
        lo[0] = fminf(lo[0], c.x), lo[1] = fminf(lo[1], c.y), lo[2] = fminf(lo[2], c.z);
        hi[0] = fmaxf(hi[0], c.x), hi[1] = fmaxf(hi[1], c.y), hi[2] = fmaxf(hi[2], c.z);
    }
    for (int k = 0; k < 3; ++k) {
        s[k][threadIdx.x] = lo[k];
        s[3 + k][threadIdx.x] = hi[k];
    }
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w)
            for (int k = 0; k < 3; ++k) {
                s[k][threadIdx.x] = fminf(s[k][threadIdx.x], s[k][threadIdx.x + w]);
                s[3 + k][threadIdx.x] = fmaxf(s[3 + k][threadIdx.x], s[3 + k][threadIdx.x + w]);
            }
        __syncthreads();
    }
    if (threadIdx.x < 6) part[blockIdx.x * 6 + threadIdx.x] = s[threadIdx.x][0];
}

__device__ inline uint32_t expand_bits(uint32_t v) {  // 10 bits -> every third bit
    v = (v * 0x00010001u) & 0xFF0000FFu;
    v = (v * 0x00000101u) & 0x0F00F00Fu;
    v = (v * 0x00000011u) & 0xC30C30C3u;
    v = (v * 0x00000005u) & 0x49249249u;
    return v;
}

__global__ void morton_codes(const rt_cl_triangle* __restrict__ tris, uint32_t n, const float* __restrict__ part,
                             uint32_t n_parts, uint32_t* __restrict__ keys, uint32_t* __restrict__ vals) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (uint32_t p = 0; p < n_parts; ++p)
        for (int k = 0; k < 3; ++k) {
            lo[k] = fminf(lo[k], part[p * 6 + k]);
            hi[k] = fmaxf(hi[k], part[p * 6 + 3 + k]);
        }
    const float3 c = tri_centroid(tris[i]);
    const float cc[3] = {c.x, c.y, c.z};
    uint32_t code = 0;
    for (int k = 0; k < 3; ++k) {
        const float ext = hi[k] - lo[k];
        float u = ext > 0.0f ? (cc[k] - lo[k]) / ext : 0.0f;
        u = fminf(fmaxf(u, 0.0f), 1.0f);
        const uint32_t q = (uint32_t)fminf(u * 1024.0f, 1023.0f);
        code |= expand_bits(q) << (2 - k);
    }
    keys[i] = code;
    vals[i] = i;
}

// common-prefix length of sorted keys i and j (positions break ties); -1 outside the array
__device__ inline int delta(const uint32_t* keys, int n, int i, int j) {
    if (j < 0 || j >= n) return -1;
    const uint32_t a = keys[i], b = keys[j];
    if (a != b) return __clz(a ^ b);
    return 32 + __clz((uint32_t)i ^ (uint32_t)j);
}

// Karras 2012: internal node i's children and covered range
__global__ void radix_tree(const uint32_t* __restrict__ keys, int n, uint32_t* __restrict__ left,
                           uint32_t* __restrict__ right, uint32_t* __restrict__ first, uint32_t* __restrict__ last,
                           uint32_t* __restrict__ parent_int, uint32_t* __restrict__ parent_leaf) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n - 1) return;
    const int d = (delta(keys, n, i, i + 1) - delta(keys, n, i, i - 1)) >= 0 ? 1 : -1;
    const int dmin = delta(keys, n, i, i - d);
    int lmax = 2;
    while (delta(keys, n, i, i + lmax * d) > dmin) lmax *= 2;
    int l = 0;
    for (int t = lmax / 2; t >= 1; t /= 2)
        if (delta(keys, n, i, i + (l + t) * d) > dmin) l += t;
    const int j = i + l * d;
    const int dnode = delta(keys, n, i, j);
    int s = 0;
    for (int t = (l + 1) / 2;; t = (t + 1) / 2) {
        if (delta(keys, n, i, i + (s + t) * d) > dnode) s += t;
        if (t == 1) break;
    }
    const int g = i + s * d + (d < 0 ? -1 : 0);
    const int lo = min(i, j), hi = max(i, j);
    const uint32_t lc = (lo == g) ? (kLeafFlag | (uint32_t)g) : (uint32_t)g;
    const uint32_t rc = (hi == g + 1) ? (kLeafFlag | (uint32_t)(g + 1)) : (uint32_t)(g + 1);
    left[i] = lc;
    right[i] = rc;
    first[i] = (uint32_t)lo;
    last[i] = (uint32_t)hi;
    if (lc & kLeafFlag) parent_leaf[g] = (uint32_t)i; else parent_int[g] = (uint32_t)i;
    if (rc & kLeafFlag) parent_leaf[g + 1] = (uint32_t)i; else parent_int[g + 1] = (uint32_t)i;
}

// bottom-up: bounds of every internal node and the size of its output subtree (a subtree
// with <= max_prims triangles is ONE output leaf)
__global__ void bottom_up(const rt_cl_triangle* __restrict__ tris, const uint32_t* __restrict__ order, int n,
                          uint32_t max_prims, const uint32_t* __restrict__ left, const uint32_t* __restrict__ right,
                          const uint32_t* __restrict__ first, const uint32_t* __restrict__ last,
                          const uint32_t* __restrict__ parent_int, const uint32_t* __restrict__ parent_leaf,
                          uint32_t* __restrict__ arrivals, Box* __restrict__ leaf_box, Box* __restrict__ int_box,
                          uint32_t* __restrict__ osize) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    leaf_box[k] = tri_box(tris[order[k]]);
    if (n == 1) return;
    __threadfence();
    uint32_t node = parent_leaf[k];
    for (;;) {
        if (atomicAdd(&arrivals[node], 1u) == 0u) return;  // the sibling subtree finishes this node
        __threadfence();
        const uint32_t l = left[node], r = right[node];
        const Box bl = (l & kLeafFlag) ? leaf_box[l & ~kLeafFlag] : int_box[l];
        const Box br = (r & kLeafFlag) ? leaf_box[r & ~kLeafFlag] : int_box[r];
        Box b;
        for (int a = 0; a < 3; ++a) {
            b.lo[a] = fminf(bl.lo[a], br.lo[a]);
            b.hi[a] = fmaxf(bl.hi[a], br.hi[a]);
        }
        int_box[node] = b;
        const uint32_t cnt = last[node] - first[node] + 1u;
        if (cnt <= max_prims) {
            osize[node] = 1u;
        } else {
            const uint32_t sl = (l & kLeafFlag) ? 1u : osize[l];
            const uint32_t sr = (r & kLeafFlag) ? 1u : osize[r];
            osize[node] = 1u + sl + sr;
        }
        __threadfence();
        if (node == 0u) return;
        node = parent_int[node];
    }
}

// one thread per Karras node (internal nodes 0..n-2, then leaves): if it is an output node,
// find its depth-first index by walking to the root and write its record
__global__ void emit_nodes(int n, uint32_t max_prims, const uint32_t* __restrict__ left,
                           const uint32_t* __restrict__ right, const uint32_t* __restrict__ first,
                           const uint32_t* __restrict__ last, const uint32_t* __restrict__ parent_int,
                           const uint32_t* __restrict__ parent_leaf, const Box* __restrict__ leaf_box,
                           const Box* __restrict__ int_box, const uint32_t* __restrict__ osize,
                           rt_cl_bvh_node* __restrict__ out) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    const int n_int = n - 1;
    if (t >= n_int + n) return;
    const bool is_leaf = t >= n_int;
    const uint32_t id = is_leaf ? (uint32_t)(t - n_int) : (uint32_t)t;
    const uint32_t self = is_leaf ? (kLeafFlag | id) : id;
    auto count_of = [&](uint32_t c) { return (c & kLeafFlag) ? 1u : last[c] - first[c] + 1u; };
    auto osize_of = [&](uint32_t c) { return (c & kLeafFlag) ? 1u : osize[c]; };
    auto parent_of = [&](uint32_t c) { return (c & kLeafFlag) ? parent_leaf[c & ~kLeafFlag] : parent_int[c]; };
    // output node: the root, or a node whose parent is an output interior node
    bool emit;
    if (n == 1) {
        emit = true;
    } else if (!is_leaf && id == 0u) {
        emit = true;
    } else {
        emit = count_of(parent_of(self)) > max_prims;
    }
    if (!emit) return;
    // depth-first index: root 0; left child = parent + 1; right child = parent + 1 + osize(left)
    uint32_t idx = 0;
    uint32_t c = self;
    while (!(n == 1 || (!(c & kLeafFlag) && c == 0u))) {
        const uint32_t p = parent_of(c);
        idx += 1u;
        if (right[p] == c) idx += osize_of(left[p]);
        c = p;
    }
    rt_cl_bvh_node nd;
    for (int k = 0; k < 9; ++k) nd.pad[k] = 0;
    const Box b = (n == 1) ? leaf_box[0] : (is_leaf ? leaf_box[id] : int_box[id]);
    nd.bounds.pmin = rt_float3{b.lo[0], b.lo[1], b.lo[2], 0.0f};
    nd.bounds.pmax = rt_float3{b.hi[0], b.hi[1], b.hi[2], 0.0f};
    const uint32_t cnt = (n == 1) ? 1u : count_of(self);
    if (is_leaf || n == 1 || cnt <= max_prims) {
        nd.offset = (n == 1 || is_leaf) ? id : first[id];
        nd.nPrimitives = (uint16_t)cnt;
        nd.axis = 0;
    } else {
        nd.offset = idx + 1u + osize_of(left[id]);
        nd.nPrimitives = 0;
        const float ex = b.hi[0] - b.lo[0], ey = b.hi[1] - b.lo[1], ez = b.hi[2] - b.lo[2];
        nd.axis = (uint8_t)((ex >= ey && ex >= ez) ? 0 : (ey >= ez ? 1 : 2));
    }
    out[idx] = nd;
}

__global__ void gather_tris(const rt_cl_triangle* __restrict__ in, const uint32_t* __restrict__ order, uint32_t n,
                            rt_cl_triangle* __restrict__ out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = in[order[i]];
}

// ---- PLOC: parallel locally-ordered clustering (Meister & Bittner 2018) -----------------------
// The same Morton order, but the tree is built bottom-up by merging clusters: every cluster finds
// the neighbour within kPlocRadius positions whose union box has the least surface area, mutual
// nearest neighbours merge (the lower position keeps the new cluster, in Morton order), the cluster
// array is compacted, until one cluster is left.  SAH-like trees at a linear BVH's build cost.
// Nodes 0 .. n-1 are the triangles (sorted positions), n .. 2n-2 the merges (allocated in merge
// order; the output depends only on the topology, so it is deterministic).
#ifndef RT_PLOC_RADIUS
#define RT_PLOC_RADIUS 32
#endif
constexpr int kPlocRadius = RT_PLOC_RADIUS;
constexpr uint32_t kNoParent = 0xffffffffu;

__device__ inline Box box_union(const Box& a, const Box& b) {
    Box u;
    for (int k = 0; k < 3; ++k) {
        u.lo[k] = fminf(a.lo[k], b.lo[k]);
        u.hi[k] = fmaxf(a.hi[k], b.hi[k]);
    }
    return u;
}
__device__ inline float box_area(const Box& b) {
    const float dx = b.hi[0] - b.lo[0], dy = b.hi[1] - b.lo[1], dz = b.hi[2] - b.lo[2];
    return 2.0f * (dx * dy + dy * dz + dz * dx);
}

__global__ void ploc_init(const rt_cl_triangle* __restrict__ tris, const uint32_t* __restrict__ order, uint32_t n,
                          Box* __restrict__ box, uint32_t* __restrict__ cnt, uint32_t* __restrict__ parent,
                          uint32_t* __restrict__ clus) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        box[i] = tri_box(tris[order[i]]);
        cnt[i] = 1u;
        clus[i] = i;
    }
    if (i < 2 * n - 1) parent[i] = kNoParent;
}

// nearest neighbour (least union surface area; ties: the lower position) of clusters [0, m)
__global__ void ploc_nn(const uint32_t* __restrict__ clus, uint32_t m, const Box* __restrict__ box,
                        uint32_t* __restrict__ nn) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    const Box bi = box[clus[i]];
    const uint32_t lo = i > (uint32_t)kPlocRadius ? i - kPlocRadius : 0u;
    const uint32_t hi = min(m - 1u, i + (uint32_t)kPlocRadius);
    float best = INFINITY;
    uint32_t bj = i == 0u ? 1u : i - 1u;
    for (uint32_t j = lo; j <= hi; ++j) {
        if (j == i) continue;
        const float c = box_area(box_union(bi, box[clus[j]]));
        if (c < best) {
            best = c;
            bj = j;
        }
    }
    nn[i] = bj;
}

// mutual nearest neighbours merge (force: pairs (0,1), (2,3), ... -- only after a round that merged
// (almost) nothing, which happens only where costs tie across the whole window)
__global__ void ploc_merge(const uint32_t* __restrict__ clus, uint32_t m, const uint32_t* __restrict__ nn,
                           uint32_t n, uint32_t force, Box* __restrict__ box, uint32_t* __restrict__ cnt,
                           uint32_t* __restrict__ left, uint32_t* __restrict__ right, uint32_t* __restrict__ parent,
                           uint32_t* __restrict__ counter, uint32_t* __restrict__ next, uint32_t* __restrict__ flag) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    uint32_t j = nn[i];
    bool pair = nn[j] == i;
    if (force) {
        j = i ^ 1u;
        pair = j < m;
    }
    if (pair && i > j) {
        flag[i] = 0u;
        return;
    }
    if (pair) {
        const uint32_t k = atomicAdd(counter, 1u), id = n + k;
        const uint32_t a = clus[i], b = clus[j];
        left[k] = a;
        right[k] = b;
        parent[a] = id;
        parent[b] = id;
        box[id] = box_union(box[a], box[b]);
        cnt[id] = cnt[a] + cnt[b];
        next[i] = id;
    } else {
        next[i] = clus[i];
    }
    flag[i] = 1u;
}

__global__ void ploc_compact(uint32_t m, const uint32_t* __restrict__ next, const uint32_t* __restrict__ flag,
                             const uint32_t* __restrict__ pos, uint32_t* __restrict__ clus_out,
                             uint32_t* __restrict__ m_out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    if (flag[i]) clus_out[pos[i]] = next[i];
    if (i == m - 1u) *m_out = pos[i] + flag[i];
}

// the axis along which two boxes' centres lie furthest apart (the node's `axis`: the walk visits
// the second child first when the ray points down that axis, kernel_bvh.cl:200-207)
__device__ inline int child_axis(const Box& a, const Box& b) {
    float d[3];
    for (int k = 0; k < 3; ++k) d[k] = fabsf((b.lo[k] + b.hi[k]) - (a.lo[k] + a.hi[k]));
    return (d[0] >= d[1] && d[0] >= d[2]) ? 0 : (d[1] >= d[2] ? 1 : 2);
}

// order every merge's children along that axis (first child = the lower one), as a split would
__global__ void ploc_orient(uint32_t n, const Box* __restrict__ box, uint32_t* __restrict__ left,
                            uint32_t* __restrict__ right) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k + 1 >= n) return;
    const uint32_t a = left[k], b = right[k];
    const int ax = child_axis(box[a], box[b]);
    if (box[a].lo[ax] + box[a].hi[ax] > box[b].lo[ax] + box[b].hi[ax]) {
        left[k] = b;
        right[k] = a;
    }
}

// output-subtree sizes bottom-up; osize 1 = the node is an output leaf.  RT_PLOC_SAH_LEAVES 0: every
// subtree of <= max_prims triangles is one leaf; 1: such a subtree becomes a leaf only where the
// surface area heuristic prefers it, as the reference's SAH build decides (CLBVHnode.cpp, pbrt:
// leaf cost = triangles, split cost = 1 + children's costs weighted by area), here on the
// children's own (recursive) costs
#ifndef RT_PLOC_SAH_LEAVES
#define RT_PLOC_SAH_LEAVES 0
#endif
__global__ void ploc_sizes(uint32_t n, uint32_t max_prims, const uint32_t* __restrict__ left,
                           const uint32_t* __restrict__ right, const uint32_t* __restrict__ parent,
                           const uint32_t* __restrict__ cnt, const Box* __restrict__ box, float* __restrict__ cost,
                           uint32_t* __restrict__ arrivals, uint32_t* __restrict__ osize) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    osize[p] = 1u;
    cost[p] = 1.0f;
    __threadfence();
    uint32_t node = parent[p];
    while (node != kNoParent) {
        const uint32_t k = node - n;
        if (atomicAdd(&arrivals[k], 1u) == 0u) return;  // the sibling subtree finishes this node
        __threadfence();
        const uint32_t l = left[k], r = right[k];
        bool leaf = cnt[node] <= max_prims;
        float c = (float)cnt[node];
        if (RT_PLOC_SAH_LEAVES) {
            const float a = box_area(box[node]);
            const float split = a > 0.0f ? 1.0f + (box_area(box[l]) * cost[l] + box_area(box[r]) * cost[r]) / a
                                         : 1.0f + cost[l] + cost[r];
            leaf = leaf && c <= split;
            if (!leaf) c = split;
        }
        cost[node] = c;
        osize[node] = leaf ? 1u : 1u + osize[l] + osize[r];
        __threadfence();
        node = parent[node];
    }
}

// every node: its depth-first index and first triangle (walk to the root); output nodes write
// their record, triangle nodes write their triangle at its depth-first position
__global__ void ploc_emit(uint32_t n, uint32_t max_prims, uint32_t root, const uint32_t* __restrict__ left,
                          const uint32_t* __restrict__ right, const uint32_t* __restrict__ parent,
                          const uint32_t* __restrict__ cnt, const uint32_t* __restrict__ osize,
                          const Box* __restrict__ box, const rt_cl_triangle* __restrict__ in,
                          const uint32_t* __restrict__ order, rt_cl_triangle* __restrict__ tris_out,
                          rt_cl_bvh_node* __restrict__ out) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= 2 * n - 1) return;
    uint32_t idx = 0, first = 0;
    bool inside = false;  // below an output leaf
    for (uint32_t c = t; c != root;) {
        const uint32_t par = parent[c], k = par - n;
        idx += 1u;
        if (right[k] == c) {
            idx += osize[left[k]];
            first += cnt[left[k]];
        }
        inside = inside || osize[par] == 1u;
        c = par;
    }
    if (t < n) tris_out[first] = in[order[t]];
    if (inside) return;
    rt_cl_bvh_node nd;
    for (int k = 0; k < 9; ++k) nd.pad[k] = 0;
    const Box b = box[t];
    nd.bounds.pmin = rt_float3{b.lo[0], b.lo[1], b.lo[2], 0.0f};
    nd.bounds.pmax = rt_float3{b.hi[0], b.hi[1], b.hi[2], 0.0f};
    if (osize[t] == 1u) {
        nd.offset = first;
        nd.nPrimitives = (uint16_t)cnt[t];
        nd.axis = 0;
    } else {
        nd.offset = idx + 1u + osize[left[t - n]];
        nd.nPrimitives = 0;
        nd.axis = (uint8_t)child_axis(box[left[t - n]], box[right[t - n]]);
    }
    out[idx] = nd;
}

}  // namespace rtb

namespace rtb {

// rocPRIM's temporary-storage query for the PLOC compaction scan; false when the query fails
static bool scan_bytes(uint32_t n, size_t& b) {
    b = 0;
    return rocprim::exclusive_scan((void*)nullptr, b, (const uint32_t*)nullptr, (uint32_t*)nullptr, 0u,
                                   (size_t)(n ? n : 1), rocprim::plus<uint32_t>()) == hipSuccess;
}

// Scratch bytes rtb::build needs for n triangles, or 0 when a rocPRIM size query fails (the caller
// reports an error instead of building in an under-sized scratch).
size_t scratch_bytes(uint32_t n) {
    const size_t nn = n ? n : 1;
    size_t sort_bytes = 0, sb = 0;
    if (rocprim::radix_sort_pairs((void*)nullptr, sort_bytes, (uint32_t*)nullptr, (uint32_t*)nullptr,
                                  (uint32_t*)nullptr, (uint32_t*)nullptr, (unsigned int)nn, 0, 30) != hipSuccess)
        return 0;
    if (!scan_bytes(n, sb)) return 0;
    auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
    const size_t common = al(64 * 6 * sizeof(float)) + 4 * al(nn * 4) +  // partials, keys/vals in+out
                          al(nn * sizeof(rt_cl_triangle)) + al(sort_bytes);  // triangle copy, sort temp
    const size_t lbvh = 6 * al(nn * 4) + al(nn * 4) +                   // tree arrays, arrivals
                        al(nn * sizeof(Box)) * 2 + al(nn * 4);          // boxes, osize
    const size_t ploc = al(2 * nn * sizeof(Box)) + 4 * al(2 * nn * 4) +  // boxes, cnt, parent, osize, cost
                        3 * al(nn * 4) +                                 // left, right, arrivals
                        7 * al(nn * 4) + al(16) + al(sb);                // clusters x2, nn, next, flag, pos, m
    return common + (lbvh > ploc ? lbvh : ploc);
}

static hipError_t build_ploc(rt_cl_triangle* tris, uint32_t n, uint32_t max_prims, rt_cl_bvh_node* nodes,
                             uint32_t* n_nodes, uint8_t* p, rt_cl_triangle* copy, const uint32_t* svals,
                             hipStream_t st);

hipError_t build(rt_cl_triangle* tris, uint32_t n, uint32_t max_prims, rt_cl_bvh_node* nodes, uint32_t* n_nodes,
                 void* scratch, hipStream_t st, int method) {
    if (n == 0) return hipErrorInvalidValue;
    auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
    uint8_t* p = static_cast<uint8_t*>(scratch);
    auto take = [&](size_t b) {
        void* r = p;
        p += al(b);
        return r;
    };
    const size_t nn = n;
    float* part = (float*)take(64 * 6 * sizeof(float));
    uint32_t* keys = (uint32_t*)take(nn * 4);
    uint32_t* vals = (uint32_t*)take(nn * 4);
    uint32_t* skeys = (uint32_t*)take(nn * 4);
    uint32_t* svals = (uint32_t*)take(nn * 4);
    rt_cl_triangle* copy = (rt_cl_triangle*)take(nn * sizeof(rt_cl_triangle));
    size_t sort_bytes = 0;
    hipError_t e = rocprim::radix_sort_pairs((void*)nullptr, sort_bytes, keys, skeys, vals, svals, (unsigned int)n, 0,
                                             30, st);
    if (e != hipSuccess) return e;
    void* sort_tmp = take(sort_bytes);

    const uint32_t parts = 64;
    const dim3 b256(256);
    hipLaunchKernelGGL(centroid_bounds, dim3(parts), b256, 0, st, tris, n, part);
    hipLaunchKernelGGL(morton_codes, dim3((n + 255) / 256), b256, 0, st, tris, n, part, parts, keys, vals);
    e = rocprim::radix_sort_pairs(sort_tmp, sort_bytes, keys, skeys, vals, svals, (unsigned int)n, 0, 30, st);
    if (e != hipSuccess) return e;
    if (method == 1) return build_ploc(tris, n, max_prims, nodes, n_nodes, p, copy, svals, st);

    uint32_t* left = (uint32_t*)take(nn * 4);
    uint32_t* right = (uint32_t*)take(nn * 4);
    uint32_t* first = (uint32_t*)take(nn * 4);
    uint32_t* last = (uint32_t*)take(nn * 4);
    uint32_t* pint = (uint32_t*)take(nn * 4);
    uint32_t* pleaf = (uint32_t*)take(nn * 4);
    uint32_t* arrivals = (uint32_t*)take(nn * 4);
    Box* lbox = (Box*)take(nn * sizeof(Box));
    Box* ibox = (Box*)take(nn * sizeof(Box));
    uint32_t* osize = (uint32_t*)take(nn * 4);
    if (n > 1) {
        hipLaunchKernelGGL(radix_tree, dim3((n - 1 + 255) / 256), b256, 0, st, skeys, (int)n, left, right, first, last,
                           pint, pleaf);
    }
    e = hipMemsetAsync(arrivals, 0, nn * 4, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(bottom_up, dim3((n + 255) / 256), b256, 0, st, tris, svals, (int)n, max_prims, left, right,
                       first, last, pint, pleaf, arrivals, lbox, ibox, osize);
    // output node count = osize(root) (a root with <= max_prims triangles is the only leaf)
    uint32_t total = 1;
    if (n > 1) {
        e = hipMemcpyAsync(&total, osize, 4, hipMemcpyDeviceToHost, st);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        if (e != hipSuccess) return e;
    }
    const uint32_t threads = (n - 1) + n;  // internal nodes, then leaves (n == 1: the single leaf)
    hipLaunchKernelGGL(emit_nodes, dim3((threads + 255) / 256), b256, 0, st, (int)n, max_prims, left, right, first,
                       last, pint, pleaf, lbox, ibox, osize, nodes);
    e = hipMemcpyAsync(copy, tris, nn * sizeof(rt_cl_triangle), hipMemcpyDeviceToDevice, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(gather_tris, dim3((n + 255) / 256), b256, 0, st, copy, svals, n, tris);
    *n_nodes = total;
    return hipGetLastError();
}

// PLOC over the sorted order `svals` (scratch from `p` on); the triangles are gathered from `copy`
static hipError_t build_ploc(rt_cl_triangle* tris, uint32_t n, uint32_t max_prims, rt_cl_bvh_node* nodes,
                             uint32_t* n_nodes, uint8_t* p, rt_cl_triangle* copy, const uint32_t* svals,
                             hipStream_t st) {
    auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
    auto take = [&](size_t b) {
        void* r = p;
        p += al(b);
        return r;
    };
    const size_t nn = n, n2 = 2 * nn;
    Box* box = (Box*)take(n2 * sizeof(Box));
    uint32_t* cnt = (uint32_t*)take(n2 * 4);
    uint32_t* parent = (uint32_t*)take(n2 * 4);
    uint32_t* osize = (uint32_t*)take(n2 * 4);
    float* cost = (float*)take(n2 * 4);
    uint32_t* left = (uint32_t*)take(nn * 4);
    uint32_t* right = (uint32_t*)take(nn * 4);
    uint32_t* arrivals = (uint32_t*)take(nn * 4);
    uint32_t* clus[2] = {(uint32_t*)take(nn * 4), (uint32_t*)take(nn * 4)};
    uint32_t* nnb = (uint32_t*)take(nn * 4);
    uint32_t* next = (uint32_t*)take(nn * 4);
    uint32_t* flag = (uint32_t*)take(nn * 4);
    uint32_t* pos = (uint32_t*)take(nn * 4);
    uint32_t* dev = (uint32_t*)take(16);  // [0] merge counter, [1] cluster count
    size_t sb = 0;
    if (!scan_bytes(n, sb)) return hipErrorInvalidValue;
    void* scan_tmp = take(sb);
    const dim3 b256(256);
    hipError_t e = hipMemsetAsync(dev, 0, 16, st);
    if (e == hipSuccess) e = hipMemsetAsync(arrivals, 0, nn * 4, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(ploc_init, dim3((uint32_t)((n2 + 255) / 256)), b256, 0, st, tris, svals, n, box, cnt, parent,
                       clus[0]);
    // (`tris` is still in file order here; `copy` takes it before the emit permutes `tris`)
    uint32_t m = n, cur = 0, force = 0;
    while (m > 1) {
        const dim3 g((m + 255) / 256);
        hipLaunchKernelGGL(ploc_nn, g, b256, 0, st, clus[cur], m, box, nnb);
        hipLaunchKernelGGL(ploc_merge, g, b256, 0, st, clus[cur], m, nnb, n, force, box, cnt, left, right, parent, dev,
                           next, flag);
        e = rocprim::exclusive_scan(scan_tmp, sb, flag, pos, 0u, (size_t)m, rocprim::plus<uint32_t>(), st);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(ploc_compact, g, b256, 0, st, m, next, flag, pos, clus[cur ^ 1], dev + 1);
        uint32_t m_new = 0;
        e = hipMemcpyAsync(&m_new, dev + 1, 4, hipMemcpyDeviceToHost, st);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        if (e != hipSuccess) return e;
        // a round that merged almost nothing (costs that tie everywhere, e.g. copies of one
        // triangle: every cluster picks the same lowest neighbour) -> pair neighbours next round
        force = m_new == m || (m > 64u && (m - m_new) * 64u < m);
        if (m_new > m) return hipErrorUnknown;
        m = m_new;
        cur ^= 1;
    }
    uint32_t root = 0;
    e = hipMemcpyAsync(&root, clus[cur], 4, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) return e;
    if (n > 1) hipLaunchKernelGGL(ploc_orient, dim3((n - 1 + 255) / 256), b256, 0, st, n, box, left, right);
    hipLaunchKernelGGL(ploc_sizes, dim3((n + 255) / 256), b256, 0, st, n, max_prims, left, right, parent, cnt, box,
                       cost, arrivals, osize);
    uint32_t total = 1;
    e = hipMemcpyAsync(&total, osize + root, 4, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipMemcpyAsync(copy, tris, nn * sizeof(rt_cl_triangle), hipMemcpyDeviceToDevice, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(ploc_emit, dim3((uint32_t)((n2 - 1 + 255) / 256)), b256, 0, st, n, max_prims, root, left, right,
                       parent, cnt, osize, box, copy, svals, tris, nodes);
    *n_nodes = total;
    return hipGetLastError();
}

}  // namespace rtb
