// scene.cpp -- host scene pipeline: OBJ/MTL loader + SAH BVH builder + DFS flatten.
//
// Restates the reference host code that produces the device arrays (it cannot be
// compiled here: it needs Win32/GL/glm headers and has case-mismatched includes,
// SURVEY.md section 2).  Semantics follow the reference exactly, including:
//   * every n-gon face emits n-2 "strip" triangles plus one closing triangle
//     (n-2, n-1, 0), so a triangle face becomes two triangles with rotated vertices
//     (CLOBJloader.cpp:101-126);
//   * face tokens of length <= 1 are skipped, tokens parse as "%d/%d/%d"
//     (CLOBJloader.cpp:87-99);
//   * material index starts at (unsigned)-1 and an unknown usemtl keeps the previous
//     index (CLOBJloader.cpp:37, :65-77);
//   * CLMaterial defaults diffuse 0.2, specular 1, roughness 9999, ior 0
//     (CLshared_structs.hpp:16); Ns -> roughness, Ni -> ior (CLOBJloader.cpp:167-174);
//   * pbrt-style recursive build: leaf for one primitive or degenerate centroid bounds,
//     median nth_element for two, otherwise 12-bucket SAH with leaf cost n, split
//     forced above max primitives (CLBVHnode.cpp:7-159); std::nth_element and
//     std::partition are the libstdc++ ones, as in the reference's MinGW g++ build
//     (Makefile:13), so the primitive order is the same;
//   * depth-first flatten, first child = index + 1, second child in `offset`
//     (CLBVHnode.cpp:161-183).
// Arithmetic is plain fp32 with no contraction (built with -ffp-contract=off), in the
// order of the reference's float3/CLBounds3 operators (CLmathlib.hpp:18-204).
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <limits>
#include <memory>
#include <new>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/rt_cl_types.h"
#include "../../include/rt_scene.h"
#include "../../include/rt_status.h"

namespace {

// ---- host vector / bounds algebra (CLmathlib.hpp) ---------------------------------
struct V3 {
    float x = 0.0f, y = 0.0f, z = 0.0f;
    V3() = default;
    V3(float a, float b, float c) : x(a), y(b), z(c) {}
    explicit V3(float s) : x(s), y(s), z(s) {}
    float operator[](int i) const { return i == 0 ? x : (i == 1 ? y : z); }
};
inline V3 operator+(const V3& a, const V3& b) { return V3(a.x + b.x, a.y + b.y, a.z + b.z); }
inline V3 operator-(const V3& a, const V3& b) { return V3(a.x - b.x, a.y - b.y, a.z - b.z); }
inline V3 operator*(const V3& a, float s) { return V3(a.x * s, a.y * s, a.z * s); }
inline V3 vmin(const V3& a, const V3& b) {
    return V3(std::min(a.x, b.x), std::min(a.y, b.y), std::min(a.z, b.z));
}
inline V3 vmax(const V3& a, const V3& b) {
    return V3(std::max(a.x, b.x), std::max(a.y, b.y), std::max(a.z, b.z));
}

struct Box {
    // empty box: min = +FLT_MAX, max = lowest (CLmathlib.hpp:122-128)
    V3 lo{std::numeric_limits<float>::max(), std::numeric_limits<float>::max(),
          std::numeric_limits<float>::max()};
    V3 hi{std::numeric_limits<float>::lowest(), std::numeric_limits<float>::lowest(),
          std::numeric_limits<float>::lowest()};
    Box() = default;
    Box(const V3& a, const V3& b) : lo(vmin(a, b)), hi(vmax(a, b)) {}
    V3 diag() const { return hi - lo; }
    float area() const {
        V3 d = diag();
        return 2 * (d.x * d.y + d.x * d.z + d.y * d.z);
    }
    unsigned widest_axis() const {
        V3 d = diag();
        if (d.x > d.y && d.x > d.z) return 0;
        return d.y > d.z ? 1u : 2u;
    }
    // relative position of p inside the box per axis (CLmathlib.hpp:173-179)
    V3 rel(const V3& p) const {
        V3 o = p - lo;
        if (hi.x > lo.x) o.x /= hi.x - lo.x;
        if (hi.y > lo.y) o.y /= hi.y - lo.y;
        if (hi.z > lo.z) o.z /= hi.z - lo.z;
        return o;
    }
};
inline Box merge(const Box& b, const V3& p) {
    Box r;
    r.lo = vmin(b.lo, p);
    r.hi = vmax(b.hi, p);
    return r;
}
inline Box merge(const Box& a, const Box& b) {
    Box r;
    r.lo = vmin(a.lo, b.lo);
    r.hi = vmax(a.hi, b.hi);
    return r;
}

inline V3 pos_of(const rt_float3& f) { return V3(f.x, f.y, f.z); }
inline rt_float3 to_f3(const V3& v) { return rt_float3{v.x, v.y, v.z, 0.0f}; }

// ---- BVH build (CLBVHnode.cpp) --------------------------------------------------------
struct BuildNode {
    Box box;
    BuildNode* kid[2] = {nullptr, nullptr};
    int axis = 0, first = 0, count = 0;
};

struct PrimRef {
    unsigned prim = 0;
    Box box;
    V3 centroid;
    PrimRef() = default;
    PrimRef(unsigned p, const Box& b) : prim(p), box(b), centroid(b.lo * 0.5f + b.hi * 0.5f) {}
};

constexpr unsigned kBuckets = 12;

struct Builder {
    const std::vector<rt_cl_triangle>& src;
    unsigned max_prims;
    std::vector<std::unique_ptr<BuildNode>> pool;
    std::vector<rt_cl_triangle> ordered;
    unsigned total = 0;

    BuildNode* make_leaf(BuildNode* n, std::vector<PrimRef>& refs, unsigned s, unsigned e,
                         const Box& box) {
        n->first = (int)ordered.size();
        for (unsigned i = s; i < e; ++i) ordered.push_back(src[refs[i].prim]);
        n->count = (int)(e - s);
        n->box = box;
        return n;
    }

    static int bucket_of(const Box& cb, const V3& c, unsigned axis) {
        const float x = kBuckets * cb.rel(c)[(int)axis];
        // finite centroids give x in [0, kBuckets]; a NaN / infinite coordinate (which the
        // reference would turn into an out-of-range index, undefined behaviour) goes to the
        // nearest end bucket
        if (!(x >= 0.0f)) return 0;
        if (x >= (float)kBuckets) return kBuckets - 1;
        return (int)x;
    }

    BuildNode* build(std::vector<PrimRef>& refs, unsigned s, unsigned e) {
        pool.emplace_back(new BuildNode());
        BuildNode* n = pool.back().get();
        ++total;
        Box box;
        for (unsigned i = s; i < e; ++i) box = merge(box, refs[i].box);
        const unsigned count = e - s;
        if (count == 1) return make_leaf(n, refs, s, e, box);

        Box cbox;
        for (unsigned i = s; i < e; ++i) cbox = merge(cbox, refs[i].centroid);
        const unsigned axis = cbox.widest_axis();
        unsigned mid = (s + e) / 2;
        if (cbox.hi[(int)axis] == cbox.lo[(int)axis]) return make_leaf(n, refs, s, e, box);

        if (count <= 2) {
            std::nth_element(&refs[s], &refs[mid], &refs[e - 1] + 1,
                             [axis](const PrimRef& a, const PrimRef& b) {
                                 return a.centroid[(int)axis] < b.centroid[(int)axis];
                             });
        } else {
            int cnt[kBuckets] = {0};
            Box bb[kBuckets];
            for (unsigned i = s; i < e; ++i) {
                int b = bucket_of(cbox, refs[i].centroid, axis);
                cnt[b]++;
                bb[b] = merge(bb[b], refs[i].box);
            }
            float cost[kBuckets - 1];
            for (unsigned i = 0; i < kBuckets - 1; ++i) {
                Box left, right;
                int nl = 0, nr = 0;
                for (unsigned j = 0; j <= i; ++j) { left = merge(left, bb[j]); nl += cnt[j]; }
                for (unsigned j = i + 1; j < kBuckets; ++j) { right = merge(right, bb[j]); nr += cnt[j]; }
                cost[i] = 1.0f + (nl * left.area() + nr * right.area()) / box.area();
            }
            float best = cost[0];
            unsigned split = 0;
            for (unsigned i = 1; i < kBuckets - 1; ++i) {
                if (cost[i] < best) { best = cost[i]; split = i; }
            }
            const float leaf_cost = float(count);
            if (count > max_prims || best < leaf_cost) {
                PrimRef* m = std::partition(&refs[s], &refs[e - 1] + 1,
                                            [=](const PrimRef& r) {
                                                int b = bucket_of(cbox, r.centroid, axis);
                                                return (unsigned)b <= split;
                                            });
                mid = (unsigned)(m - &refs[0]);
                if (mid == s || mid == e) {
                    // an empty side: impossible for finite centroids (the lowest centroid is
                    // always in bucket 0), reachable with NaN coordinates -- the reference would
                    // recurse forever; split at the median instead, NaN ordered last
                    mid = (s + e) / 2;
                    auto key = [axis](const PrimRef& r) {
                        const float c = r.centroid[(int)axis];
                        return c != c ? std::numeric_limits<float>::infinity() : c;
                    };
                    std::nth_element(&refs[s], &refs[mid], &refs[e - 1] + 1,
                                     [&key](const PrimRef& a, const PrimRef& b) { return key(a) < key(b); });
                }
            } else {
                return make_leaf(n, refs, s, e, box);
            }
        }
        BuildNode* a = build(refs, s, mid);
        BuildNode* b = build(refs, mid, e);
        n->kid[0] = a;
        n->kid[1] = b;
        n->box = merge(a->box, b->box);
        n->axis = (int)axis;
        n->count = 0;
        return n;
    }
};

unsigned flatten(const BuildNode* n, std::vector<rt_cl_bvh_node>& out, unsigned* next) {
    rt_cl_bvh_node& ln = out[*next];
    std::memset(&ln, 0, sizeof(ln));
    ln.bounds.pmin = to_f3(n->box.lo);
    ln.bounds.pmax = to_f3(n->box.hi);
    const unsigned me = (*next)++;
    if (n->count > 0) {
        out[me].offset = (uint32_t)n->first;
        out[me].nPrimitives = (uint16_t)n->count;
    } else {
        out[me].axis = (uint8_t)n->axis;
        out[me].nPrimitives = 0;
        flatten(n->kid[0], out, next);
        const unsigned second = flatten(n->kid[1], out, next);
        out[me].offset = second;
    }
    return me;
}

}  // namespace

struct rt_scene {
    std::vector<rt_cl_triangle> tris;
    std::vector<rt_cl_material> mats;
    std::vector<std::string> mat_names;
    std::vector<rt_cl_bvh_node> nodes;
    unsigned max_prims = 0;
};

namespace {

rt_cl_material default_material() {
    rt_cl_material m;
    std::memset(&m, 0, sizeof(m));
    m.diffuse = rt_float3{0.2f, 0.2f, 0.2f, 0.0f};
    m.specular = rt_float3{1.0f, 1.0f, 1.0f, 0.0f};
    m.emission = rt_float3{0.0f, 0.0f, 0.0f, 0.0f};
    m.roughness = 9999.0f;
    m.ior = 0.0f;
    return m;
}

// CLOBJloader::LoadMaterials (CLOBJloader.cpp:131-176)
int load_mtl(const char* path, rt_scene* s) {
    FILE* f = std::fopen(path, "r");
    if (!f) return RT_FILE_NOT_FOUND;
    char tok[128];
    while (std::fscanf(f, "%127s", tok) != EOF) {
        if (std::strcmp(tok, "newmtl") == 0) {
            char name[80] = {0};
            if (std::fscanf(f, "%79s\n", name) != 1) break;
            s->mat_names.emplace_back(name);
            s->mats.push_back(default_material());
            continue;
        }
        if (s->mats.empty()) continue;  // the reference would write through back() of an empty vector
        rt_cl_material& m = s->mats.back();
        if (std::strcmp(tok, "Kd") == 0) {
            if (std::fscanf(f, "%f %f %f\n", &m.diffuse.x, &m.diffuse.y, &m.diffuse.z) < 0) break;
        } else if (std::strcmp(tok, "Ks") == 0) {
            if (std::fscanf(f, "%f %f %f\n", &m.specular.x, &m.specular.y, &m.specular.z) < 0) break;
        } else if (std::strcmp(tok, "Ke") == 0) {
            if (std::fscanf(f, "%f %f %f\n", &m.emission.x, &m.emission.y, &m.emission.z) < 0) break;
        } else if (std::strcmp(tok, "Ns") == 0) {
            if (std::fscanf(f, "%f\n", &m.roughness) < 0) break;
        } else if (std::strcmp(tok, "Ni") == 0) {
            if (std::fscanf(f, "%f\n", &m.ior) < 0) break;
        }
    }
    std::fclose(f);
    return RT_SUCCESS;
}

rt_cl_vertex make_vertex(const V3& p, float u, float v, const V3& n) {
    rt_cl_vertex vx;
    std::memset(&vx, 0, sizeof(vx));
    vx.position = to_f3(p);
    vx.uv = rt_float3{u, v, 0.0f, 0.0f};
    vx.normal = to_f3(n);
    return vx;
}

// CLOBJloader::LoadTriangles (CLOBJloader.cpp:16-129)
int load_obj(const char* path, rt_scene* s) {
    const size_t len = std::strlen(path);
    if (len < 4) return RT_INVALID_VALUE;  // (the reference copies into char[80]; no such limit here)
    std::string mtl(path, len - 4);
    mtl += ".mtl";
    int rc = load_mtl(mtl.c_str(), s);
    if (rc != RT_SUCCESS) return rc;

    FILE* f = std::fopen(path, "r");
    if (!f) return RT_FILE_NOT_FOUND;
    std::vector<V3> pos, nrm;
    std::vector<std::pair<float, float>> tex;
    unsigned material = (unsigned)-1;
    char tok[128];
    rc = RT_SUCCESS;
    while (std::fscanf(f, "%127s", tok) != EOF) {
        if (std::strcmp(tok, "v") == 0) {
            V3 p;
            if (std::fscanf(f, "%f %f %f\n", &p.x, &p.y, &p.z) < 0) break;
            pos.push_back(p);
        } else if (std::strcmp(tok, "vt") == 0) {
            float u = 0.0f, v = 0.0f;
            if (std::fscanf(f, "%f %f\n", &u, &v) < 0) break;
            tex.emplace_back(u, v);
        } else if (std::strcmp(tok, "vn") == 0) {
            V3 n;
            if (std::fscanf(f, "%f %f %f\n", &n.x, &n.y, &n.z) < 0) break;
            nrm.push_back(n);
        } else if (std::strcmp(tok, "usemtl") == 0) {
            char name[80] = {0};
            if (std::fscanf(f, "%79s\n", name) != 1) break;
            for (unsigned i = 0; i < s->mat_names.size(); ++i) {
                if (s->mat_names[i] == name) { material = i; break; }
            }
        } else if (std::strcmp(tok, "f") == 0) {
            char line[128];
            if (!std::fgets(line, sizeof(line), f)) break;
            std::vector<unsigned> iv, it, in;
            for (char* t = std::strtok(line, " "); t; t = std::strtok(nullptr, " ")) {
                if (std::strlen(t) <= 1) continue;
                int a = 0, b = 0, c = 0;
                std::sscanf(t, "%d/%d/%d", &a, &b, &c);
                iv.push_back((unsigned)a);
                it.push_back((unsigned)b);
                in.push_back((unsigned)c);
            }
            const size_t k = iv.size();
            if (k < 3) { rc = RT_PARSE_ERROR; break; }  // the reference indexes out of range here
            auto vert = [&](size_t j) -> rt_cl_vertex {
                const size_t pi = iv[j] - 1, ti = it[j] - 1, ni = in[j] - 1;
                if (pi >= pos.size() || ti >= tex.size() || ni >= nrm.size()) {
                    throw std::out_of_range("face index");
                }
                return make_vertex(pos[pi], tex[ti].first, tex[ti].second, nrm[ni]);
            };
            try {
                auto emit = [&](size_t a, size_t b, size_t c) {
                    rt_cl_triangle tri;
                    std::memset(&tri, 0, sizeof(tri));
                    tri.v1 = vert(a);
                    tri.v2 = vert(b);
                    tri.v3 = vert(c);
                    tri.mtlIndex = material;
                    s->tris.push_back(tri);
                };
                for (size_t i = 0; i + 2 < k; ++i) emit(i, i + 1, i + 2);
                emit(k - 2, k - 1, 0);
            } catch (const std::out_of_range&) {
                rc = RT_PARSE_ERROR;
                break;
            }
        }
    }
    std::fclose(f);
    return rc;
}

// CLBVHScene::CreateBVHTrees (CLBVHnode.cpp:185-207)
int create_bvh(rt_scene* s, unsigned max_prims) {
    s->max_prims = max_prims;
    if (s->tris.empty()) return RT_INVALID_VALUE;
    std::vector<PrimRef> refs(s->tris.size());
    for (unsigned i = 0; i < s->tris.size(); ++i) {
        const rt_cl_triangle& t = s->tris[i];
        Box b = merge(Box(pos_of(t.v1.position), pos_of(t.v2.position)), pos_of(t.v3.position));
        refs[i] = PrimRef(i, b);
    }
    Builder bld{s->tris, max_prims, {}, {}, 0};
    BuildNode* root = bld.build(refs, 0, (unsigned)s->tris.size());
    s->tris.swap(bld.ordered);
    s->nodes.assign(bld.total, rt_cl_bvh_node());
    unsigned next = 0;
    flatten(root, s->nodes, &next);
    return next == bld.total ? RT_SUCCESS : RT_INVALID_OPERATION;
}

}  // namespace

extern "C" {

int rtsLoadOBJUnbuilt(const char* obj_path, rt_scene** out) {
    if (!obj_path || !out) return RT_INVALID_VALUE;
    *out = nullptr;
    std::unique_ptr<rt_scene> s(new (std::nothrow) rt_scene());
    if (!s) return RT_OUT_OF_HOST_MEMORY;
    int rc = load_obj(obj_path, s.get());
    if (rc != RT_SUCCESS) return rc;
    *out = s.release();
    return RT_SUCCESS;
}

int rtsLoadOBJ(const char* obj_path, unsigned max_prims_in_node, rt_scene** out) {
    rt_scene* s = nullptr;
    int rc = rtsLoadOBJUnbuilt(obj_path, &s);
    if (rc != RT_SUCCESS) return rc;
    rc = create_bvh(s, max_prims_in_node);
    if (rc != RT_SUCCESS) { delete s; return rc; }
    *out = s;
    return RT_SUCCESS;
}

int rtsBuildFromTriangles(const rt_cl_triangle* tris, size_t n_tris, const rt_cl_material* mats,
                          size_t n_mats, unsigned max_prims_in_node, rt_scene** out) {
    if (!out || (!tris && n_tris) || (!mats && n_mats)) return RT_INVALID_VALUE;
    *out = nullptr;
    std::unique_ptr<rt_scene> s(new (std::nothrow) rt_scene());
    if (!s) return RT_OUT_OF_HOST_MEMORY;
    s->tris.assign(tris, tris + n_tris);
    s->mats.assign(mats, mats + n_mats);
    int rc = create_bvh(s.get(), max_prims_in_node);
    if (rc != RT_SUCCESS) return rc;
    *out = s.release();
    return RT_SUCCESS;
}

int rtsGetTriangles(const rt_scene* s, const rt_cl_triangle** tris, size_t* count) {
    if (!s || !tris || !count) return RT_INVALID_VALUE;
    *tris = s->tris.data();
    *count = s->tris.size();
    return RT_SUCCESS;
}

int rtsGetNodes(const rt_scene* s, const rt_cl_bvh_node** nodes, size_t* count) {
    if (!s || !nodes || !count) return RT_INVALID_VALUE;
    *nodes = s->nodes.data();
    *count = s->nodes.size();
    return RT_SUCCESS;
}

int rtsGetMaterials(const rt_scene* s, const rt_cl_material** mats, size_t* count) {
    if (!s || !mats || !count) return RT_INVALID_VALUE;
    *mats = s->mats.data();
    *count = s->mats.size();
    return RT_SUCCESS;
}

int rtsGetTreeStats(const rt_scene* s, unsigned* max_depth, unsigned* n_leaves,
                    unsigned* max_leaf_prims) {
    if (!s || s->nodes.empty()) return RT_INVALID_VALUE;
    unsigned md = 0, nl = 0, mp = 0;
    // iterative DFS over the flattened layout
    std::vector<std::pair<unsigned, unsigned>> st{{0u, 0u}};
    while (!st.empty()) {
        auto [i, d] = st.back();
        st.pop_back();
        if (i >= s->nodes.size()) return RT_INVALID_VALUE;
        const rt_cl_bvh_node& n = s->nodes[i];
        if (n.nPrimitives > 0) {
            ++nl;
            md = std::max(md, d);
            mp = std::max(mp, (unsigned)n.nPrimitives);
        } else {
            st.push_back({i + 1, d + 1});
            st.push_back({n.offset, d + 1});
        }
    }
    if (max_depth) *max_depth = md;
    if (n_leaves) *n_leaves = nl;
    if (max_leaf_prims) *max_leaf_prims = mp;
    return RT_SUCCESS;
}

namespace {

constexpr char kSceneMagic[8] = {'R', 'T', 'S', 'C', 'E', 'N', 'E', '1'};
constexpr uint32_t kSceneVersion = 1;

uint64_t fnv1a(const void* p, size_t n, uint64_t h) {
    const unsigned char* b = static_cast<const unsigned char*>(p);
    for (size_t i = 0; i < n; ++i) {
        h ^= b[i];
        h *= 1099511628211ull;
    }
    return h;
}

int check_arrays(const std::vector<rt_cl_bvh_node>& nodes, size_t n_tris) {
    for (size_t i = 0; i < nodes.size(); ++i) {
        const rt_cl_bvh_node& x = nodes[i];
        if (x.nPrimitives > 0) {
            if ((uint64_t)x.offset + x.nPrimitives > n_tris) return RT_INVALID_VALUE;
        } else if (x.offset <= i + 1 || x.offset >= nodes.size() || i + 1 >= nodes.size()) {
            return RT_INVALID_VALUE;
        }
    }
    return RT_SUCCESS;
}

}  // namespace

int rtsFromArrays(const rt_cl_triangle* tris, size_t n_tris, const rt_cl_bvh_node* nodes, size_t n_nodes,
                  const rt_cl_material* mats, size_t n_mats, unsigned max_prims_in_node, rt_scene** out) {
    if (!out || (!tris && n_tris) || (!nodes && n_nodes) || (!mats && n_mats)) return RT_INVALID_VALUE;
    *out = nullptr;
    std::unique_ptr<rt_scene> s(new (std::nothrow) rt_scene());
    if (!s) return RT_OUT_OF_HOST_MEMORY;
    s->tris.assign(tris, tris + n_tris);
    s->nodes.assign(nodes, nodes + n_nodes);
    s->mats.assign(mats, mats + n_mats);
    s->max_prims = max_prims_in_node;
    int rc = check_arrays(s->nodes, s->tris.size());
    if (rc) return rc;
    *out = s.release();
    return RT_SUCCESS;
}

int rtsSaveScene(const rt_scene* s, const char* path) {
    if (!s || !path) return RT_INVALID_VALUE;
    uint32_t hdr32[2] = {kSceneVersion, s->max_prims};
    uint64_t hdr64[3] = {s->tris.size(), s->nodes.size(), s->mats.size()};
    uint64_t h = 14695981039346656037ull;
    h = fnv1a(kSceneMagic, 8, h);
    h = fnv1a(hdr32, sizeof(hdr32), h);
    h = fnv1a(hdr64, sizeof(hdr64), h);
    h = fnv1a(s->tris.data(), s->tris.size() * sizeof(rt_cl_triangle), h);
    h = fnv1a(s->nodes.data(), s->nodes.size() * sizeof(rt_cl_bvh_node), h);
    h = fnv1a(s->mats.data(), s->mats.size() * sizeof(rt_cl_material), h);
    FILE* f = std::fopen(path, "wb");
    if (!f) return RT_INVALID_VALUE;
    bool ok = std::fwrite(kSceneMagic, 1, 8, f) == 8 && std::fwrite(hdr32, sizeof(hdr32), 1, f) == 1 &&
              std::fwrite(hdr64, sizeof(hdr64), 1, f) == 1;
    // (an empty array has no data pointer to hand to fwrite: nothing to write)
    auto put = [f](const void* p, size_t size, size_t n) { return n == 0 || std::fwrite(p, size, n, f) == n; };
    ok = ok && put(s->tris.data(), sizeof(rt_cl_triangle), s->tris.size());
    ok = ok && put(s->nodes.data(), sizeof(rt_cl_bvh_node), s->nodes.size());
    ok = ok && put(s->mats.data(), sizeof(rt_cl_material), s->mats.size());
    ok = ok && std::fwrite(&h, sizeof(h), 1, f) == 1;
    ok = (std::fclose(f) == 0) && ok;
    return ok ? RT_SUCCESS : RT_OUT_OF_RESOURCES;
}

int rtsLoadScene(const char* path, rt_scene** out) {
    if (!path || !out) return RT_INVALID_VALUE;
    *out = nullptr;
    FILE* f = std::fopen(path, "rb");
    if (!f) return RT_FILE_NOT_FOUND;
    std::unique_ptr<FILE, int (*)(FILE*)> guard(f, std::fclose);
    char magic[8];
    uint32_t hdr32[2];
    uint64_t hdr64[3];
    if (std::fread(magic, 1, 8, f) != 8 || std::memcmp(magic, kSceneMagic, 8) != 0) return RT_PARSE_ERROR;
    if (std::fread(hdr32, sizeof(hdr32), 1, f) != 1 || hdr32[0] != kSceneVersion) return RT_PARSE_ERROR;
    if (std::fread(hdr64, sizeof(hdr64), 1, f) != 1) return RT_PARSE_ERROR;
    // sizes must match the file before anything is allocated
    if (std::fseek(f, 0, SEEK_END) != 0) return RT_PARSE_ERROR;
    const long fsize = std::ftell(f);
    const uint64_t body = hdr64[0] * sizeof(rt_cl_triangle) + hdr64[1] * sizeof(rt_cl_bvh_node) +
                          hdr64[2] * sizeof(rt_cl_material);
    if (hdr64[0] > (1ull << 32) || hdr64[1] > (1ull << 32) || hdr64[2] > (1ull << 32) || fsize < 0 ||
        (uint64_t)fsize != 8 + sizeof(hdr32) + sizeof(hdr64) + body + 8)
        return RT_PARSE_ERROR;
    if (std::fseek(f, 8 + sizeof(hdr32) + sizeof(hdr64), SEEK_SET) != 0) return RT_PARSE_ERROR;
    std::unique_ptr<rt_scene> s(new (std::nothrow) rt_scene());
    if (!s) return RT_OUT_OF_HOST_MEMORY;
    s->tris.resize(hdr64[0]);
    s->nodes.resize(hdr64[1]);
    s->mats.resize(hdr64[2]);
    s->max_prims = hdr32[1];
    uint64_t stored = 0;
    auto get = [f](void* p, size_t size, size_t n) { return n == 0 || std::fread(p, size, n, f) == n; };
    bool ok = get(s->tris.data(), sizeof(rt_cl_triangle), s->tris.size());
    ok = ok && get(s->nodes.data(), sizeof(rt_cl_bvh_node), s->nodes.size());
    ok = ok && get(s->mats.data(), sizeof(rt_cl_material), s->mats.size());
    ok = ok && std::fread(&stored, sizeof(stored), 1, f) == 1;
    if (!ok) return RT_PARSE_ERROR;
    uint64_t h = 14695981039346656037ull;
    h = fnv1a(kSceneMagic, 8, h);
    h = fnv1a(hdr32, sizeof(hdr32), h);
    h = fnv1a(hdr64, sizeof(hdr64), h);
    h = fnv1a(s->tris.data(), s->tris.size() * sizeof(rt_cl_triangle), h);
    h = fnv1a(s->nodes.data(), s->nodes.size() * sizeof(rt_cl_bvh_node), h);
    h = fnv1a(s->mats.data(), s->mats.size() * sizeof(rt_cl_material), h);
    if (h != stored) return RT_PARSE_ERROR;
    if (check_arrays(s->nodes, s->tris.size())) return RT_PARSE_ERROR;
    *out = s.release();
    return RT_SUCCESS;
}

void rtsRelease(rt_scene* s) { delete s; }

}  // extern "C"
