/*
 * rt_oracle.c -- CPU ORACLE (test infrastructure only).
 *
 * A plain-C restatement of the reference OpenCL kernel /root/reference/kernel_bvh.cl
 * under the pinned builtin semantics of include/rt_pinned_math.h.  It is the checker
 * the parity tests compare the HIP path against, and the timed CPU baseline of
 * bench.py ("kind": "port").  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it; the product (librt_hip.so) never links or calls it.
 *
 * Every function cites the reference line range it restates.  Reference quirks are
 * preserved on purpose (hard part 3):
 *   - negative-t hits are accepted (no t > 0 test, kernel_bvh.cl:140);
 *   - back faces are always rejected (det < 1e-8, kernel_bvh.cl:116);
 *   - the far child is pushed by sign[axis], not by distance (kernel_bvh.cl:200-207);
 *   - the two gamma exponents differ (0.45454545f at :450, 0.454545f at :407);
 *   - frameSeed is unused (kernel_bvh.cl:424, :445);
 *   - lightPixel has no shadow ray (kernel_bvh.cl:304-347);
 *   - the point-light attenuation divides in double (`1.0 /`, kernel_bvh.cl:335).
 *
 * Build (see oracle/Makefile): gcc -O2 -ffp-contract=off -fno-fast-math -shared -fPIC.
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/rt_pinned_math.h"

/* ---- layout contract: CLshared_structs.hpp:7-87 (float3 = 16-byte slot) ---------- */
typedef struct { float x, y, z, w; } of3;
typedef struct { of3 position, uv, normal, tangent_s, tangent_t; } o_vertex;        /* 80 B */
typedef struct { o_vertex v1, v2, v3; uint32_t mtlIndex; uint32_t padding[3]; } o_tri; /* 256 B */
typedef struct { of3 bmin, bmax; uint32_t offset; uint16_t nPrimitives; uint8_t axis;
                 uint8_t pad[9]; } o_node;                                          /* 48 B */
typedef struct { of3 diffuse, specular, emission; uint32_t type; float roughness, ior;
                 int32_t padding; } o_mat;                                          /* 64 B */

_Static_assert(sizeof(o_vertex) == 80, "CLVertex is 80 bytes");
_Static_assert(sizeof(o_tri) == 256, "CLTriangle is 256 bytes");
_Static_assert(sizeof(o_node) == 48, "CLLinearBVHNode is 48 bytes");
_Static_assert(sizeof(o_mat) == 64, "CLMaterial is 64 bytes");

/* §8(d) counters */
typedef struct { uint64_t rays, node_visits, tri_tests, hits; } o_counts;

/* ---- float3 algebra, pinned (rt_pinned_math.h) ------------------------------------ */
static inline of3 v3(float x, float y, float z) { of3 r = {x, y, z, 0.0f}; return r; }
static inline of3 vs(float s) { return v3(s, s, s); }
static inline of3 vadd(of3 a, of3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline of3 vsub(of3 a, of3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline of3 vmul(of3 a, of3 b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline of3 vdiv(of3 a, of3 b) { return v3(a.x / b.x, a.y / b.y, a.z / b.z); }
static inline of3 vscale(of3 a, float s) { return v3(a.x * s, a.y * s, a.z * s); }
static inline of3 vneg(of3 a) { return v3(-a.x, -a.y, -a.z); }
static inline float vdot(of3 a, of3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
static inline of3 vcross(of3 a, of3 b) {
    return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
static inline of3 vnormalize(of3 v) {
    if (v.x == 0.0f && v.y == 0.0f && v.z == 0.0f) return v;
    float d = vdot(v, v);
    if (d < 0x1p-126f) {
        v = vscale(v, 0x1p86f);
        d = vdot(v, v);
    } else if (pm_isinf(d)) {
        v = vscale(v, 0x1p-66f);
        d = vdot(v, v);
        if (pm_isinf(d)) {
            v = v3(pm_copysign(pm_isinf(v.x) ? 1.0f : 0.0f, v.x),
                   pm_copysign(pm_isinf(v.y) ? 1.0f : 0.0f, v.y),
                   pm_copysign(pm_isinf(v.z) ? 1.0f : 0.0f, v.z));
            d = vdot(v, v);
        }
    }
    return vscale(v, pm_rsqrt(d));
}
static inline of3 vmax_s(of3 a, float s) { return v3(pm_max(a.x, s), pm_max(a.y, s), pm_max(a.z, s)); }
static inline of3 vpow_s(of3 a, float e) { return v3(pm_pow(a.x, e), pm_pow(a.y, e), pm_pow(a.z, e)); }

/* ---- data types: kernel_bvh.cl:10-40 ---------------------------------------------- */
typedef struct { of3 origin, dir, invDir; int sign[3]; } o_ray;
typedef struct {
    int hit;
    o_ray ray;
    float t;
    of3 pos, uv, normal;
    int32_t object; /* index into the triangle array; -1 = none */
} o_isect;
typedef struct {
    const o_tri* tris;
    const o_node* nodes;
    const o_mat* mats;
    uint32_t lightBounces;
    int lightType;
    float skyboxIntensity;
    of3 camPos, camFront, camUp;
} o_scene;

#define O_TWO_PI 6.28318530718f
#define O_INV_PI 0.31830988618f
#define O_MAX_RENDER_DIST 100000.0f

/* kernel_bvh.cl:42-55 */
static o_ray o_init_ray(of3 origin, of3 dir) {
    o_ray r;
    dir = vnormalize(dir);
    r.origin = origin;
    r.dir = dir;
    r.invDir = vdiv(vs(1.0f), dir);
    r.sign[0] = r.invDir.x < 0.0f;
    r.sign[1] = r.invDir.y < 0.0f;
    r.sign[2] = r.invDir.z < 0.0f;
    return r;
}

/* kernel_bvh.cl:57-71 */
static uint32_t o_frame_hash(uint32_t x) { return 1103515245u * x + 12345u; }
static uint32_t o_hash(uint32_t* x) {
    uint32_t v = *x;
    v ^= v >> 16;
    v *= 0x7feb352du;
    v ^= v >> 15;
    v *= 0x846ca68bu;
    v ^= v >> 16;
    *x = v;
    return v;
}
static float o_rand(uint32_t* seed) { return (float)o_hash(seed) / (float)0xffffffffu; }

/* kernel_bvh.cl:74-77 */
static of3 o_reflect(of3 v, of3 n) { return vadd(vneg(v), vscale(n, 2.0f * vdot(v, n))); }

/* orthonormal frame around n, kernel_bvh.cl:85-87 and :234-236 */
static void o_frame(of3 n, of3* s, of3* t) {
    of3 axis = pm_fabs(n.x) > 0.001f ? v3(0.0f, 1.0f, 0.0f) : v3(1.0f, 0.0f, 0.0f);
    *t = vnormalize(vcross(axis, n));
    *s = vcross(n, *t);
}

/* kernel_bvh.cl:79-90 */
static of3 o_sample_hemisphere_cosine(of3 n, uint32_t* seed) {
    float phi = O_TWO_PI * o_rand(seed);
    float s2 = o_rand(seed);
    float sinT = pm_sqrt(s2);
    of3 s, t;
    o_frame(n, &s, &t);
    of3 a = vscale(vscale(s, pm_cos(phi)), sinT);
    of3 b = vscale(vscale(t, pm_sin(phi)), sinT);
    of3 c = vscale(n, pm_sqrt(1.0f - s2));
    return vnormalize(vadd(vadd(a, b), c));
}

/* kernel_bvh.cl:98-153.  The reference loops twice over a rejected triangle
 * (`for i < 2` + `continue`) and recomputes the same values; that has no effect and
 * is done once here. */
static int o_ray_triangle(const o_ray* r, const o_tri* tris, int32_t idx, o_isect* is) {
    const o_tri* tri = &tris[idx];
    const float EPS = 1.0e-8f;
    of3 p1 = tri->v1.position, p2 = tri->v2.position, p3 = tri->v3.position;
    of3 e1 = vsub(p2, p1);
    of3 e2 = vsub(p3, p1);
    of3 pvec = vcross(r->dir, e2);
    float det = vdot(e1, pvec);
    if (det < EPS || -det > EPS) return 0;
    float inv_det = 1.0f / det;
    of3 tvec = vsub(r->origin, p1);
    float u = vdot(tvec, pvec) * inv_det;
    if (u < 0.0f || u > 1.0f) return 0;
    of3 qvec = vcross(tvec, e1);
    float v = vdot(r->dir, qvec) * inv_det;
    if (v < 0.0f || u + v > 1.0f) return 0;
    float t = vdot(e2, qvec) * inv_det;
    if (t < is->t) {
        float w = 1.0f - u - v;
        is->hit = 1;
        is->t = t;
        is->pos = vadd(is->ray.origin, vscale(is->ray.dir, t));
        is->object = idx;
        is->normal = vnormalize(vadd(vadd(vscale(tri->v2.normal, u), vscale(tri->v3.normal, v)),
                                     vscale(tri->v1.normal, w)));
        is->uv = vadd(vadd(vscale(tri->v2.uv, u), vscale(tri->v3.uv, v)), vscale(tri->v1.uv, w));
        return 1;
    }
    return 0;
}

/* kernel_bvh.cl:156-169 */
static int o_ray_bounds(const o_node* nd, const o_ray* r, float t) {
    const of3* b[2] = {&nd->bmin, &nd->bmax};
    float t0 = pm_max(0.0f, (b[r->sign[0]]->x - r->origin.x) * r->invDir.x);
    float t1 = pm_min(t, (b[1 - r->sign[0]]->x - r->origin.x) * r->invDir.x);
    t0 = pm_max(t0, (b[r->sign[1]]->y - r->origin.y) * r->invDir.y);
    t1 = pm_min(t1, (b[1 - r->sign[1]]->y - r->origin.y) * r->invDir.y);
    t0 = pm_max(t0, (b[r->sign[2]]->z - r->origin.z) * r->invDir.z);
    t1 = pm_min(t1, (b[1 - r->sign[2]]->z - r->origin.z) * r->invDir.z);
    return t1 >= t0;
}

/* kernel_bvh.cl:171-219 */
static o_isect o_intersect(const o_ray* ray, const o_scene* sc, o_counts* cnt) {
    o_isect is;
    memset(&is, 0, sizeof(is));
    is.hit = 0;
    is.ray = *ray;
    is.t = O_MAX_RENDER_DIST;
    is.object = -1;
    int stack[64];
    int sp = 0, cur = 0;
    cnt->rays++;
    for (;;) {
        const o_node* nd = &sc->nodes[cur];
        cnt->node_visits++;
        if (o_ray_bounds(nd, ray, is.t)) {
            if (nd->nPrimitives > 0) {
                for (int i = 0; i < (int)nd->nPrimitives; ++i) {
                    cnt->tri_tests++;
                    o_ray_triangle(ray, sc->tris, (int32_t)(nd->offset + (uint32_t)i), &is);
                }
                if (sp == 0) break;
                cur = stack[--sp];
            } else {
                if (sp >= 64) abort(); /* the reference overflows silently here */
                if (ray->sign[nd->axis]) {
                    stack[sp++] = cur + 1;
                    cur = (int)nd->offset;
                } else {
                    stack[sp++] = (int)nd->offset;
                    cur = cur + 1;
                }
            }
        } else {
            if (sp == 0) break;
            cur = stack[--sp];
        }
    }
    if (is.hit) cnt->hits++;
    return is;
}

/* kernel_bvh.cl:221-225 */
static float o_distribution_ggx(float c, float alpha) {
    float a2 = alpha * alpha;
    return a2 * O_INV_PI / pm_sq(c * c * (a2 - 1.0f) + 1.0f); /* pow(., 2.0f) */
}

/* kernel_bvh.cl:227-239 */
static of3 o_sample_ggx(of3 n, float alpha, float* cosTheta, uint32_t* seed) {
    float phi = O_TWO_PI * o_rand(seed);
    (void)o_rand(seed); /* `xi` is drawn and never used (kernel_bvh.cl:230) */
    float r = o_rand(seed);
    *cosTheta = pm_pow(r, 1.0f / (alpha + 1.0f));
    float sinT = pm_sqrt(pm_max(0.0f, 1.0f - (*cosTheta) * (*cosTheta)));
    of3 s, t;
    o_frame(n, &s, &t);
    of3 a = vscale(vscale(s, pm_cos(phi)), sinT);
    of3 b = vscale(vscale(t, pm_sin(phi)), sinT);
    of3 c = vscale(n, *cosTheta);
    return vnormalize(vadd(vadd(a, b), c));
}

/* kernel_bvh.cl:264-269 */
static of3 o_sample_diffuse(of3* wi, float* pdf, of3 n, const o_mat* m, uint32_t* seed) {
    *wi = o_sample_hemisphere_cosine(n, seed);
    *pdf = vdot(*wi, n) * O_INV_PI;
    return vscale(m->diffuse, O_INV_PI);
}

/* kernel_bvh.cl:271-292.  GeometrySmith (:282) and FresnelSchlick (:284) feed nothing
 * (`G` and `F` are never read) and have no side effects, so they are not evaluated. */
static of3 o_sample_specular(of3 wo, of3* wi, float* pdf, of3 n, const o_mat* m, uint32_t* seed) {
    float cosTheta = 1.0f;
    float alpha = 2.0f / pm_sq(m->roughness) - 2.0f; /* pow(roughness, 2.0f) */
    of3 wh = o_sample_ggx(n, alpha, &cosTheta, seed);
    *wi = o_reflect(wo, wh);
    if (vdot(*wi, n) * vdot(wo, n) < 0.000001f) return vs(0.0f);
    float D = o_distribution_ggx(cosTheta, alpha);
    *pdf = D * cosTheta / (4.0f * pm_max(vdot(wo, wh), 0.0f));
    float denom = 4.0f * pm_max(vdot(*wi, n), 0.0f) * pm_max(vdot(wo, n), 0.0f) + 0.001f;
    return vscale(m->specular, D / denom);
}

/* kernel_bvh.cl:294-302 (`* 1.0f` is exact and omitted) */
static of3 o_sample_brdf(of3 wo, of3* wi, float* pdf, of3 n, const o_mat* m, uint32_t* seed) {
    if (o_rand(seed) > 0.5f) return o_sample_specular(wo, wi, pdf, n, m, seed);
    return o_sample_diffuse(wi, pdf, n, m, seed);
}

/* kernel_bvh.cl:304-347 */
static float o_light_pixel(const o_ray* ray, const o_scene* sc, const o_isect* is) {
    const of3 lightPosition = v3(0.0f, -10.0f, 16.0f);
    const of3 lightDirection = v3(-0.5f, 0.4f, -0.1f);
    float intensity = 1.0f, NdotL = 1.0f, attn = 1.0f;
    if (sc->lightType <= 0) {
        NdotL = pm_max(vdot(is->normal, vneg(lightDirection)), 0.0f);
    } else if (sc->lightType == 1) {
        intensity = 16.0f;
        float falloff = 0.8f;
        of3 X = vadd(ray->origin, vscale(ray->dir, is->t));
        of3 L = vsub(lightPosition, X);
        NdotL = pm_max(vdot(is->normal, L), 0.0f);
        of3 eye = vsub(L, X);
        float d = pm_sqrt(vdot(eye, eye));
        attn = (float)(1.0 / (double)(falloff * (d * d)));
    } else {
        of3 X = vadd(ray->origin, vscale(ray->dir, is->t));
        of3 L = vsub(lightPosition, X);
        NdotL = pm_max(vdot(is->normal, L), 0.0f);
    }
    return attn * intensity * NdotL;
}

/* kernel_bvh.cl:349-384 */
static of3 o_render(o_ray* ray, const o_scene* sc, uint32_t* seed, o_counts* cnt,
                    int32_t* prim_id, float* prim_t) {
    of3 radiance = vs(0.0f), beta = vs(1.0f);
    if (prim_id) *prim_id = -1;
    if (prim_t) *prim_t = 0.0f;
    for (int i = 0; (uint32_t)i < sc->lightBounces; ++i) {
        o_isect is = o_intersect(ray, sc, cnt);
        if (i == 0) {
            if (prim_id) *prim_id = is.hit ? is.object : -1;
            if (prim_t) *prim_t = is.t;
        }
        if (!is.hit) {
            radiance = vadd(radiance, vmul(beta, vs(0.5f * sc->skyboxIntensity)));
            break;
        }
        const o_mat* m = &sc->mats[sc->tris[is.object].mtlIndex];
        radiance = vadd(radiance, vscale(vmul(beta, m->emission), 50.0f));
        of3 wi = vs(0.0f);
        of3 wo = vneg(ray->dir);
        float pdf = 0.0f;
        of3 f = o_sample_brdf(wo, &wi, &pdf, is.normal, m, seed);
        if (pdf <= 0.0f || pdf != pdf) break;
        of3 mul = vscale(f, vdot(wi, is.normal));
        mul = v3(mul.x / pdf, mul.y / pdf, mul.z / pdf);
        beta = vmul(beta, mul);
        float lp = o_light_pixel(ray, sc, &is);
        radiance = vadd(radiance, vmul(vmul(vs(lp), m->diffuse), beta));
        *ray = o_init_ray(vadd(is.pos, vscale(wi, 0.01f)), wi);
    }
    return vmax_s(radiance, 0.0f);
}

/* kernel_bvh.cl:386-403 */
static o_ray o_create_ray(uint32_t gid, uint32_t W, uint32_t H, of3 pos, of3 front, of3 up,
                          uint32_t* seed) {
    float invW = 1.0f / (float)W;
    float invH = 1.0f / (float)H;
    float aspect = (float)W / (float)H;
    float angle = pm_tan(0.5f * (45.0f * 3.1415f / 180.0f));
    float x = (float)(gid % W) + o_rand(seed) - 0.5f;
    float y = (float)(gid / W) + o_rand(seed) - 0.5f;
    x = (2.0f * ((x + 0.5f) * invW) - 1.0f) * angle * aspect;
    y = -(1.0f - 2.0f * ((y + 0.5f) * invH)) * angle;
    of3 dir = vnormalize(vadd(vadd(vscale(vcross(front, up), x), vscale(up, y)), front));
    return o_init_ray(pos, dir);
}

/* kernel_bvh.cl:415-456 for one work-item */
static void o_kernel_entry(uint32_t gid, of3* result, const o_scene* sc, uint32_t W, uint32_t H,
                           uint32_t frameCount, o_counts* cnt, int32_t* prim_id, float* prim_t) {
    uint32_t seed = gid + o_frame_hash(frameCount);
    o_ray ray = o_create_ray(gid, W, H, sc->camPos, sc->camFront, sc->camUp, &seed);
    of3 rad = o_render(&ray, sc, &seed, cnt, prim_id, prim_t);
    of3 out;
    if (frameCount == 0) {
        out = vpow_s(rad, 0.45454545f);
    } else {
        of3 lin = vpow_s(result[gid], 2.2f);
        of3 acc = vadd(vscale(lin, (float)(frameCount - 1)), rad);
        acc = v3(acc.x / (float)frameCount, acc.y / (float)frameCount, acc.z / (float)frameCount);
        out = vpow_s(acc, 0.454545f);
    }
    result[gid] = out;
}

/* ==== exported C ABI (ctypes) ====================================================== */

typedef struct {
    const void* tris; const void* nodes; const void* mats;
    uint32_t width, height, frameCount;
    int32_t lightBounces, lightType;
    float skyboxIntensity;
    float cam[12]; /* pos.xyzw front.xyzw up.xyzw */
} oracle_args;

static void o_make_scene(const oracle_args* a, o_scene* sc) {
    sc->tris = (const o_tri*)a->tris;
    sc->nodes = (const o_node*)a->nodes;
    sc->mats = (const o_mat*)a->mats;
    sc->lightBounces = (uint32_t)a->lightBounces;
    sc->lightType = a->lightType;
    sc->skyboxIntensity = a->skyboxIntensity;
    sc->camPos = v3(a->cam[0], a->cam[1], a->cam[2]);
    sc->camFront = v3(a->cam[4], a->cam[5], a->cam[6]);
    sc->camUp = v3(a->cam[8], a->cam[9], a->cam[10]);
}

/* Render work-items [g0, g1) of one frame into `result` (W*H float4 slots).  Optional
 * outputs: primary hit ids / t (indexed by gid), counters (summed). */
int oracle_render_range(const oracle_args* a, float* result, uint32_t g0, uint32_t g1,
                        int32_t* prim_ids, float* prim_t, uint64_t* counts4) {
    o_scene sc;
    o_make_scene(a, &sc);
    o_counts cnt = {0, 0, 0, 0};
    for (uint32_t g = g0; g < g1; ++g) {
        o_kernel_entry(g, (of3*)result, &sc, a->width, a->height, a->frameCount, &cnt,
                       prim_ids ? &prim_ids[g] : NULL, prim_t ? &prim_t[g] : NULL);
    }
    if (counts4) {
        counts4[0] += cnt.rays;
        counts4[1] += cnt.node_visits;
        counts4[2] += cnt.tri_tests;
        counts4[3] += cnt.hits;
    }
    return 0;
}

typedef struct {
    const oracle_args* a; float* result; int32_t* ids; float* t;
    uint32_t g0, g1; uint64_t counts[4];
} o_job;

static void* o_worker(void* p) {
    o_job* j = (o_job*)p;
    oracle_render_range(j->a, j->result, j->g0, j->g1, j->ids, j->t, j->counts);
    return NULL;
}

/* Multi-threaded render of work-items [g0, g1) over `threads` pthreads (interleaved
 * 64-pixel chunks would balance better; contiguous slices keep it simple). */
int oracle_render_mt(const oracle_args* a, float* result, uint32_t g0, uint32_t g1,
                     int32_t* prim_ids, float* prim_t, uint64_t* counts4, int threads) {
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    o_job jobs[256];
    pthread_t th[256];
    uint64_t n = g1 - g0;
    for (int i = 0; i < threads; ++i) {
        jobs[i].a = a; jobs[i].result = result; jobs[i].ids = prim_ids; jobs[i].t = prim_t;
        jobs[i].g0 = g0 + (uint32_t)(n * (uint64_t)i / (uint64_t)threads);
        jobs[i].g1 = g0 + (uint32_t)(n * (uint64_t)(i + 1) / (uint64_t)threads);
        memset(jobs[i].counts, 0, sizeof(jobs[i].counts));
        pthread_create(&th[i], NULL, o_worker, &jobs[i]);
    }
    for (int i = 0; i < threads; ++i) {
        pthread_join(th[i], NULL);
        if (counts4) for (int k = 0; k < 4; ++k) counts4[k] += jobs[i].counts[k];
    }
    return 0;
}

/* Per-pixel work estimate for load-balance modelling (scripts/balance_model.py):
 * node visits + 2 * triangle tests + 15 * rays (the relative cost of a traversal step, a
 * triangle step and a shading round per lane on the GPU kernel). */
typedef struct { const oracle_args* a; float* result; uint32_t* cost; uint32_t g0, g1; } o_cost_job;

static void* o_cost_worker(void* p) {
    o_cost_job* j = (o_cost_job*)p;
    o_scene sc;
    o_make_scene(j->a, &sc);
    for (uint32_t g = j->g0; g < j->g1; ++g) {
        o_counts c = {0, 0, 0, 0};
        o_kernel_entry(g, (of3*)j->result, &sc, j->a->width, j->a->height, j->a->frameCount, &c, NULL, NULL);
        j->cost[g] = (uint32_t)(c.node_visits + 2 * c.tri_tests + 15 * c.rays);
    }
    return NULL;
}

int oracle_pixel_cost_mt(const oracle_args* a, float* result, uint32_t* cost, int threads) {
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    o_cost_job jobs[256];
    pthread_t th[256];
    const uint64_t n = (uint64_t)a->width * a->height;
    for (int i = 0; i < threads; ++i) {
        jobs[i].a = a; jobs[i].result = result; jobs[i].cost = cost;
        jobs[i].g0 = (uint32_t)(n * (uint64_t)i / (uint64_t)threads);
        jobs[i].g1 = (uint32_t)(n * (uint64_t)(i + 1) / (uint64_t)threads);
        pthread_create(&th[i], NULL, o_cost_worker, &jobs[i]);
    }
    for (int i = 0; i < threads; ++i) pthread_join(th[i], NULL);
    return 0;
}

/* Known-answer hooks for the unit tests. */
uint32_t oracle_hash(uint32_t x) { return o_hash(&x); }
uint32_t oracle_frame_hash(uint32_t x) { return o_frame_hash(x); }
float oracle_rand(uint32_t* seed) { return o_rand(seed); }
float oracle_pow(float x, float y) { return pm_pow(x, y); }
float oracle_sin(float x) { return pm_sin(x); }
float oracle_cos(float x) { return pm_cos(x); }
float oracle_tan(float x) { return pm_tan(x); }
/* number of inputs where pm_sincos differs (bitwise) from pm_sin / pm_cos */
long oracle_sincos_mismatches(const float* xs, long n) {
    long bad = 0;
    for (long i = 0; i < n; ++i) {
        float s, c;
        pm_sincos(xs[i], &s, &c);
        const float s1 = pm_sin(xs[i]), c1 = pm_cos(xs[i]);
        if (pm_f2u(s) != pm_f2u(s1) || pm_f2u(c) != pm_f2u(c1)) ++bad;
    }
    return bad;
}
float oracle_max(float x, float y) { return pm_max(x, y); }
float oracle_min(float x, float y) { return pm_min(x, y); }

/* Single ray/triangle and ray/box probes for hand-built cases. */
int oracle_ray_triangle(const float* org, const float* dir, const void* tri, float t_in,
                        float* t_out) {
    o_ray r = o_init_ray(v3(org[0], org[1], org[2]), v3(dir[0], dir[1], dir[2]));
    o_isect is;
    memset(&is, 0, sizeof(is));
    is.ray = r;
    is.t = t_in;
    is.object = -1;
    int hit = o_ray_triangle(&r, (const o_tri*)tri, 0, &is);
    *t_out = is.t;
    return hit;
}
int oracle_ray_bounds(const float* org, const float* dir, const void* node, float t) {
    o_ray r = o_init_ray(v3(org[0], org[1], org[2]), v3(dir[0], dir[1], dir[2]));
    return o_ray_bounds((const o_node*)node, &r, t);
}
