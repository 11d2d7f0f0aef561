/*
 * ref_cpu_host.c -- host side of the reference kernel compiled for the CPU (test
 * infrastructure and bench.py's cpu_baseline; never part of the product).
 *
 * `make -C oracle refcpu` compiles the UNMODIFIED /root/reference/kernel_bvh.cl in place
 * for x86-64 (clang -x cl); its object leaves the 14 OpenCL builtins it
 * uses undefined.  This file supplies them under their OpenCL (Itanium-mangled) names with
 * the pinned semantics of include/rt_pinned_math.h -- the same definitions the C oracle
 * (rt_oracle.c) and the HIP "pinned" math policy use -- and drives KernelEntry
 * (kernel_bvh.cl:415-456) over a work-item range on N pthreads, one call per work-item,
 * as a CPU OpenCL device would.  So the reference's own kernel source runs here on the
 * host cores: the CPU baseline of kind "reference", and a second pin of the oracle (the
 * oracle restates this very source under these very builtins, tests/test_ref_cpu.py).
 *
 * Builtin semantics (rt_pinned_math.h): dot left to right, cross the textbook formula,
 * normalize = v * (1/sqrt(dot(v,v))) with libclc-style scaling guards, max/min IEEE
 * maxNum/minNum, sin/cos/tan/pow evaluated in fp64 and rounded once, and pow(x, 2.0f)
 * = x*x (the reference only ever passes a literal 2.0f there, kernel_bvh.cl:224, :273).
 */
#include <pthread.h>
#include <stddef.h>
#include <stdint.h>

#include "../include/rt_pinned_math.h"

typedef float f3 __attribute__((ext_vector_type(3)));

/* ---- OpenCL builtins used by kernel_bvh.cl ------------------------------------------ */
static _Thread_local size_t tl_gid;

size_t _Z13get_global_idj(unsigned int dim) { (void)dim; return tl_gid; }
float _Z3cosf(float x) { return pm_cos(x); }
float _Z3sinf(float x) { return pm_sin(x); }
float _Z3tanf(float x) { return pm_tan(x); }
float _Z4fabsf(float x) { return pm_fabs(x); }
float _Z4sqrtf(float x) { return pm_sqrt(x); }
float _Z3maxff(float x, float y) { return pm_max(x, y); }
float _Z3minff(float x, float y) { return pm_min(x, y); }
static float pow1(float x, float y) { return y == 2.0f ? x * x : pm_pow(x, y); }
float _Z3powff(float x, float y) { return pow1(x, y); }

f3 _Z3powDv3_fS_(f3 x, f3 y) {
    f3 r = {pow1(x.x, y.x), pow1(x.y, y.y), pow1(x.z, y.z)};
    return r;
}

f3 _Z3maxDv3_ff(f3 x, float y) {
    f3 r = {pm_max(x.x, y), pm_max(x.y, y), pm_max(x.z, y)};
    return r;
}

static float dot3(f3 a, f3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
float _Z3dotDv3_fS_(f3 a, f3 b) { return dot3(a, b); }

f3 _Z5crossDv3_fS_(f3 a, f3 b) {
    f3 r = {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
    return r;
}

f3 _Z9normalizeDv3_f(f3 v) {
    if (v.x == 0.0f && v.y == 0.0f && v.z == 0.0f) return v;
    float d = dot3(v, v);
    if (d < 0x1p-126f) {
        v = v * 0x1p86f;
        d = dot3(v, v);
    } else if (pm_isinf(d)) {
        v = v * 0x1p-66f;
        d = dot3(v, v);
        if (pm_isinf(d)) {
            f3 u = {pm_copysign(pm_isinf(v.x) ? 1.0f : 0.0f, v.x), pm_copysign(pm_isinf(v.y) ? 1.0f : 0.0f, v.y),
                    pm_copysign(pm_isinf(v.z) ? 1.0f : 0.0f, v.z)};
            v = u;
            d = dot3(v, v);
        }
    }
    return v * pm_rsqrt(d);
}

/* ---- the reference kernel (kernel_bvh.cl:415-431), as compiled for x86-64 ------------ */
void KernelEntry(f3* result, const void* triangles, const void* nodes, const void* materials, unsigned int width,
                 unsigned int height, unsigned int frameCount, unsigned int frameSeed, int lightBounces,
                 int lightType, float skyboxIntensity, f3 cameraPos, f3 cameraFront, f3 cameraUp);

typedef struct {
    float* result;
    const void *tris, *nodes, *mats;
    unsigned width, height, frame;
    int bounces, light_type;
    float sky;
    f3 pos, front, up;
    size_t first, last;
    int threads, index;
} job_t;

static void* worker(void* p) {
    const job_t* j = (const job_t*)p;
    /* interleaved 64-work-item chunks: cheap sky rows and costly rows spread over threads */
    for (size_t base = j->first + (size_t)j->index * 64; base < j->last; base += (size_t)j->threads * 64) {
        const size_t end = base + 64 < j->last ? base + 64 : j->last;
        for (size_t g = base; g < end; ++g) {
            tl_gid = g;
            KernelEntry((f3*)j->result, j->tris, j->nodes, j->mats, j->width, j->height, j->frame, 0u, j->bounces,
                        j->light_type, j->sky, j->pos, j->front, j->up);
        }
    }
    return NULL;
}

/* One NDRange launch of the reference kernel over work-items [first, last): `result` is the
 * float3 buffer (16 B per work-item); cam = {pos, front, up} as 3 x 4 floats. */
int ref_cpu_enqueue(float* result, const void* tris, const void* nodes, const void* mats, unsigned width,
                    unsigned height, unsigned frame_count, int light_bounces, int light_type, float skybox,
                    const float* cam, size_t first, size_t last, int threads) {
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t tid[256];
    job_t jobs[256];
    for (int i = 0; i < threads; ++i) {
        job_t j = {result, tris, nodes, mats, width, height, frame_count, light_bounces, light_type, skybox,
                   {cam[0], cam[1], cam[2]}, {cam[4], cam[5], cam[6]}, {cam[8], cam[9], cam[10]},
                   first, last, threads, i};
        jobs[i] = j;
    }
    int started = 0;
    for (int i = 1; i < threads; ++i) {
        if (pthread_create(&tid[i], NULL, worker, &jobs[i]) != 0) break;
        started = i;
    }
    worker(&jobs[0]);
    for (int i = 1; i <= started; ++i) pthread_join(tid[i], NULL);
    /* work-items a failed thread creation left undone run here */
    for (int i = started + 1; i < threads; ++i) worker(&jobs[i]);
    return 0;
}
