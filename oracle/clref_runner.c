/*
 * clref_runner.c -- OpenCL host for the reference kernel (test infrastructure only).
 *
 * Loads a gfx950 code object built from /root/reference/kernel_bvh.cl (oracle/_ref,
 * see `make -C oracle ref`) through the system OpenCL runtime (ICD -> libamdocl64) and
 * drives it the way the reference host does: buffers created READ_ONLY|COPY_HOST_PTR
 * (CLBVHnode.cpp:209-236), the 14 KernelEntry arguments (CLutils.h:11-27), a 1-D
 * NDRange of W*H work-items with a runtime-chosen local size (CLutils.cpp:44-50), and a
 * read-back of the float3 output (CLutils.cpp:37-42).  Exposed as a small C API for
 * ctypes (tests/test_ref_opencl.py).  The output buffer starts zero-filled (the
 * reference leaves it uninitialised).
 */
#define CL_TARGET_OPENCL_VERSION 120
#include <CL/cl.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef struct clref {
    cl_context ctx;
    cl_command_queue q;
    cl_program prog;
    cl_kernel entry, hits;
    cl_device_id dev;
    char device_name[256];
} clref;

static unsigned char* read_file(const char* path, size_t* len) {
    FILE* f = fopen(path, "rb");
    if (!f) return NULL;
    fseek(f, 0, SEEK_END);
    long n = ftell(f);
    fseek(f, 0, SEEK_SET);
    unsigned char* b = (unsigned char*)malloc((size_t)n);
    if (b && fread(b, 1, (size_t)n, f) != (size_t)n) {
        free(b);
        b = NULL;
    }
    fclose(f);
    *len = (size_t)n;
    return b;
}

/* Returns NULL and sets *err (cl_int or -1000 for a file error) on failure. */
clref* clref_open(const char* code_object, int* err) {
    cl_int e;
    cl_platform_id plats[8];
    cl_uint np = 0;
    *err = 0;
    e = clGetPlatformIDs(8, plats, &np);
    if (e != CL_SUCCESS || np == 0) { *err = e ? e : CL_DEVICE_NOT_FOUND; return NULL; }
    cl_device_id dev = NULL;
    for (cl_uint i = 0; i < np && !dev; ++i) {
        cl_uint nd = 0;
        if (clGetDeviceIDs(plats[i], CL_DEVICE_TYPE_GPU, 1, &dev, &nd) != CL_SUCCESS || nd == 0) dev = NULL;
    }
    if (!dev) { *err = CL_DEVICE_NOT_FOUND; return NULL; }
    clref* r = (clref*)calloc(1, sizeof(clref));
    r->dev = dev;
    clGetDeviceInfo(dev, CL_DEVICE_NAME, sizeof(r->device_name) - 1, r->device_name, NULL);
    r->ctx = clCreateContext(NULL, 1, &dev, NULL, NULL, &e);
    if (e != CL_SUCCESS) { *err = e; free(r); return NULL; }
    r->q = clCreateCommandQueue(r->ctx, dev, 0, &e);
    if (e != CL_SUCCESS) { *err = e; clReleaseContext(r->ctx); free(r); return NULL; }
    size_t len = 0;
    unsigned char* bin = read_file(code_object, &len);
    if (!bin) { *err = -1000; clReleaseCommandQueue(r->q); clReleaseContext(r->ctx); free(r); return NULL; }
    cl_int status = 0;
    const unsigned char* bins[1] = {bin};
    r->prog = clCreateProgramWithBinary(r->ctx, 1, &dev, &len, bins, &status, &e);
    free(bin);
    if (e == CL_SUCCESS) e = clBuildProgram(r->prog, 1, &dev, "", NULL, NULL);
    if (e == CL_SUCCESS) r->entry = clCreateKernel(r->prog, "KernelEntry", &e);
    if (e == CL_SUCCESS) r->hits = clCreateKernel(r->prog, "PrimaryHitEntry", &e);
    if (e != CL_SUCCESS) { *err = e; return NULL; }
    return r;
}

const char* clref_device_name(clref* r) { return r ? r->device_name : ""; }

void clref_close(clref* r) {
    if (!r) return;
    if (r->entry) clReleaseKernel(r->entry);
    if (r->hits) clReleaseKernel(r->hits);
    if (r->prog) clReleaseProgram(r->prog);
    if (r->q) clReleaseCommandQueue(r->q);
    if (r->ctx) clReleaseContext(r->ctx);
    free(r);
}

typedef struct {
    const void* tris; size_t tris_bytes;
    const void* nodes; size_t nodes_bytes;
    const void* mats; size_t mats_bytes;
    uint32_t width, height;
    int32_t lightBounces, lightType;
    float skyboxIntensity;
    float cam[12];
} clref_scene;

/* KernelEntry for frames frame_first..frame_last (accumulating in one buffer), then the
 * W*H float4 result is read into `result`.  Returns a cl_int. */
int clref_render(clref* r, const clref_scene* s, uint32_t frame_first, uint32_t frame_last, float* result) {
    cl_int e;
    const size_t n = (size_t)s->width * s->height;
    cl_mem tb = clCreateBuffer(r->ctx, CL_MEM_READ_ONLY | CL_MEM_COPY_HOST_PTR, s->tris_bytes, (void*)s->tris, &e);
    if (e) return e;
    cl_mem nb = clCreateBuffer(r->ctx, CL_MEM_READ_ONLY | CL_MEM_COPY_HOST_PTR, s->nodes_bytes, (void*)s->nodes, &e);
    if (e) return e;
    cl_mem mb = clCreateBuffer(r->ctx, CL_MEM_READ_ONLY | CL_MEM_COPY_HOST_PTR, s->mats_bytes, (void*)s->mats, &e);
    if (e) return e;
    cl_mem ob = clCreateBuffer(r->ctx, CL_MEM_READ_WRITE | CL_MEM_COPY_HOST_PTR, n * 16, result, &e);
    if (e) return e;
    cl_kernel k = r->entry;
    cl_uint seed = 0;
    e = clSetKernelArg(k, 0, sizeof(cl_mem), &ob);
    e |= clSetKernelArg(k, 1, sizeof(cl_mem), &tb);
    e |= clSetKernelArg(k, 2, sizeof(cl_mem), &nb);
    e |= clSetKernelArg(k, 3, sizeof(cl_mem), &mb);
    e |= clSetKernelArg(k, 4, sizeof(cl_uint), &s->width);
    e |= clSetKernelArg(k, 5, sizeof(cl_uint), &s->height);
    e |= clSetKernelArg(k, 7, sizeof(cl_uint), &seed);
    e |= clSetKernelArg(k, 8, sizeof(cl_int), &s->lightBounces);
    e |= clSetKernelArg(k, 9, sizeof(cl_int), &s->lightType);
    e |= clSetKernelArg(k, 10, sizeof(cl_float), &s->skyboxIntensity);
    e |= clSetKernelArg(k, 11, sizeof(cl_float3), &s->cam[0]);
    e |= clSetKernelArg(k, 12, sizeof(cl_float3), &s->cam[4]);
    e |= clSetKernelArg(k, 13, sizeof(cl_float3), &s->cam[8]);
    for (uint32_t f = frame_first; e == CL_SUCCESS && f <= frame_last; ++f) {
        e = clSetKernelArg(k, 6, sizeof(cl_uint), &f);
        if (e == CL_SUCCESS) e = clEnqueueNDRangeKernel(r->q, k, 1, NULL, &n, NULL, 0, NULL, NULL);
    }
    if (e == CL_SUCCESS) e = clEnqueueReadBuffer(r->q, ob, CL_TRUE, 0, n * 16, result, 0, NULL, NULL);
    if (e == CL_SUCCESS) e = clFinish(r->q);
    clReleaseMemObject(ob);
    clReleaseMemObject(mb);
    clReleaseMemObject(nb);
    clReleaseMemObject(tb);
    return e;
}

/* PrimaryHitEntry for one frame: hit primitive index and t per work-item. */
int clref_primary_hits(clref* r, const clref_scene* s, uint32_t frame, int32_t* ids, float* t) {
    cl_int e;
    const size_t n = (size_t)s->width * s->height;
    cl_mem tb = clCreateBuffer(r->ctx, CL_MEM_READ_ONLY | CL_MEM_COPY_HOST_PTR, s->tris_bytes, (void*)s->tris, &e);
    if (e) return e;
    cl_mem nb = clCreateBuffer(r->ctx, CL_MEM_READ_ONLY | CL_MEM_COPY_HOST_PTR, s->nodes_bytes, (void*)s->nodes, &e);
    if (e) return e;
    cl_mem mb = clCreateBuffer(r->ctx, CL_MEM_READ_ONLY | CL_MEM_COPY_HOST_PTR, s->mats_bytes, (void*)s->mats, &e);
    if (e) return e;
    cl_mem ib = clCreateBuffer(r->ctx, CL_MEM_WRITE_ONLY, n * 4, NULL, &e);
    if (e) return e;
    cl_mem fb = clCreateBuffer(r->ctx, CL_MEM_WRITE_ONLY, n * 4, NULL, &e);
    if (e) return e;
    cl_kernel k = r->hits;
    e = clSetKernelArg(k, 0, sizeof(cl_mem), &ib);
    e |= clSetKernelArg(k, 1, sizeof(cl_mem), &fb);
    e |= clSetKernelArg(k, 2, sizeof(cl_mem), &tb);
    e |= clSetKernelArg(k, 3, sizeof(cl_mem), &nb);
    e |= clSetKernelArg(k, 4, sizeof(cl_mem), &mb);
    e |= clSetKernelArg(k, 5, sizeof(cl_uint), &s->width);
    e |= clSetKernelArg(k, 6, sizeof(cl_uint), &s->height);
    e |= clSetKernelArg(k, 7, sizeof(cl_uint), &frame);
    e |= clSetKernelArg(k, 8, sizeof(cl_float3), &s->cam[0]);
    e |= clSetKernelArg(k, 9, sizeof(cl_float3), &s->cam[4]);
    e |= clSetKernelArg(k, 10, sizeof(cl_float3), &s->cam[8]);
    if (e == CL_SUCCESS) e = clEnqueueNDRangeKernel(r->q, k, 1, NULL, &n, NULL, 0, NULL, NULL);
    if (e == CL_SUCCESS) e = clEnqueueReadBuffer(r->q, ib, CL_TRUE, 0, n * 4, ids, 0, NULL, NULL);
    if (e == CL_SUCCESS) e = clEnqueueReadBuffer(r->q, fb, CL_TRUE, 0, n * 4, t, 0, NULL, NULL);
    if (e == CL_SUCCESS) e = clFinish(r->q);
    clReleaseMemObject(fb);
    clReleaseMemObject(ib);
    clReleaseMemObject(mb);
    clReleaseMemObject(nb);
    clReleaseMemObject(tb);
    return e;
}
