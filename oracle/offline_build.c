/*
 * offline_build.c -- test infrastructure: build the UNMODIFIED reference kernel with the image's
 * own OpenCL runtime exactly as the reference host does, without a GPU.
 *
 * The reference JIT-compiles kernel_bvh.cl at start-up with program.build(" -I . ")
 * (/root/reference/CLutils.cpp:52-66).  AMD's OpenCL runtime can build for devices that are not
 * present through its offline-device extension (cl_amd_offline_devices: context property
 * CL_CONTEXT_OFFLINE_DEVICES_AMD), so the same clCreateProgramWithSource + clBuildProgram path the
 * reference takes -- the runtime's own option handling, device-library selection and code
 * generation -- runs here, and the resulting code object (clGetProgramInfo CL_PROGRAM_BINARIES)
 * can be compared with oracle/_ref/kernel_bvh_shipped.co, the clang build the `shipped` math
 * policy was derived from (tests/test_ref_runtime_build.py).
 *
 * usage: offline_build <source.cl> <dir> <device name> <out.co> [build options]
 *   <device name>: exactly as the runtime names the GPU the reference would run on -- an MI355X is
 *   "gfx950:sramecc+:xnack-" (clinfo on the GPU box)
 *   The program is built from <source.cl> with the working directory set to <dir> during
 *   clBuildProgram, so the reference's own " -I . " (the default options) resolves as it does for
 *   the reference; nothing is written there.  <source.cl> = <dir>/kernel_bvh.cl builds the
 *   reference program itself; oracle/ref_entry.cl (which #includes it) adds the PrimaryHitEntry
 *   harness so the code object runs through oracle/clref.py.
 */
#define CL_TARGET_OPENCL_VERSION 200
#include <CL/cl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#ifndef CL_CONTEXT_OFFLINE_DEVICES_AMD
#define CL_CONTEXT_OFFLINE_DEVICES_AMD 0x403F
#endif

static char* slurp(const char* path, size_t* n) {
    FILE* f = fopen(path, "rb");
    if (!f) return NULL;
    fseek(f, 0, SEEK_END);
    long sz = ftell(f);
    fseek(f, 0, SEEK_SET);
    char* b = malloc((size_t)sz + 1);
    if (b && fread(b, 1, (size_t)sz, f) != (size_t)sz) {
        free(b);
        b = NULL;
    }
    fclose(f);
    if (b) b[sz] = 0;
    if (n) *n = (size_t)sz;
    return b;
}

int main(int argc, char** argv) {
    if (argc < 5) {
        fprintf(stderr, "usage: %s <source.cl> <dir> <device> <out.co> [options]\n", argv[0]);
        return 2;
    }
    const char* src_path = argv[1];
    const char* dir = argv[2];
    const char* want = argv[3];
    const char* outp = argv[4];
    const char* opts = argc > 5 ? argv[5] : " -I . ";
    char cwd[4096];
    if (!getcwd(cwd, sizeof cwd)) return 2;
    size_t n = 0;
    char* src = slurp(src_path, &n);
    if (!src) {
        fprintf(stderr, "cannot read %s\n", src_path);
        return 2;
    }
    cl_platform_id plat;
    cl_uint np = 0;
    if (clGetPlatformIDs(1, &plat, &np) != CL_SUCCESS || np == 0) {
        fprintf(stderr, "no OpenCL platform\n");
        return 3;
    }
    cl_context_properties props[] = {CL_CONTEXT_PLATFORM, (cl_context_properties)plat,
                                     CL_CONTEXT_OFFLINE_DEVICES_AMD, (cl_context_properties)1, 0};
    cl_int err = 0;
    cl_context ctx = clCreateContextFromType(props, CL_DEVICE_TYPE_ALL, NULL, NULL, &err);
    if (!ctx || err != CL_SUCCESS) {
        fprintf(stderr, "offline context: error %d\n", err);
        return 3;
    }
    size_t dbytes = 0;
    clGetContextInfo(ctx, CL_CONTEXT_DEVICES, 0, NULL, &dbytes);
    cl_uint nd = (cl_uint)(dbytes / sizeof(cl_device_id));
    cl_device_id* devs = malloc(dbytes);
    clGetContextInfo(ctx, CL_CONTEXT_DEVICES, dbytes, devs, NULL);
    cl_device_id dev = NULL;
    for (cl_uint i = 0; i < nd; ++i) {
        char name[256] = {0};
        clGetDeviceInfo(devs[i], CL_DEVICE_NAME, sizeof name, name, NULL);
        if (strcmp(name, want) == 0) dev = devs[i];
    }
    if (!dev) {
        fprintf(stderr, "no offline device %s among %u\n", want, nd);
        return 3;
    }
    const char* s = src;
    cl_program prog = clCreateProgramWithSource(ctx, 1, &s, &n, &err);
    if (err != CL_SUCCESS) return 4;
    if (chdir(dir) != 0) return 4;
    err = clBuildProgram(prog, 1, &dev, opts, NULL, NULL);
    if (chdir(cwd) != 0) return 4;
    size_t lb = 0;
    clGetProgramBuildInfo(prog, dev, CL_PROGRAM_BUILD_LOG, 0, NULL, &lb);
    char* log = malloc(lb + 1);
    clGetProgramBuildInfo(prog, dev, CL_PROGRAM_BUILD_LOG, lb, log, NULL);
    log[lb] = 0;
    if (err != CL_SUCCESS) {
        fprintf(stderr, "clBuildProgram(\"%s\"): error %d\n%s\n", opts, err, log);
        return 5;
    }
    size_t bsz = 0;
    clGetProgramInfo(prog, CL_PROGRAM_BINARY_SIZES, sizeof bsz, &bsz, NULL);
    unsigned char* bin = malloc(bsz);
    unsigned char* bins[1] = {bin};
    clGetProgramInfo(prog, CL_PROGRAM_BINARIES, sizeof bins, bins, NULL);
    FILE* f = fopen(outp, "wb");
    if (!f || fwrite(bin, 1, bsz, f) != bsz) return 6;
    fclose(f);
    printf("built %s for %s with \"%s\": %zu bytes\n", src_path, want, opts, bsz);
    return 0;
}
