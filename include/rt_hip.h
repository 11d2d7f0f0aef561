/*
 * rt_hip.h -- C ABI of the MI355X hot path (librt_hip.so).
 *
 * Drop-in for the reference's OpenCL device boundary: the CLContext / CLKernel wrapper
 * (/root/reference/CLutils.h:107-145, CLutils.cpp:9-77) and the clCreateBuffer calls of
 * its callers (CLBVHnode.cpp:209-236, CLRaytracer.cpp:122-137).  Plain C types only;
 * every entry point returns 0 (RT_SUCCESS) or a negative cl_int-style code from
 * rt_status.h -- no exception crosses the ABI (the C++ wrapper in rt_cl_compat.hpp
 * turns codes back into the reference's CLException).
 *
 * The kernel "KernelEntry" is precompiled for gfx950 (no runtime JIT).  It takes the
 * reference's 14 argument slots (RenderKernelArgument_t, CLutils.h:11-27):
 *    0 BUFFER_OUT (rt_mem)       4 WIDTH (uint)        8 LIGHT_BOUNCES (int)
 *    1 BUFFER_SCENE (rt_mem)     5 HEIGHT (uint)       9 LIGHT_TYPE (int)
 *    2 BUFFER_NODE (rt_mem)      6 FRAME_COUNT (uint) 10 SKYBOX_INTENSITY (float)
 *    3 BUFFER_MATERIAL (rt_mem)  7 FRAME_SEED (uint)  11-13 CAMERA_POS/FRONT/UP (float3,
 *                                                        16 bytes, w ignored)
 * Buffers hold the CLTriangle / CLLinearBVHNode / CLMaterial bytes of rt_cl_types.h;
 * the output is one 16-byte float3 slot per work-item, as the reference's.
 */
#ifndef RT_HIP_H
#define RT_HIP_H

#include <stddef.h>
#include <stdint.h>

#include "rt_status.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct rt_context_s* rt_context; /* cl::Context + in-order cl::CommandQueue */
typedef struct rt_mem_s* rt_mem;         /* cl::Buffer */
typedef struct rt_kernel_s* rt_kernel;   /* cl::Kernel */

/* cl_mem_flags values (CL/cl.h) accepted by rtCreateBuffer */
#define RT_MEM_READ_WRITE (1u << 0)
#define RT_MEM_WRITE_ONLY (1u << 1)
#define RT_MEM_READ_ONLY (1u << 2)
#define RT_MEM_COPY_HOST_PTR (1u << 5)

/* RenderKernelArgument_t (CLutils.h:11-27) */
enum rt_kernel_arg {
    RT_ARG_BUFFER_OUT = 0,
    RT_ARG_BUFFER_SCENE = 1,
    RT_ARG_BUFFER_NODE = 2,
    RT_ARG_BUFFER_MATERIAL = 3,
    RT_ARG_WIDTH = 4,
    RT_ARG_HEIGHT = 5,
    RT_ARG_FRAME_COUNT = 6,
    RT_ARG_FRAME_SEED = 7,
    RT_ARG_LIGHT_BOUNCES = 8,
    RT_ARG_LIGHT_TYPE = 9,
    RT_ARG_SKYBOX_INTENSITY = 10,
    RT_ARG_CAMERA_POS = 11,
    RT_ARG_CAMERA_FRONT = 12,
    RT_ARG_CAMERA_UP = 13,
    RT_ARG_COUNT = 14
};

/* ---- reference surface --------------------------------------------------------------- */

/* CLContext::CLContext(platform) (CLutils.cpp:9-35): context + in-order queue on GPU
 * `device_index` (the reference always takes device[0]). */
int rtCreateContext(int device_index, rt_context* out);
int rtReleaseContext(rt_context ctx);

/* cl::Buffer(context, flags, size, host_ptr) (CLBVHnode.cpp:215-236,
 * CLRaytracer.cpp:132-135).  With RT_MEM_COPY_HOST_PTR the device gets a copy of
 * `size` bytes of `host_ptr` and the caller keeps its memory.  Other buffers are
 * zero-filled (the reference leaves the output buffer uninitialised). */
int rtCreateBuffer(rt_context ctx, uint64_t flags, size_t size, const void* host_ptr, rt_mem* out);
int rtReleaseBuffer(rt_mem mem);

/* CLKernel::CLKernel(file, devices) (CLutils.cpp:52-66).  The only kernel name is
 * "KernelEntry"; any other -> RT_INVALID_KERNEL_NAME. */
int rtCreateKernel(rt_context ctx, const char* name, rt_kernel* out);
int rtReleaseKernel(rt_kernel k);

/* CLKernel::SetArgument(index, data, size) (CLutils.cpp:68-77).  Buffer slots take a
 * pointer to an rt_mem and size == sizeof(rt_mem); scalar slots size 4; float3 slots
 * size 16 (the reference's host float3, CLmathlib.hpp:18-54).  Values are copied;
 * they persist across launches (set-then-launch, as in RenderFrame). */
int rtSetKernelArg(rt_kernel k, unsigned index, size_t size, const void* value);

/* CLContext::ExecuteKernel(kernel, workSize) (CLutils.cpp:44-50): one work-item per
 * pixel, 1-D NDRange of `global_work_size` (= width*height in the reference).
 * Asynchronous on the context's in-order stream. */
int rtEnqueueKernel(rt_context ctx, rt_kernel k, size_t global_work_size);
/* Extension: frames FRAME_COUNT .. FRAME_COUNT + n_frames - 1 rendered and accumulated into
 * BUFFER_OUT exactly as n_frames rtEnqueueKernel calls with those frame counts would (the
 * reference's RenderFrame loop, CLRaytracer.cpp:35-47, without the per-frame read-back).  The
 * step schedule runs them as ONE launch over (frame, pixel) work items -- one ramp-up and one
 * drain instead of n_frames -- plus a per-pixel accumulation launch; other schedules launch
 * per frame.  The FRAME_COUNT slot is left unchanged; hit buffers receive the last frame's.
 * The accumulation launch runs on a second stream of the context, overlapping the next
 * fused render; every other call on the context (buffer reads/writes/copies, per-frame
 * launches, rtFinish, rtContextGetStream) is ordered after it, so the context still behaves
 * as one in-order queue.  rtContextSetAccumOverlap(ctx, 0) keeps it on the main stream. */
int rtEnqueueKernelFrames(rt_context ctx, rt_kernel k, size_t global_work_size, unsigned n_frames);

/* CLContext::ReadBuffer (CLutils.cpp:37-42, non-blocking in the reference) and
 * CLContext::Finish (CLutils.h:122-125). */
int rtEnqueueReadBuffer(rt_context ctx, rt_mem mem, int blocking, size_t offset, size_t size,
                        void* dst);
int rtFinish(rt_context ctx);

/* ---- extensions (no reference counterpart) ------------------------------------------- */

int rtEnqueueWriteBuffer(rt_context ctx, rt_mem mem, int blocking, size_t offset, size_t size,
                         const void* src);

/* Math policy of the kernel:
 *   RT_MATH_PINNED    -- bit-identical to the pinned CPU semantics of rt_pinned_math.h (oracle);
 *   RT_MATH_DEVICELIB -- the AMD OpenCL device-library builtins the reference kernel
 *                        gets on this GPU, contraction off, correctly rounded / and sqrt
 *                        (the reference built -ffp-contract=off
 *                        -cl-fp32-correctly-rounded-divide-sqrt);
 *   RT_MATH_SHIPPED   -- default: the reference as clBuildProgram(" -I . ") builds it on this GPU
 *                        (CLutils.cpp:52-66): devicelib builtins plus the compiler's default
 *                        FP contraction and OpenCL C's 2.5-ulp division / 3-ulp sqrt. */
#define RT_MATH_PINNED 0
#define RT_MATH_DEVICELIB 1
#define RT_MATH_SHIPPED 2
int rtKernelSetMathMode(rt_kernel k, int mode);

/* Work schedule of the kernel (same results, different lane scheduling):
 * RT_SCHED_TILES           -- one pixel per lane for all of its bounces (16x16 tiles): the
 *                             reference's own shape (one work-item per pixel);
 * RT_SCHED_STEP (default)  -- per-wave state machine: every step advances each lane by one
 *                             BVH node or one triangle; shading and pixel refill run when
 *                             enough lanes are ready;
 * RT_SCHED_WAVEFRONT       -- wavefront path tracing: per bounce an extend
 *                             launch (traversal only, persistent waves pulling rays from an
 *                             HBM ray queue) and a shade launch (one lane per queued path,
 *                             continuations compacted into the next queue); radiance goes to
 *                             per-frame slots and the fused accumulation launch, for
 *                             rtEnqueueKernel too.  Queues take 72 B per work-item and frame.
 *                             lightBounces outside 1..64 run the step schedule. */
#define RT_SCHED_TILES 0
#define RT_SCHED_STEP 2
#define RT_SCHED_WAVEFRONT 4
/* (1 and 3 -- path regeneration and a per-wave LDS path pool -- were measured slower than
 * RT_SCHED_STEP and retired in round 3: rtKernelSetSchedule returns RT_INVALID_VALUE) */
int rtKernelSetSchedule(rt_kernel k, int sched);

/* Device-side BVH build (extension) over the `n_tris` CLTriangle records of
 * `tris` (file order), for meshes too large to build on the host quickly: the triangles sorted
 * by Morton code, then clustered bottom-up (PLOC: mutual nearest neighbours by union surface
 * area within a window of the sorted order -- SAH-like trees) or split by the radix tree of
 * the codes (a linear BVH, cheaper to build and slower to render; rtBuildBVHEx).  Permutes `tris` in place into leaf order and writes the
 * depth-first CLLinearBVHNode[] into `nodes` (capacity >= (2*n_tris - 1) * 48 bytes), count
 * in *n_nodes -- the node contract of CLBVHnode.cpp:161-183, so the buffers bind to
 * KernelEntry as they are (the tree is the first *n_nodes records; the rest of a 2n-1 buffer is
 * ignored, see rtValidateBVH).  The tree is not the host SAH tree (hit IDs may differ where
 * triangles tie). */
int rtBuildBVH(rt_context ctx, rt_mem tris, size_t n_tris, unsigned max_prims_in_node, rt_mem nodes,
               size_t* n_nodes);
/* The same with the tree's topology chosen: RT_BVH_PLOC (rtBuildBVH's) or RT_BVH_LBVH. */
#define RT_BVH_LBVH 0
#define RT_BVH_PLOC 1
int rtBuildBVHEx(rt_context ctx, rt_mem tris, size_t n_tris, unsigned max_prims_in_node, int method, rt_mem nodes,
                 size_t* n_nodes);

/* Restrict the next launches to work-items [first, last) (pixel-row tiles for
 * multi-GPU sharding); last = 0 means "to global_work_size".  Work-item ids, and
 * therefore seeds and output slots, stay global. */
int rtKernelSetWorkRange(rt_kernel k, uint64_t first, uint64_t last);

/* Interleaved 8-row bands for load-balanced multi-GPU sharding: the next launches render
 * only the bands b (rows 8b..8b+7 of the work range) with b % period == phase.  (1, 0)
 * = every band.  Not available with RT_SCHED_TILES (RT_INVALID_OPERATION at launch). */
int rtKernelSetRowInterleave(rt_kernel k, unsigned period, unsigned phase);

/* 2-D device copies for packing / unpacking band-interleaved tiles around a collective:
 * `rows` rows of `width_bytes`, source and destination row pitches in bytes. */
int rtEnqueueCopyBufferRectToPointer(rt_context ctx, rt_mem src, size_t src_offset, size_t src_pitch,
                                     size_t width_bytes, size_t rows, void* dst_device, size_t dst_pitch);
int rtEnqueueCopyPointerRectToBuffer(rt_context ctx, const void* src_device, size_t src_pitch, rt_mem dst,
                                     size_t dst_offset, size_t dst_pitch, size_t width_bytes, size_t rows);

/* Primary-ray outputs per work-item: hit primitive index into the BVH-ordered triangle
 * array (-1 = miss) and isect.t.  Pass NULL to disable. Buffers need 4 B per work-item. */
int rtKernelSetHitBuffers(rt_kernel k, rt_mem hit_ids, rt_mem hit_t);

/* Counters (section 8(d) of SURVEY.md): rays = Intersect() calls, node visits,
 * triangle tests, closest hits.  Enabling selects an instrumented kernel variant. */
typedef struct rt_stats {
    uint64_t rays, node_visits, tri_tests, hits;
    uint64_t launches;
    double kernel_ms;  /* sum of KernelEntry durations (HIP events) when timing is on */
    /* diagnostic (step schedule, stats on): shader-clock cycles summed over waves spent
     * refilling/finishing pixels, traversing, shading, and in total */
    uint64_t cycles_refill, cycles_traverse, cycles_shade, cycles_total;
    /* diagnostic (step schedule, stats on): node steps, lanes served by node steps,
     * triangle steps, lanes served, shading rounds, lanes shaded, refill rounds, lanes freed,
     * then summed over all steps: lanes of the other traversal kind, lanes waiting to shade,
     * free lanes, reserved */
    uint64_t sched[12];
    double accum_ms;   /* sum of the fused frames' accumulation launches (rtEnqueueKernelFrames);
                        * when overlapped (default) the spans include the wait for the render */
    double render_period_ms; /* timed renders: mean interval between the ends of consecutive
                              * launches -- the per-launch time of back-to-back renders, which
                              * overlap (a launch's event span also holds its wait for the CUs
                              * the previous one frees) */
} rt_stats;
int rtKernelSetStats(rt_kernel k, int enable);
int rtKernelSetTiming(rt_kernel k, int enable);
int rtKernelGetStats(rt_kernel k, rt_stats* out);
int rtKernelResetStats(rt_kernel k);

/* Where the scene lives: 1 = staged in LDS (when it fits), 0 = read from HBM/L2. */
int rtKernelGetSceneInLDS(rt_kernel k, int* in_lds);
/* Force the global-memory path even if the scene fits in LDS (testing). */
int rtKernelForceGlobalScene(rt_kernel k, int force);

/* Device-to-device copy of [offset, offset+size) of `src` to a device address (e.g. a
 * collective's staging tensor), asynchronous on the context's stream. */
int rtEnqueueCopyBufferToPointer(rt_context ctx, rt_mem src, size_t offset, size_t size, void* dst_device);

/* Device address of a buffer and the context's HIP stream (for collectives/interop).  The
 * stream is returned after pending fused-frame accumulations have been ordered into it; work
 * enqueued on it directly after a later rtEnqueueKernelFrames must call this again first. */
int rtBufferGetDevicePointer(rt_mem mem, void** dptr);
int rtBufferGetSize(rt_mem mem, size_t* size);
int rtContextGetStream(rt_context ctx, void** hip_stream);
/* Extension (multi-GPU gather): with `enable`, rtEnqueueCopyBufferRectToPointer runs on the
 * context's accumulation stream, right after the fused-frame accumulations enqueued so far
 * and before later ones, instead of joining them into the main stream -- so the next fused
 * render is not held up by the read-back.  Work that consumes the copied bytes waits on the
 * stream rtContextGetAccumStream returns (e.g. an event recorded there after the copies);
 * later calls on the context stay ordered after the copies as before. */
int rtContextSetReadbackOnAccumStream(rt_context ctx, int enable);
int rtContextGetAccumStream(rt_context ctx, void** hip_stream);
int rtContextGetDevice(rt_context ctx, int* device_index);

/* Host-only check (no GPU) of a flattened BVH against the contract KernelEntry relies on
 * (CLBVHnode.cpp:161-183).  The tree is the prefix [0, end) of the n_nodes records, `end` = one
 * past the leaf that node 0's chain of second children reaches (depth-first layout); records
 * past it are never read (by the reference's walk from node 0 either), so a node buffer may be
 * larger than its tree -- e.g. rtBuildBVH's buffer of 2n-1 records holding `count`.  Within the
 * tree: interior node i has children i+1 and offset > i+1, both < end, axis <= 2; leaves
 * [offset, offset + nPrimitives) lie within the n_tris triangles; every node but the root has
 * exactly one parent (one tree, every node reachable).  Every launch runs it on the bound
 * arrays first (RT_INVALID_MEM_OBJECT, never a GPU walk).  *depth = the deepest leaf's depth. */
int rtValidateBVH(const void* nodes, size_t n_nodes, size_t n_tris, int* depth);

/* Scheduling parameters of the persistent schedules (extension; no effect on results, only on
 * speed -- every value renders the same bits).  Defaults were swept on MI355X
 * (profiles/r01/ *_sweep*.txt); these calls exist for re-tuning, replacing environment reads so
 * that library behaviour does not depend on the caller's environment.  Out-of-range values ->
 * RT_INVALID_VALUE.
 *   REFILL_MIN / SHADE_MIN            step schedule, LDS scenes: finish + refill when this many
 *                                     lanes are free (1-64, default 6); shade when this many are
 *                                     ready (1-64, default 48)
 *   REFILL_MIN_GLOBAL / SHADE_MIN_GLOBAL  the same for scenes read from HBM/L2 (0-64; default 0 =
 *                                     auto: 32 / 48 walking octant records, 8 / 48 the 64-B records)
 *   STEP_WEIGHT_NODE / STEP_WEIGHT_LEAF   relative cost of a node / triangle step (35 / 55)
 *   STEP_WEIGHT_NODE_GLOBAL / STEP_WEIGHT_LEAF_GLOBAL  the same for scenes read from HBM/L2 (0 =
 *                                     auto: 65 / 55 walking octant records, else the LDS weights)
 *   CHUNK_PIXELS / TAIL_CHUNK         pixels per work-counter fetch, multiples of 64: bulk chunk
 *                                     (0 = auto: 512, 1024 in the pixel-major order) / largest tail
 *                                     chunk (256; a launch uses the largest
 *                                     power-of-two multiple of 64 up to it that gives every
 *                                     wave >= 2.5 tail chunks)
 *   BULK_PERCENT                      share of the work handed out in bulk chunks (80)
 *   TOP_NODES                         global path: top-of-tree nodes staged in LDS (0-1024, 384)
 *   TILE_MAJOR                        fused work order: -1 auto (default: scenes in HBM/L2 pixel-major
 *                                     for 2, 4 or 8 frames, else tile-major for large launches and
 *                                     frame-major for small ones; LDS scenes frame-major),
 *                                     0 frame-major, 1 tile-major (a tile's frames back to back),
 *                                     2 pixel-major (a pixel's frames side by side in a wave; 2, 4 or 8
 *                                     frames on scenes in HBM/L2, otherwise tile-major)
 *   PERFRAME_SKY                      per-frame sky shortcut: 0 off, 1 large launches (default),
 *                                     2 always
 *   WF_REFILL_MIN                     wavefront extend: take queued rays once this many lanes
 *                                     are free (1-64, default 32)
 *   WF_STREAMS_PER_CU                 wavefront queues: streams per compute unit (0-64; default 0 =
 *                                     the shade workgroups one CU holds at once)
 *   WF_TOP_NODES                      wavefront extend, global path: top-of-tree nodes staged in
 *                                     LDS (0-1024, default 256)
 *   GLOBAL_OCT                        step schedule, scenes not in LDS: 1 (default) = walk the
 *                                     octant-resolved node records (32 B per node and octant) in
 *                                     HBM/L2, 0 = the 64-B node records with the top of the tree
 *                                     in LDS
 *   PERFRAME_DEFER                    step schedule, rtEnqueueKernel: 1 = render into a radiance slot
 *                                     and accumulate in a second launch (as a fused launch of one
 *                                     frame), so frames queued back to back overlap (4K Cornell
 *                                     1.11 -> 0.92 ms/frame); 0 = accumulate inside the render
 *                                     (faster when the host synchronises every frame, as the
 *                                     reference's RenderFrame does, and for small frames);
 *                                     2 (default) = defer a launch of at least PERFRAME_DEFER_MIN
 *                                     work items when the host has not waited on the context
 *                                     through this API (rtFinish, a blocking read or write) since
 *                                     the kernel's previous per-frame launch -- i.e. frames are
 *                                     being queued -- and no stream or device pointer of the
 *                                     context has been handed out (rtContextGetStream,
 *                                     rtContextGetAccumStream, rtBufferGetDevicePointer: the host
 *                                     may then synchronise outside the library, which this rule
 *                                     cannot see; such a host's frames launch on the main stream,
 *                                     at once -- see PERFRAME_BATCH).  Results never change.
 *   PERFRAME_DEFER_MIN                work items from which PERFRAME_DEFER 2 defers (default 4 Mi)
 *   MAX_BLOCKS                        persistent schedules: workgroups per CU of the grid (0 =
 *                                     as many as fit, default; fewer = fewer waves per SIMD)
 *   PERFRAME_BATCH                    step schedule: rtEnqueueKernel calls of this kernel queued
 *                                     back to back with consecutive frameCount and otherwise equal
 *                                     arguments (FRAME_SEED aside: KernelEntry never reads it) are
 *                                     coalesced into one fused launch of up to this many frames
 *                                     (1..8, default 8; 1 = every call launches).  The launch is
 *                                     made before any other call touches the context -- a read, a
 *                                     write, rtFinish, another launch, a kernel setting, a release
 *                                     -- so results are the same bits at every point the host can
 *                                     observe; kernels with stats or timing on are not coalesced.
 *                                     An error of a coalesced launch is returned by the next call
 *                                     on the context that returns one (rtFinish at the latest; a
 *                                     frame enqueued over such an error is not queued).  Once the
 *                                     context's stream (rtContextGetStream, rtContextGetAccumStream)
 *                                     or a device pointer of one of its buffers
 *                                     (rtBufferGetDevicePointer) has been handed out, the host may
 *                                     synchronise outside the library, so from then on every
 *                                     rtEnqueueKernel launches at once. */
enum rt_tuning {
    RT_TUNE_REFILL_MIN = 0,
    RT_TUNE_SHADE_MIN = 1,
    RT_TUNE_REFILL_MIN_GLOBAL = 2,
    RT_TUNE_SHADE_MIN_GLOBAL = 3,
    RT_TUNE_STEP_WEIGHT_NODE = 4,
    RT_TUNE_STEP_WEIGHT_LEAF = 5,
    RT_TUNE_CHUNK_PIXELS = 6,
    RT_TUNE_TAIL_CHUNK = 7,
    RT_TUNE_BULK_PERCENT = 8,
    RT_TUNE_TOP_NODES = 9,
    /* 10-12: the retired pool schedule's thresholds (RT_INVALID_VALUE) */
    RT_TUNE_TILE_MAJOR = 13,
    RT_TUNE_PERFRAME_SKY = 14,
    RT_TUNE_WF_REFILL_MIN = 15,
    RT_TUNE_WF_STREAMS_PER_CU = 16,
    RT_TUNE_WF_TOP_NODES = 17,
    RT_TUNE_GLOBAL_OCT = 18,
    RT_TUNE_PERFRAME_DEFER = 19,
    RT_TUNE_MAX_BLOCKS = 20,
    RT_TUNE_PERFRAME_DEFER_MIN = 21,
    /* 22: the retired speculative walk's switch (RT_INVALID_VALUE) */
    RT_TUNE_PERFRAME_BATCH = 23,
    RT_TUNE_STEP_WEIGHT_NODE_GLOBAL = 24,
    RT_TUNE_STEP_WEIGHT_LEAF_GLOBAL = 25
};
int rtKernelSetTuning(rt_kernel k, int param, int value);
int rtKernelGetTuning(rt_kernel k, int param, int* value);

/* Fused frames' accumulation on the context's second stream, overlapping the next render
 * (default 1), or on the main stream (0).  Synchronises the context. */
int rtContextSetAccumOverlap(rt_context ctx, int enable);

/* ---- multi-GPU: band sharding + RCCL gather (extension) -----------------------
 * The reference renders on one OpenCL device (CLRaytracer.cpp:104-120, CLutils.cpp:29).  Pixels
 * are independent -- the seed depends only on the global work-item id and frameCount
 * (kernel_bvh.cl:445) and the accumulation is per pixel (:449-455) -- so a frame shards by
 * interleaved 8-row bands (band b -> rank b % nranks; rtCommShardKernel) rendered at their
 * global positions, with one exchange at the end: the bands are gathered to a root rank (copy
 * engines over xGMI, or RCCL; rtCommSetTransport), byte-identical to a one-GPU render.
 *
 * Communicators: one rank per GPU, either one process per GPU (rtCommGetUniqueId on one rank,
 * the 128-byte id passed to the others by any host means, rtCommInitRank everywhere) or one
 * process driving several GPUs, one context each (rtCommInitAll = ncclCommInitAll). */
typedef struct rt_comm_s* rt_comm;
#define RT_COMM_ID_BYTES 128
int rtCommGetUniqueId(void* id /* RT_COMM_ID_BYTES */);
int rtCommInitRank(rt_context ctx, int nranks, const void* id, int rank, rt_comm* out);
int rtCommInitAll(const rt_context* ctxs, int n, rt_comm* comms_out);
/* A world of n ranks inside this process WITHOUT RCCL: the same sharding and copy-engine gather as
 * above, the ranks linked by address.  The contexts may share one device (several ranks on one
 * GPU), so the N > 1 gather runs where there is only one GPU.  Every gather and reduction must
 * pass all n communicators (n_local == n); n <= 64. */
int rtCommInitLoopback(const rt_context* ctxs, int n, rt_comm* comms_out);
/* A world of processes on one node WITHOUT RCCL -- e.g. several ranks sharing one GPU, which RCCL
 * refuses: rank `rank` of `nranks`, one process each, meeting through files in the directory `dir`
 * (the same for every rank, empty, on a file system they share; rank 0 writes the world's id into
 * it -- a directory holding an earlier world's is refused, RT_INVALID_VALUE -- and the others wait
 * up to a minute for it, so exchange files an earlier world left are never read; the caller
 * removes the directory after rtCommDestroy).  Setup
 * exchanges, rtCommAllReduceF64 and rtCommBarrier go through the files (each waits at most a
 * minute for the slowest rank); the gathers run on the copy engines over IPC mappings exactly as
 * in an RCCL world (RT_COMM_TRANSPORT_RCCL is refused).  It ships because it is the only way to
 * run the one-process-per-GPU gather (IPC handles, the trial round, flags written into another
 * process's memory) on a machine with one GPU: bench.py --shared-world and the GPU tests use it. */
int rtCommInitShared(rt_context ctx, int nranks, int rank, const char* dir, rt_comm* out);
int rtCommDestroy(rt_comm comm);
int rtCommGetRank(rt_comm comm, int* rank, int* nranks);
/* The kernel renders this rank's bands: rtKernelSetRowInterleave(k, nranks, rank).  The gather's
 * plan counts bands from image row 0, so a kernel with a work range (rtKernelSetWorkRange) is
 * refused (RT_INVALID_OPERATION), and so is setting one on a kernel sharded this way. */
int rtCommShardKernel(rt_comm comm, rt_kernel k);
/* Gather the band-sharded image: every rank's bands of its `out` buffer (width x height pixels
 * of 16 bytes, rendered after rtCommShardKernel) are assembled in the root's `root_dst` (NULL =
 * the root's own `out`).  `comms`/`outs`: the n_local communicators this host thread drives
 * (1 per process in the one-process-per-GPU setup) and their output buffers.  Asynchronous and
 * pipelined, so neither the next fused render nor the next accumulation waits for a transfer:
 *   copy engines (default transport): each rank's copy engine writes its bands, straight from
 *     its `out` (after the fused-frame accumulations and per-frame launches enqueued so far),
 *     into the rows they occupy in the root's destination -- no staging, no pack or unpack
 *     kernel, no compute unit anywhere in the gather -- and raises an arrival flag in the root's
 *     memory; the root's reads of the image wait for every flag.  The root's own bands are in
 *     place when it gathers into its own `out`; else its copy engine copies them like any rank's.
 *     A rank's copies of gather k start once the root has enqueued gather k and finished the
 *     calls it queued before (reads of image k - 1): the root's image never changes under a read
 *     queued on it.  The destination is part of the plan, with the size and the root: in a world
 *     of one rank per process the root refuses (RT_INVALID_OPERATION) a gather into another
 *     buffer until the plan is rebuilt (a size or root change, or rtCommSetTransport -- collective
 *     steps); a destination released meanwhile stays allocated until then.
 *   RCCL: each rank packs its bands into a staging slot on its accumulation stream, grouped
 *     ncclSend/ncclRecv move the slots to the root on the communicator's stream, and the root
 *     unpacks them on a third stream; two staging slots, so step k's gather overlaps step k+1's
 *     render.
 * The communicator's streams run at the device's greatest stream priority.  Every later call on a
 * context that reads or writes memory (rtFinish, rtEnqueueReadBuffer, per-frame launches, ...) is
 * ordered after its part of the gather. */
int rtCommEnqueueGatherBands(const rt_comm* comms, const rt_mem* outs, int n_local, unsigned width,
                             unsigned height, int root, rt_mem root_dst);
/* How the gather moves the bands (set alike on every rank, before a gather; a change takes effect
 * at the next gather, which rebuilds the plan -- a collective step):
 *   RT_COMM_TRANSPORT_COPY_ENGINES (default): the copy engines (SDMA; over xGMI between GPUs) write
 *     every band into the root's destination -- mapped by IPC handle (exchanged with one
 *     ncclAllGather per plan, then checked with one trial copy and flag round across the world)
 *     or, for ranks driven by one process, by address.  Arrival and release are flags
 *     (hipStreamWriteValue64 / hipStreamWaitValue64) between the processes, events within one.  No
 *     compute unit is used for the transfer, so it runs beside a persistent render.  A world in
 *     which some rank cannot map the root's memory falls back to RCCL transfers for the plan
 *     (rtCommGetStatus reports it).
 *   RT_COMM_TRANSPORT_RCCL: grouped ncclSend/ncclRecv on the communicator stream (the root's own
 *     bands too: a device-local send), i.e. RCCL's transfer kernel, with the pack and unpack copies.
 *   RT_COMM_TRANSPORT_COPY_ENGINES_IPC: the copy engines with the links always set up the
 *     multi-process way (IPC handles through ncclAllGather, a world-wide ncclAllReduce on the
 *     outcome) even when every rank is driven by this process -- the one-process-per-GPU path,
 *     selectable at any world size (one local communicator per call).
 * Loopback worlds always use the copy engines. */
#define RT_COMM_TRANSPORT_COPY_ENGINES 0
#define RT_COMM_TRANSPORT_RCCL 1
#define RT_COMM_TRANSPORT_COPY_ENGINES_IPC 2
int rtCommSetTransport(rt_comm comm, int transport);
/* *transport: the requested one; *active: the one the current plan runs (-1: no plan yet). */
int rtCommGetTransport(rt_comm comm, int* transport, int* active);
/* What the communicator's current plan does (self-description for benchmarks and logs). */
#define RT_COMM_FALLBACK_NONE 0
#define RT_COMM_FALLBACK_NO_PEER_ACCESS 1  /* one process, several GPUs: no peer access */
#define RT_COMM_FALLBACK_IPC_MAP 2         /* some rank could not export or map an IPC handle */
#define RT_COMM_FALLBACK_HANDSHAKE 3       /* the trial copy / flag round failed or timed out */
typedef struct rt_comm_status {
    int rank, nranks;
    int transport;         /* requested (rtCommSetTransport) */
    int active;            /* the current plan's transport, -1 before the first gather */
    int fallback;          /* 1: the plan asked for the copy engines and runs RCCL instead */
    int fallback_reason;   /* RT_COMM_FALLBACK_* */
    unsigned copies_per_gather;        /* copy commands this rank issues per gather */
    unsigned long long bytes_per_gather;  /* bytes this rank moves per gather */
    unsigned long long gathers;        /* gathers enqueued with the current plan */
    double last_xfer_ms;   /* the last completed gather's transfer on this rank (its copies, or
                              its RCCL transfer; -1: none measured) */
} rt_comm_status;
int rtCommGetStatus(rt_comm comm, rt_comm_status* out);
/* Test hooks.  RT_COMM_OPT_FAIL_LINKS (value 1): this rank reports its copy-engine links as
 * broken at the next plan's link step, so the world takes the RCCL fallback (what a world whose
 * IPC mappings or trial round fail does). */
#define RT_COMM_OPT_FAIL_LINKS 1
/* RT_COMM_OPT_REPLAN_PERIOD (value 2): gathers per plan before the world re-plans collectively
 * (default 65,534, the flag values a copy-engine plan holds; 1 .. 65,534; every rank of the world
 * must set the same value before its next gather).  RT_COMM_OPT_SYSTEM_ACQUIRE (value 3): the
 * root's first read of a gathered image runs its system-scope acquire (L1 + every XCD's L2) even
 * when every writer is on the root's device -- it always does when another device's copy engines
 * write the image. */
#define RT_COMM_OPT_REPLAN_PERIOD 2
#define RT_COMM_OPT_SYSTEM_ACQUIRE 3
int rtCommSetOption(rt_comm comm, int option, int value);
/* Blocking reductions of `count` doubles per local rank (values: n_local x count, in place),
 * op RT_COMM_SUM or RT_COMM_MAX; rtCommBarrier = a one-value reduction. */
#define RT_COMM_SUM 0
#define RT_COMM_MAX 1
int rtCommAllReduceF64(const rt_comm* comms, int n_local, double* values, int count, int op);
int rtCommBarrier(const rt_comm* comms, int n_local);

/* The pack plan behind the gather (host-only, no GPU needed): the 2-D copies moving rank
 * `phase`'s bands (period ranks) of a width x height image between the image
 * ([img_offset + i*img_pitch, +width) bytes) and a dense staging buffer
 * ([stage_offset + i*width, +width)); at most 2 rects; *staging_bytes = the per-rank staging
 * size (the largest rank's share). */
typedef struct rt_rect {
    uint64_t img_offset, img_pitch, width, rows, stage_offset;
} rt_rect;
int rtBandPackPlan(unsigned width, unsigned height, unsigned period, unsigned phase, rt_rect* rects,
                   int capacity, int* n_rects, size_t* staging_bytes);

/* The pinned math policy's builtins evaluated on the GPU, element-wise over n host values (for
 * tests: the same device functions the pinned KernelEntry runs).  op: RT_PINNED_OP_*; b is read
 * by the two-operand ops only.  Blocking. */
#define RT_PINNED_OP_RCP 0    /* 1.0f / a  (correctly rounded) */
#define RT_PINNED_OP_DIV 1    /* a / b     (correctly rounded) */
#define RT_PINNED_OP_SQRT 2   /* sqrt(a)   (correctly rounded) */
#define RT_PINNED_OP_RSQRT 3  /* 1.0f / sqrt(a), two rounded operations (normalize's, a >= 2^-126) */
#define RT_PINNED_OP_POW 4    /* pow(a, b) (rt_pinned_math.h pm_pow) */
#define RT_PINNED_OP_SIN 5
#define RT_PINNED_OP_COS 6
int rtDiagPinnedMath(int device_index, int op, const float* a, const float* b, float* out, size_t n);

/* Library identification (for smoke checks): returns a static string. */
const char* rtGetBuildInfo(void);

#ifdef __cplusplus
}
#endif

#endif /* RT_HIP_H */
