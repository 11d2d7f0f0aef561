// rt_internal.hpp -- objects shared by the C ABI translation units (rt_capi.cpp, rt_comm.cpp):
// the context (cl::Context + in-order cl::CommandQueue, CLutils.cpp:9-35) and the buffer
// (cl::Buffer, CLBVHnode.cpp:215-236).  Not part of the public ABI.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

#include "../../include/rt_hip.h"

// fused frames: radiance sets used in rotation, so a render waits only for the accumulation of the
// launch RT_RAD_SETS steps back; consecutive renders alternate between RT_RENDER_STREAMS streams, so
// at most that many renders are in flight
#ifndef RT_RAD_SETS
#define RT_RAD_SETS 2
#endif
#ifndef RT_RENDER_STREAMS
#define RT_RENDER_STREAMS 2
#endif

struct rt_context_s {
    int device = 0;
    hipStream_t stream = nullptr;
    int num_cus = 0;
    int n_xcd = 1;  // XCDs (CU-mask bit b selects CU b / n_xcd of XCD b % n_xcd)
    // Fused frames: the accumulation launch runs on its own stream, so it overlaps the next
    // render (its waves fit beside the render grid: 32 VGPRs).  Every other operation
    // goes through qs(), which first makes the context's in-order stream wait for the
    // accumulations enqueued so far -- to the caller the context stays one in-order queue.
    hipStream_t astream = nullptr;
    hipEvent_t atail = nullptr;  // last accumulation enqueued on astream
    // fused renders alternate between two streams, one per radiance set (rt_capi.cpp enqueue):
    // renders of consecutive steps are independent, so step k+1's waves take the CUs that step
    // k's draining waves free instead of waiting for its last path
    hipStream_t rstream[RT_RENDER_STREAMS] = {};
    int rnext = 0;  // the render stream of the next fused render
    hipEvent_t mtail = nullptr;  // main stream's tail, for copies issued on astream
    // Work may have been enqueued on the main stream since mtail was last recorded
    // (main_tail_wait).  Streams share hardware queues (GPU_MAX_HW_QUEUES 4 < the context's and
    // communicator's streams), so a fresh record on an idle main stream can land behind another
    // stream's packets -- the previous step's gather transfer -- and make the next fused render
    // wait for it.  Set by every path that enqueues there: qs() (all of them but enqueue's own
    // launches, which set it themselves); sticky once the stream handle is exposed
    // (rtContextGetStream), since the caller may then enqueue without telling us.
    bool mdirty = true;
    bool mexposed = false;
    // a device pointer of one of the context's buffers, or its accumulation stream, was handed out:
    // the host may synchronise outside the library, so per-frame launches are no longer coalesced
    bool dexposed = false;
    bool apending = false;
    // host waits on the queue (rtFinish, blocking reads / writes): a per-frame launch with no wait
    // since the previous one is being queued back to back (automatic per-frame deferral)
    uint64_t host_waits = 0;
    bool overlap = true;  // rtContextSetAccumOverlap(ctx, 0): accumulate on the main stream
    // rtContextSetReadbackOnAccumStream: buffer -> pointer rect copies go to astream, right after
    // the accumulation they read, so the main stream runs on into the next render
    bool readback_on_astream = false;
    // multi-GPU gather (rt_comm.cpp) in flight on the communicator's streams: joined by qs() like
    // the accumulations, so reads of the gathered image are ordered after it
    hipEvent_t gtail = nullptr;
    bool gpending = false;
    // a copy-engine gather between processes whose arrivals the root has not joined yet: the
    // stream that next reads the image waits for the arrival flags (rti::join_gather) -- no
    // waiting kernel is enqueued while nobody reads (rt_comm.cpp)
    rt_comm gjoin = nullptr;
    // a root gathering into another buffer copies its own bands straight from its output: the
    // next accumulation -- which rewrites the output -- waits for those copies (oread_ev)
    hipEvent_t oread_ev = nullptr;
    bool oread = false;
    // per-frame launches queued back to back and not launched yet (rt_capi.cpp, frame
    // coalescing): frames pend_f0 .. pend_f0 + pend_n - 1 of pend_k with the arguments they were
    // enqueued with; launched as one fused launch before anything else touches the context
    // (flush_frames; qs() flushes, so every enqueue, read, write and wait does)
    rt_kernel pend_k = nullptr;
    size_t pend_gws = 0;
    uint32_t pend_f0 = 0, pend_n = 0;
    uint32_t pend_u32[RT_ARG_COUNT] = {};
    float pend_f3[3][4] = {};
    rt_mem pend_bufs[4] = {};
    int pend_error = RT_SUCCESS;  // a failed coalesced launch, reported by the next call that can
};

struct rt_mem_s {
    rt_context ctx = nullptr;
    void* dptr = nullptr;
    size_t size = 0;
    uint64_t flags = 0;
    std::vector<uint8_t> shadow;  // host copy of the bytes (valid when shadow_valid)
    bool shadow_valid = false;
    uint64_t generation = 0;      // bumped on every host write
    // a copy-engine gather plan writes into this buffer (the root's destination, rt_comm.cpp):
    // rtReleaseBuffer then only marks it, and the plan frees it when it lets go (rti::unpin)
    int pins = 0;
    bool released = false;
};

namespace rti {

inline int map_hip(hipError_t e) {
    switch (e) {
        case hipSuccess: return RT_SUCCESS;
        case hipErrorOutOfMemory: return RT_MEM_OBJECT_ALLOCATION_FAILURE;
        case hipErrorNoDevice:
        case hipErrorInvalidDevice: return RT_DEVICE_NOT_FOUND;
        case hipErrorLaunchOutOfResources: return RT_OUT_OF_RESOURCES;
        default: return RT_INVALID_OPERATION;
    }
}

// Launch the coalesced per-frame launches of `ctx`, if any (rt_capi.cpp).  Returns their error,
// which is also kept in ctx->pend_error for the next call that reports one.
int flush_frames(rt_context ctx);

// `s` waits for the root's pending gather arrivals (rt_comm.cpp; records gtail behind them)
hipError_t join_gather(rt_comm c, hipStream_t s);

// `s` waits for the gathers enqueued on the context so far (reads of a gathered image).  A join
// that fails keeps its state (gjoin): the next read joins again, and the error is kept for the
// next call that reports one (qs)
inline hipError_t gather_wait(rt_context ctx, hipStream_t s) {
    hipError_t e = hipSuccess;
    if (ctx->gjoin) {
        e = join_gather(ctx->gjoin, s);  // (then gtail is the joining stream's tail)
        if (e != hipSuccess) return e;
        ctx->gjoin = nullptr;
        ctx->gpending = s != ctx->stream;
        return e;
    }
    if (ctx->gpending) {
        e = hipStreamWaitEvent(s, ctx->gtail, 0);
        if (e == hipSuccess && s == ctx->stream) ctx->gpending = false;
    }
    return e;
}

// The context's stream, after every pending accumulation and gather (see rt_context_s) and the
// coalesced per-frame launches.  A failed wait is reported by the next call that returns a status
// (ctx->pend_error).
inline hipStream_t qs(rt_context ctx) {
    if (ctx->pend_k) (void)flush_frames(ctx);
    if (ctx->apending) {
        (void)hipStreamWaitEvent(ctx->stream, ctx->atail, 0);
        ctx->apending = false;
    }
    const hipError_t ge = gather_wait(ctx, ctx->stream);
    if (ge != hipSuccess && ctx->pend_error == RT_SUCCESS) ctx->pend_error = map_hip(ge);
    ctx->mdirty = true;  // the caller enqueues on it
    return ctx->stream;
}

// Make `s` wait for everything enqueued on the main stream so far.  The main stream's tail is
// re-recorded only when something may have been enqueued there since the last record.
inline hipError_t main_tail_wait(rt_context ctx, hipStream_t s) {
    if (ctx->mdirty || ctx->mexposed) {
        const hipError_t e = hipEventRecord(ctx->mtail, ctx->stream);
        if (e != hipSuccess) return e;
        ctx->mdirty = false;
    }
    return hipStreamWaitEvent(s, ctx->mtail, 0);
}

// the next accumulation launch on `s` rewrites the output: after the gather copies reading it
inline hipError_t out_read_wait(rt_context ctx, hipStream_t s) {
    if (!ctx->oread) return hipSuccess;
    ctx->oread = false;
    return hipStreamWaitEvent(s, ctx->oread_ev, 0);
}

// Gather destinations (rt_mem_s::pins): a pinned buffer outlives rtReleaseBuffer until unpinned.
inline void pin(rt_mem m) { ++m->pins; }
void unpin(rt_mem m);  // rt_capi.cpp: frees a released buffer on its last unpin

// rtCommShardKernel's interleave (rt_capi.cpp): refused for a kernel with a work range
int shard_kernel(rt_kernel k, unsigned period, unsigned phase);


}  // namespace rti
