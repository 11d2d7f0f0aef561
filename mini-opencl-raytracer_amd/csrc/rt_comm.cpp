// rt_comm.cpp -- multi-GPU band sharding + RCCL gather, behind include/rt_hip.h.
//
// The reference is single-device (CLRaytracer.cpp:104-120, one in-order queue CLutils.cpp:29).
// A frame shards with no exchange until the image is needed, because every pixel's seed is
// gid + HashUInt32(frameCount) over the GLOBAL work-item id (kernel_bvh.cl:445) and the gamma
// accumulation is per pixel (:449-455).  Rank r renders the interleaved 8-row bands
// b % nranks == r into its full-size output buffer (rtKernelSetRowInterleave); the gather then
// moves each rank's bands, packed densely, to the root:
//
//   context accumulation stream : [accumulate k] [pack k -> stage[s]]  [accumulate k+1] ...
//   communicator stream         :                 (wait pack) [RCCL send/recv k]   ...
//   root unpack stream          :                              (wait recv) [unpack k -> dst]
//   context main stream         : [render k+1 ..........................................]
//
// Two staging slots alternate, so step k's transfer runs under step k+1's render.  RCCL p2p
// (grouped ncclSend/ncclRecv) lets the root receive from all peers at once on its xGMI links
// (a ring all-gather would push N x the bytes through single links).  The packs/unpacks are 2-D
// copies (one per rank: full bands are equally strided, plus at most one short last band).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <cstring>
#include <new>
#include <vector>

#include "../../include/rt_hip.h"
#include "rt_internal.hpp"

using rti::map_hip;
using rti::qs;

namespace {

constexpr unsigned kBandRows = 8;     // = the 8x8 tile height of the persistent schedules
constexpr size_t kPixelBytes = 16;    // one float3 slot of the output buffer

int map_nccl(ncclResult_t r) {
    switch (r) {
        case ncclSuccess: return RT_SUCCESS;
        case ncclInvalidArgument:
        case ncclInvalidUsage: return RT_INVALID_VALUE;
        case ncclSystemError: return RT_OUT_OF_RESOURCES;
        default: return RT_INVALID_OPERATION;
    }
}

// mirror of clrt/multigpu.py pack_plan (tests compare the two)
int band_plan(unsigned W, unsigned H, unsigned period, unsigned phase, rt_rect* rects, int cap, int* n,
              size_t* staging) {
    if (W == 0 || H == 0 || period == 0 || phase >= period) return RT_INVALID_VALUE;
    const uint64_t nb = (H + kBandRows - 1) / kBandRows;
    const uint64_t band_bytes = (uint64_t)kBandRows * W * kPixelBytes;
    const uint64_t per_rank = (nb + period - 1) / period;
    if (staging) *staging = (size_t)(per_rank * band_bytes);
    // bands phase, phase + period, ... < nb; only band nb - 1 can be short
    uint64_t count = phase < nb ? (nb - 1 - phase) / period + 1 : 0;
    const uint64_t last = count ? phase + (count - 1) * period : 0;
    const bool short_last = count && (last + 1) * kBandRows > H;
    const uint64_t full = short_last ? count - 1 : count;
    int k = 0;
    rt_rect tmp[2];
    if (full) tmp[k++] = rt_rect{phase * band_bytes, period * band_bytes, band_bytes, full, 0};
    if (short_last) {
        const uint64_t rows = H - last * kBandRows;
        tmp[k++] = rt_rect{last * band_bytes, band_bytes, rows * W * kPixelBytes, 1, full * band_bytes};
    }
    if (n) *n = k;
    if (rects) {
        if (cap < k) return RT_INVALID_VALUE;
        for (int i = 0; i < k; ++i) rects[i] = tmp[i];
    }
    return RT_SUCCESS;
}

}  // namespace

struct rt_comm_s {
    rt_context ctx = nullptr;
    ncclComm_t nc = nullptr;
    // loopback worlds (rtCommInitLoopback): no RCCL; `group` identifies the world (shared by its
    // members) and the transfer is a device copy on the root's communicator stream
    const void* group = nullptr;
    hipEvent_t xfer = nullptr;  // root: the copies of one gather done
    bool reserved = false;      // holds a CU reservation on ctx (rti::reserve_cus)
    int rank = 0, nranks = 1;
    hipStream_t cstream = nullptr;  // RCCL
    hipStream_t ustream = nullptr;  // root: unpack
    // gather buffers for one (width, height); rebuilt when the image size changes
    unsigned W = 0, H = 0;
    int root = -1;
    size_t stage_bytes = 0;
    std::vector<std::vector<rt_rect>> plans;  // per rank
    void* stage[2] = {};                      // this rank's packed bands
    void* parts[2] = {};                      // root: nranks x stage_bytes received bands
    hipEvent_t packed[2] = {}, sent[2] = {}, unpacked[2] = {};
    bool sent_valid[2] = {}, unpacked_valid[2] = {};
    int slot = 0;
    double* scratch = nullptr;  // reductions
};

namespace {

// The communicator's transfer and unpack streams run at the device's greatest stream priority.
// Two reasons, both read off a kernel trace of the world-1 flow (profiles/r04/dist_streams.txt):
// * HIP maps streams onto a few hardware queues (GPU_MAX_HW_QUEUES 4); at normal priority these two
//   shared the main stream's and a render stream's queue, so the next fused render sat behind the
//   previous step's unpack, which sat behind its transfer.  High-priority streams get queues of
//   their own.
// * RCCL's transfer kernel needs CU slots, and a persistent render holds them all until it
//   drains; at normal priority the next render's workgroups took the slots the draining one
//   freed, and the transfer waited (6.4 ms for a 0.11-ms copy).  At high priority its workgroups
//   are dispatched first.
#ifndef RT_COMM_STREAM_PRIO
#define RT_COMM_STREAM_PRIO 1
#endif
// RCCL communicators: CUs of every XCD kept for the communicator's streams (rti::reserve_cus).
// RCCL's transfer kernel (64 workgroups of 256 threads, 37 KB of LDS and 248 VGPRs each on
// gfx950) does not fit beside a persistent render on any CU, so without a reservation it runs
// only where renders drain (profiles/r04/dist_streams.txt); with one it runs at once on its own
// CUs, and the renders lose those CUs' share (1 per XCD = 8 of 256 = 3 %).  0 = none.
int comm_events(rt_comm c, hipError_t e);
#ifndef RT_COMM_RESERVE_PER_XCD
#define RT_COMM_RESERVE_PER_XCD 0
#endif
int comm_streams(rt_comm c, bool rccl) {
    hipError_t e = hipSuccess;
    if (rccl && RT_COMM_RESERVE_PER_XCD > 0) {
        std::vector<uint32_t> mask;
        int rc = rti::reserve_cus(c->ctx, RT_COMM_RESERVE_PER_XCD, &mask);
        if (rc) return rc;
        c->reserved = true;
        ++c->ctx->reserve_refs;
        e = hipExtStreamCreateWithCUMask(&c->cstream, (uint32_t)mask.size(), mask.data());
        if (e == hipSuccess) e = hipExtStreamCreateWithCUMask(&c->ustream, (uint32_t)mask.size(), mask.data());
        return comm_events(c, e);
    }
    int least = 0, greatest = 0;
    e = hipDeviceGetStreamPriorityRange(&least, &greatest);
    const int prio = RT_COMM_STREAM_PRIO ? greatest : least;
    if (e == hipSuccess) e = hipStreamCreateWithPriority(&c->cstream, hipStreamNonBlocking, prio);
    if (e == hipSuccess) e = hipStreamCreateWithPriority(&c->ustream, hipStreamNonBlocking, prio);
    return comm_events(c, e);
}

int comm_events(rt_comm c, hipError_t e) {
    for (int s = 0; s < 2 && e == hipSuccess; ++s) {
        e = hipEventCreateWithFlags(&c->packed[s], hipEventDisableTiming);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&c->sent[s], hipEventDisableTiming);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&c->unpacked[s], hipEventDisableTiming);
    }
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->xfer, hipEventDisableTiming);
    if (e == hipSuccess) e = hipMalloc(&c->scratch, 64 * sizeof(double));
    return map_hip(e);
}

void free_buffers(rt_comm c) {
    for (int s = 0; s < 2; ++s) {
        if (c->stage[s]) (void)hipFree(c->stage[s]);
        if (c->parts[s]) (void)hipFree(c->parts[s]);
        c->stage[s] = c->parts[s] = nullptr;
        c->sent_valid[s] = c->unpacked_valid[s] = false;
    }
    c->W = c->H = 0;
    c->root = -1;
}

void release(rt_comm c) {
    if (c->ctx) (void)hipSetDevice(c->ctx->device);
    if (c->cstream) (void)hipStreamSynchronize(c->cstream);
    if (c->ustream) (void)hipStreamSynchronize(c->ustream);
    free_buffers(c);
    for (int s = 0; s < 2; ++s)
        for (hipEvent_t ev : {c->packed[s], c->sent[s], c->unpacked[s]})
            if (ev) (void)hipEventDestroy(ev);
    if (c->xfer) (void)hipEventDestroy(c->xfer);
    if (c->scratch) (void)hipFree(c->scratch);
    if (c->nc) (void)ncclCommDestroy(c->nc);
    if (c->cstream) (void)hipStreamDestroy(c->cstream);
    if (c->ustream) (void)hipStreamDestroy(c->ustream);
    // the last communicator of the context gives its CUs back to the renders
    if (c->reserved && --c->ctx->reserve_refs == 0) (void)rti::reserve_cus(c->ctx, 0, nullptr);
    delete c;
}

// buffers and plans for a W x H gather (all earlier gathers of this comm have completed)
int ensure_plan(rt_comm c, unsigned W, unsigned H, int root) {
    if (c->W == W && c->H == H && c->root == root) return RT_SUCCESS;
    (void)hipStreamSynchronize(c->cstream);
    (void)hipStreamSynchronize(c->ustream);
    (void)hipStreamSynchronize(c->ctx->astream);
    free_buffers(c);
    c->plans.assign(c->nranks, {});
    size_t sb = 0;
    for (int q = 0; q < c->nranks; ++q) {
        rt_rect r[2];
        int n = 0;
        int rc = band_plan(W, H, (unsigned)c->nranks, (unsigned)q, r, 2, &n, &sb);
        if (rc) return rc;
        c->plans[q].assign(r, r + n);
    }
    c->stage_bytes = sb;
    hipError_t e = hipSuccess;
    for (int s = 0; s < 2 && e == hipSuccess; ++s) {
        e = hipMalloc(&c->stage[s], std::max<size_t>(sb, 16));
        if (e == hipSuccess && c->rank == root) e = hipMalloc(&c->parts[s], std::max<size_t>(sb * c->nranks, 16));
    }
    if (e != hipSuccess) {
        free_buffers(c);
        return map_hip(e);
    }
    c->W = W;
    c->H = H;
    c->root = root;
    return RT_SUCCESS;
}

// pack / unpack copies on the copy engines (hipMemcpyDeviceToDeviceNoCU) instead of blit kernels
#ifndef RT_COMM_NOCU
#define RT_COMM_NOCU 0
#endif
hipError_t copy_rects(const std::vector<rt_rect>& plan, uint8_t* img, uint8_t* stage, bool to_stage, hipStream_t s) {
    const hipMemcpyKind kind = RT_COMM_NOCU ? hipMemcpyDeviceToDeviceNoCU : hipMemcpyDeviceToDevice;
    for (const rt_rect& r : plan) {
        hipError_t e = to_stage
            ? hipMemcpy2DAsync(stage + r.stage_offset, r.width, img + r.img_offset, r.img_pitch, r.width, r.rows,
                               kind, s)
            : hipMemcpy2DAsync(img + r.img_offset, r.img_pitch, stage + r.stage_offset, r.width, r.width, r.rows,
                               kind, s);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

int rccl_transfer(const rt_comm* comms, int n_local, int root);
int loopback_transfer(const rt_comm* comms, int n_local, int root);
int finish_gather(const rt_comm* comms, int n_local, int root, rt_mem root_dst, const rt_mem* outs);
int check_loopback(const rt_comm* comms, int n_local);

}  // namespace

extern "C" {

int rtCommGetUniqueId(void* id) {
    if (!id) return RT_INVALID_VALUE;
    static_assert(sizeof(ncclUniqueId) == RT_COMM_ID_BYTES, "unique id size");
    ncclUniqueId u;
    int rc = map_nccl(ncclGetUniqueId(&u));
    if (rc) return rc;
    std::memcpy(id, &u, sizeof(u));
    return RT_SUCCESS;
}

int rtCommInitRank(rt_context ctx, int nranks, const void* id, int rank, rt_comm* out) {
    if (!out) return RT_INVALID_VALUE;
    *out = nullptr;
    if (!ctx) return RT_INVALID_CONTEXT;
    if (!id || nranks < 1 || rank < 0 || rank >= nranks) return RT_INVALID_VALUE;
    hipError_t he = hipSetDevice(ctx->device);
    if (he != hipSuccess) return map_hip(he);
    rt_comm c = new (std::nothrow) rt_comm_s();
    if (!c) return RT_OUT_OF_HOST_MEMORY;
    c->ctx = ctx;
    c->rank = rank;
    c->nranks = nranks;
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof(u));
    int rc = map_nccl(ncclCommInitRank(&c->nc, nranks, u, rank));
    if (!rc) rc = comm_streams(c, true);
    if (rc) {
        release(c);
        return rc;
    }
    *out = c;
    return RT_SUCCESS;
}

int rtCommInitAll(const rt_context* ctxs, int n, rt_comm* comms_out) {
    if (!ctxs || !comms_out || n < 1) return RT_INVALID_VALUE;
    std::vector<int> devs(n);
    for (int i = 0; i < n; ++i) {
        comms_out[i] = nullptr;
        if (!ctxs[i]) return RT_INVALID_CONTEXT;
        devs[i] = ctxs[i]->device;
    }
    std::vector<ncclComm_t> nc(n, nullptr);
    int rc = map_nccl(ncclCommInitAll(nc.data(), n, devs.data()));
    if (rc) return rc;
    for (int i = 0; i < n; ++i) {
        rt_comm c = new (std::nothrow) rt_comm_s();
        if (c) {
            c->ctx = ctxs[i];
            c->nc = nc[i];
            nc[i] = nullptr;
            c->rank = i;
            c->nranks = n;
            (void)hipSetDevice(ctxs[i]->device);
            rc = comm_streams(c, true);
        } else {
            (void)ncclCommDestroy(nc[i]);
            nc[i] = nullptr;
            rc = RT_OUT_OF_HOST_MEMORY;
        }
        if (rc) {
            if (c) release(c);
            for (int j = 0; j < i; ++j) {
                release(comms_out[j]);
                comms_out[j] = nullptr;
            }
            for (int j = i + 1; j < n; ++j)
                if (nc[j]) (void)ncclCommDestroy(nc[j]);
            return rc;
        }
        comms_out[i] = c;
    }
    return RT_SUCCESS;
}

int rtCommInitLoopback(const rt_context* ctxs, int n, rt_comm* comms_out) {
    // (check_loopback tracks the members of a call in a 64-bit mask)
    if (!ctxs || !comms_out || n < 1 || n > 64) return RT_INVALID_VALUE;
    for (int i = 0; i < n; ++i) {
        comms_out[i] = nullptr;
        if (!ctxs[i]) return RT_INVALID_CONTEXT;
    }
    static std::atomic<uintptr_t> next_group{1};
    const void* group = reinterpret_cast<const void*>(next_group.fetch_add(1));
    for (int i = 0; i < n; ++i) {
        rt_comm c = new (std::nothrow) rt_comm_s();
        int rc = RT_OUT_OF_HOST_MEMORY;
        if (c) {
            c->ctx = ctxs[i];
            c->group = group;
            c->rank = i;
            c->nranks = n;
            hipError_t e = hipSetDevice(ctxs[i]->device);
            rc = e == hipSuccess ? comm_streams(c, false) : map_hip(e);
        }
        if (rc) {
            if (c) release(c);
            for (int j = 0; j < i; ++j) {
                release(comms_out[j]);
                comms_out[j] = nullptr;
            }
            return rc;
        }
        comms_out[i] = c;
    }
    return RT_SUCCESS;
}

int rtCommDestroy(rt_comm c) {
    if (!c) return RT_INVALID_VALUE;
    (void)hipSetDevice(c->ctx->device);
    (void)hipStreamSynchronize(qs(c->ctx));
    release(c);
    return RT_SUCCESS;
}

int rtCommGetRank(rt_comm c, int* rank, int* nranks) {
    if (!c) return RT_INVALID_VALUE;
    if (rank) *rank = c->rank;
    if (nranks) *nranks = c->nranks;
    return RT_SUCCESS;
}

int rtCommShardKernel(rt_comm c, rt_kernel k) {
    if (!c) return RT_INVALID_VALUE;
    return rti::shard_kernel(k, (unsigned)c->nranks, (unsigned)c->rank);
}

int rtCommEnqueueGatherBands(const rt_comm* comms, const rt_mem* outs, int n_local, unsigned W, unsigned H,
                             int root, rt_mem root_dst) {
    if (!comms || !outs || n_local < 1 || W == 0 || H == 0) return RT_INVALID_VALUE;
    const uint64_t img_bytes = (uint64_t)W * H * kPixelBytes;
    for (int i = 0; i < n_local; ++i) {
        rt_comm c = comms[i];
        if (!c || !outs[i]) return RT_INVALID_VALUE;
        if (root < 0 || root >= c->nranks) return RT_INVALID_VALUE;
        if (outs[i]->ctx != c->ctx || outs[i]->size < img_bytes) return RT_INVALID_MEM_OBJECT;
        if (c->rank == root && root_dst && (root_dst->ctx != c->ctx || root_dst->size < img_bytes))
            return RT_INVALID_MEM_OBJECT;
    }
    if (int rc = check_loopback(comms, n_local)) return rc;
    // phase 1: every rank (the root too) packs its bands on its context's accumulation stream
    for (int i = 0; i < n_local; ++i) {
        rt_comm c = comms[i];
        rt_context ctx = c->ctx;
        hipError_t e = hipSetDevice(ctx->device);
        if (e != hipSuccess) return map_hip(e);
        int rc = ensure_plan(c, W, H, root);
        if (rc) return rc;
        const int s = c->slot;
        uint8_t* out = static_cast<uint8_t*>(outs[i]->dptr);
        // the bands are final after every accumulation enqueued so far (astream, in order) and
        // after whatever the main stream has queued (per-frame launches write `out` there)
        e = rti::main_tail_wait(ctx, ctx->astream);
        if (e == hipSuccess && c->sent_valid[s]) e = hipStreamWaitEvent(ctx->astream, c->sent[s], 0);  // slot free
        if (e == hipSuccess)
            e = copy_rects(c->plans[c->rank], out, static_cast<uint8_t*>(c->stage[s]), true, ctx->astream);
        if (e == hipSuccess) e = hipEventRecord(c->packed[s], ctx->astream);
        if (e == hipSuccess) e = hipStreamWaitEvent(c->cstream, c->packed[s], 0);
        if (e == hipSuccess && c->rank == root && c->unpacked_valid[s])
            e = hipStreamWaitEvent(c->cstream, c->unpacked[s], 0);  // receive slot's last unpack done
        if (e == hipSuccess) e = hipEventRecord(ctx->atail, ctx->astream);
        if (e != hipSuccess) return map_hip(e);
        ctx->apending = true;
    }
    // phase 2: the transfers, one group over every local rank (required when one thread drives
    // several GPUs).  The root posts one receive per rank, so all its links carry data at once;
    // its own bands take the same path (a send to itself, a device-local copy) -- one uniform
    // unpack, and a world of one still runs the whole RCCL flow.
    if (comms[0]->group) {
        int rc = loopback_transfer(comms, n_local, root);
        if (rc) return rc;
    } else {
        int rc = rccl_transfer(comms, n_local, root);
        if (rc) return rc;
    }
    return finish_gather(comms, n_local, root, root_dst, outs);
}

}  // extern "C"

namespace {

int rccl_transfer(const rt_comm* comms, int n_local, int root) {
    int rc = map_nccl(ncclGroupStart());
    if (rc) return rc;
    for (int i = 0; i < n_local && rc == RT_SUCCESS; ++i) {
        rt_comm c = comms[i];
        const int s = c->slot;
        rc = map_nccl(ncclSend(c->stage[s], c->stage_bytes, ncclInt8, root, c->nc, c->cstream));
        if (c->rank == root)
            for (int q = 0; q < c->nranks && rc == RT_SUCCESS; ++q)
                rc = map_nccl(ncclRecv(static_cast<uint8_t*>(c->parts[s]) + (size_t)q * c->stage_bytes,
                                       c->stage_bytes, ncclInt8, q, c->nc, c->cstream));
    }
    const int rc_end = map_nccl(ncclGroupEnd());
    if (rc) return rc;
    return rc_end;
}

// loopback world: the root's communicator stream copies every rank's staging slot into its
// receive slots (after each rank's pack), then every rank's communicator stream waits for those
// copies -- the same stream and event chain as the RCCL send/receive above.
int loopback_transfer(const rt_comm* comms, int n_local, int root) {
    rt_comm R = nullptr;
    for (int i = 0; i < n_local; ++i)
        if (comms[i]->rank == root) R = comms[i];
    hipError_t e = hipSetDevice(R->ctx->device);
    for (int i = 0; i < n_local && e == hipSuccess; ++i) {
        rt_comm c = comms[i];
        e = hipStreamWaitEvent(R->cstream, c->packed[c->slot], 0);
        if (e == hipSuccess)
            e = hipMemcpyAsync(static_cast<uint8_t*>(R->parts[R->slot]) + (size_t)c->rank * R->stage_bytes,
                               c->stage[c->slot], c->stage_bytes, hipMemcpyDeviceToDevice, R->cstream);
    }
    if (e == hipSuccess) e = hipEventRecord(R->xfer, R->cstream);
    for (int i = 0; i < n_local && e == hipSuccess; ++i) {
        rt_comm c = comms[i];
        if (c == R) continue;
        e = hipSetDevice(c->ctx->device);
        if (e == hipSuccess) e = hipStreamWaitEvent(c->cstream, R->xfer, 0);
    }
    return map_hip(e);
}

// phase 3: the root unpacks every rank's bands into the destination
int finish_gather(const rt_comm* comms, int n_local, int root, rt_mem root_dst, const rt_mem* outs) {
    for (int i = 0; i < n_local; ++i) {
        rt_comm c = comms[i];
        rt_context ctx = c->ctx;
        const int s = c->slot;
        hipError_t e = hipSetDevice(ctx->device);
        if (e == hipSuccess) e = hipEventRecord(c->sent[s], c->cstream);
        if (e != hipSuccess) return map_hip(e);
        c->sent_valid[s] = true;
        if (c->rank == root) {
            // Gathering into the root's own output: its own bands are in place already and are
            // not unpacked, so the unpack writes only other ranks' rows, which no later render,
            // accumulation or pack of this context touches -- nothing on the context waits for
            // it.  (An unpack that the next accumulation had to wait for chained that
            // accumulation, and the render after it, to the transfer: RCCL's kernel gets CUs only
            // as a persistent render drains, so every second render started a step late --
            // world-1 0.90 vs 0.77 ms/frame, profiles/r04/dist_streams.txt.)  Reads of the
            // image wait for it through the context's queue (gtail, qs()).
            const bool into_out = !root_dst || root_dst == outs[i];
            uint8_t* dst = static_cast<uint8_t*>((root_dst ? root_dst : outs[i])->dptr);
            e = hipStreamWaitEvent(c->ustream, c->sent[s], 0);
            for (int q = 0; q < c->nranks && e == hipSuccess; ++q)
                if (!(into_out && q == c->rank))
                    e = copy_rects(c->plans[q], dst, static_cast<uint8_t*>(c->parts[s]) + (size_t)q * c->stage_bytes,
                                   false, c->ustream);
            if (e == hipSuccess) e = hipEventRecord(c->unpacked[s], c->ustream);
            if (e != hipSuccess) return map_hip(e);
            c->unpacked_valid[s] = true;
        }
        e = hipEventRecord(ctx->gtail, c->rank == root ? c->ustream : c->cstream);
        if (e != hipSuccess) return map_hip(e);
        ctx->gpending = true;
        c->slot ^= 1;
    }
    return RT_SUCCESS;
}

// a loopback world's calls must name all its members, each once
int check_loopback(const rt_comm* comms, int n_local) {
    const void* g = comms[0]->group;
    if (!g) {
        for (int i = 1; i < n_local; ++i)
            if (comms[i]->group) return RT_INVALID_VALUE;
        return RT_SUCCESS;
    }
    if (n_local != comms[0]->nranks) return RT_INVALID_VALUE;
    uint64_t seen = 0;
    for (int i = 0; i < n_local; ++i) {
        if (comms[i]->group != g || comms[i]->rank >= 64) return RT_INVALID_VALUE;
        const uint64_t bit = 1ull << comms[i]->rank;
        if (seen & bit) return RT_INVALID_VALUE;
        seen |= bit;
    }
    return RT_SUCCESS;
}

}  // namespace

extern "C" {

int rtCommAllReduceF64(const rt_comm* comms, int n_local, double* values, int count, int op) {
    if (!comms || n_local < 1 || !values || count < 1 || count > 64) return RT_INVALID_VALUE;
    if (op != RT_COMM_SUM && op != RT_COMM_MAX) return RT_INVALID_VALUE;
    for (int i = 0; i < n_local; ++i)
        if (!comms[i]) return RT_INVALID_VALUE;
    if (int rc = check_loopback(comms, n_local)) return rc;
    if (comms[0]->group) {
        // loopback world: every member is here, so the reduction is over these rows, after the
        // members' communicator streams (earlier gathers) have drained, as RCCL's would
        for (int i = 0; i < n_local; ++i) {
            hipError_t e = hipSetDevice(comms[i]->ctx->device);
            if (e == hipSuccess) e = hipStreamSynchronize(comms[i]->cstream);
            if (e != hipSuccess) return map_hip(e);
        }
        for (int j = 0; j < count; ++j) {
            double acc = values[j];
            for (int i = 1; i < n_local; ++i) {
                const double v = values[(size_t)i * count + j];
                acc = op == RT_COMM_SUM ? acc + v : std::max(acc, v);
            }
            for (int i = 0; i < n_local; ++i) values[(size_t)i * count + j] = acc;
        }
        return RT_SUCCESS;
    }
    for (int i = 0; i < n_local; ++i) {
        hipError_t e = hipSetDevice(comms[i]->ctx->device);
        if (e == hipSuccess)
            e = hipMemcpyAsync(comms[i]->scratch, values + (size_t)i * count, count * sizeof(double),
                               hipMemcpyHostToDevice, comms[i]->cstream);
        if (e != hipSuccess) return map_hip(e);
    }
    int rc = map_nccl(ncclGroupStart());
    if (rc) return rc;
    for (int i = 0; i < n_local && rc == RT_SUCCESS; ++i)
        rc = map_nccl(ncclAllReduce(comms[i]->scratch, comms[i]->scratch, count, ncclFloat64,
                                    op == RT_COMM_SUM ? ncclSum : ncclMax, comms[i]->nc, comms[i]->cstream));
    const int rc_end = map_nccl(ncclGroupEnd());
    if (rc) return rc;
    if (rc_end) return rc_end;
    for (int i = 0; i < n_local; ++i) {
        hipError_t e = hipSetDevice(comms[i]->ctx->device);
        if (e == hipSuccess)
            e = hipMemcpyAsync(values + (size_t)i * count, comms[i]->scratch, count * sizeof(double),
                               hipMemcpyDeviceToHost, comms[i]->cstream);
        if (e == hipSuccess) e = hipStreamSynchronize(comms[i]->cstream);
        if (e != hipSuccess) return map_hip(e);
    }
    return RT_SUCCESS;
}

int rtCommBarrier(const rt_comm* comms, int n_local) {
    if (!comms || n_local < 1) return RT_INVALID_VALUE;
    std::vector<double> v((size_t)n_local, 0.0);
    return rtCommAllReduceF64(comms, n_local, v.data(), 1, RT_COMM_SUM);
}

int rtBandPackPlan(unsigned width, unsigned height, unsigned period, unsigned phase, rt_rect* rects, int capacity,
                   int* n_rects, size_t* staging_bytes) {
    return band_plan(width, height, period, phase, rects, capacity, n_rects, staging_bytes);
}

}  // extern "C"
