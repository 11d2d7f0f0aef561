// rt_comm.cpp -- multi-GPU band sharding + gather, behind include/rt_hip.h.
//
// The reference is single-device (CLRaytracer.cpp:104-120, one in-order queue CLutils.cpp:29).
// A frame shards with no exchange until the image is needed, because every pixel's seed is
// gid + HashUInt32(frameCount) over the GLOBAL work-item id (kernel_bvh.cl:445) and the gamma
// accumulation is per pixel (:449-455).  Rank r renders the interleaved 8-row bands
// b % nranks == r into its full-size output buffer (rtKernelSetRowInterleave), at the rows they
// occupy in the image; the gather moves them to the root.
//
// Copy-engine transport (default): nothing in a gather's steady state needs a compute unit.  A
// persistent render holds every CU slot until it drains, and anything that needs one -- RCCL's
// transfer kernel, the runtime's 2-D blit copies, and ROCclr's hipStreamWriteValue64 /
// hipStreamWaitValue64, which run as kernels (__amd_rocclr_streamOps*) -- waits behind it and then
// crawls beside it (profiles/r04/dist_flow_ab.txt, profiles/r05/flag_probe.txt).  So the bytes AND
// the flags move on the copy engines (SDMA, hipMemcpyDeviceToDeviceNoCU; over xGMI between GPUs):
//
//   rank q accumulation stream : [accumulate k] [pack k -> stage[s] (SDMA, per band)] [accumulate k+1]
//   rank q comm stream         :     (packed k)(release k-1) [bands -> root image (SDMA)] [arrive k (SDMA)]
//   root unpack stream         : (root's queue so far) [release k-1 -> every rank (SDMA)]
//   root, first read of image k: (wait arrive k from every rank)
//
// * The pack copies the rank's bands densely into one of two staging slots right after the
//   accumulation, on the accumulation stream: the next accumulation never waits for anything
//   across GPUs.  The transfer writes every band from the slot into the rows it occupies in the
//   root's destination -- mapped into the rank by IPC handle (one ncclAllGather per plan), or by
//   address for ranks driven by one process: no receive slot, no unpack.
// * `release k-1` (a flag in each rank's memory, written by the root's copy engine once everything
//   its context queued before gather k -- reads of image k-1 -- has run): a rank's copies never
//   change the root's image under a read.  The rank's wait for it is the one waiting kernel of a
//   gather, and it gates only the transfer.
// * `arrive k` (a flag per rank in the root's memory, written by the rank's copy engine after its
//   bands): the root joins the arrivals only when it next reads (rti::join_gather, from qs): no
//   kernel spins on the root while nobody looks at the image.
// * The root gathering into another buffer copies its own bands straight from its output (local
//   copies, ordered by events); gathering into its output, they are in place.
// * Flag values are copied from a device array holding 0, 1, 2, ... (vals); a plan is rebuilt
//   before the gather count reaches its end (every rank at the same gather).
//
// RCCL transport (RT_COMM_TRANSPORT_RCCL, and the fallback of a world whose copy-engine links do
// not hold): each rank packs its bands densely into a staging slot on its accumulation stream,
// grouped ncclSend/ncclRecv move the slots to the root, the root unpacks them; two slots alternate
// so step k's transfer runs under step k+1's render.  RCCL also carries the setup exchanges,
// reductions and barriers.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <cerrno>
#include <unistd.h>
#include <string>
#include <thread>
#include <memory>
#include <new>
#include <utility>
#include <vector>

#include "../../include/rt_hip.h"
#include "rt_internal.hpp"

using rti::map_hip;
using rti::qs;

namespace {

constexpr unsigned kBandRows = 8;     // = the 8x8 tile height of the persistent schedules
constexpr size_t kPixelBytes = 16;    // one float3 slot of the output buffer
constexpr size_t kProbeBytes = 4096;  // per rank, the trial round's copy
// flag values 0 .. kFlagValues - 1 (512 KB per rank): the world re-plans, collectively, every
// kFlagValues - 2 gathers (ensure_plan), a few milliseconds once per 65k steps
constexpr uint64_t kFlagValues = 1ull << 16;

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

// The byte runs of the image one rank's bands occupy (adjacent bands merged: one run for a world of
// one), in image order.
std::vector<std::pair<uint64_t, uint64_t>> band_runs(const std::vector<rt_rect>& plan) {
    std::vector<std::pair<uint64_t, uint64_t>> runs;
    for (const rt_rect& r : plan)
        for (uint64_t i = 0; i < r.rows; ++i) {
            const uint64_t off = r.img_offset + i * r.img_pitch;
            if (!runs.empty() && runs.back().first + runs.back().second == off)
                runs.back().second += r.width;
            else
                runs.emplace_back(off, r.width);
        }
    return runs;
}

}  // namespace

struct rt_comm_s {
    rt_context ctx = nullptr;
    ncclComm_t nc = nullptr;
    // loopback worlds (rtCommInitLoopback): no RCCL; `group` identifies the world (shared by its
    // members), whose gathers always run on the copy engines with the members linked by address
    const void* group = nullptr;
    int rank = 0, nranks = 1;
    hipStream_t cstream = nullptr;  // transfers (copy engines or RCCL), RCCL setup and reductions
    hipStream_t ustream = nullptr;  // root: releases (copy engines), unpack (RCCL)
    // the plan: one (width, height, root, destination); rebuilt when any changes
    unsigned W = 0, H = 0;
    int root = -1;
    std::vector<std::vector<rt_rect>> plans;  // per rank: its bands as 2-D rects (rtBandPackPlan)
    int transport = RT_COMM_TRANSPORT_COPY_ENGINES;  // requested (rtCommSetTransport)
    bool ce = false;                 // this plan moves bytes on the copy engines
    bool ipc_linked = false;         // ... with its links exchanged as IPC handles (link_ipc)
    int fallback_reason = RT_COMM_FALLBACK_NONE;  // the plan wanted the copy engines and runs RCCL
    bool fail_links = false;         // test hook (RT_COMM_OPT_FAIL_LINKS)
    uint64_t replan_after = kFlagValues - 2;  // gathers per plan (RT_COMM_OPT_REPLAN_PERIOD)
    // root: other devices' copy engines write its destination, so its first read of a gathered
    // image runs a system-scope acquire on every XCD first (join_gather; RT_COMM_OPT_SYSTEM_ACQUIRE
    // forces it on one device)
    bool remote_writers = false;
    bool force_acquire = false;
    uint64_t seq = 0;                // gathers enqueued with this plan (1, 2, ...)
    // ---- copy engines ----
    rt_mem target = nullptr;         // root: the plan's destination (pinned)
    uint8_t* peer_target = nullptr;  // the root's destination as this rank addresses it
    std::vector<std::pair<uint64_t, uint64_t>> runs;  // this rank's band runs (image byte offset, bytes)
    bool sends = false;              // this rank copies its bands (all but a root gathering into its out)
    uint64_t* sflags = nullptr;      // [1] (fine-grained, this rank's memory): image released by the root, seq
    uint64_t* rflags = nullptr;      // root, [nranks] (fine-grained): rank q's bands of image seq in place
    uint8_t* probe = nullptr;        // root, [nranks][kProbeBytes] (fine-grained): the trial round's copies
    uint8_t* peer_probe = nullptr;
    uint64_t* peer_rflags = nullptr; // the root's arrival flags, as this rank addresses them
    std::vector<uint64_t*> peer_sflags;  // root: every rank's release flag
    std::vector<void*> ipc_opened;       // IPC mappings to close with the plan
    uint64_t* vals = nullptr;        // device: vals[i] = i, the sources of the flag copies (kFlagValues)
    uint64_t join_seq = 0;           // root, IPC links: the gather whose arrivals the next read joins
    std::vector<hipEvent_t> join_events;  // root, one process: the ranks' `sent` events of that gather
    // one-process worlds (rtCommInitLoopback, rtCommInitAll): the members still alive -- a member
    // released before its root joined takes its events out of the root's join (it has drained)
    std::shared_ptr<std::vector<rt_comm>> members;
    hipEvent_t ready = nullptr;      // the root's bands of `out` are final (accumulation stream)
    hipEvent_t dsent = nullptr;      // the root's own copies (gathering into another buffer) are done
    hipEvent_t released = nullptr;   // root: the previous image is released (unpack stream)
    hipEvent_t xt0 = nullptr, xt1 = nullptr;  // timing: the last gather's transfer on cstream
    bool xt_valid = false;
    // the copies split over streams of their own, which the runtime spreads over several SDMA
    // engines (one engine: 61 GB/s; 2 streams 120, 8 streams 154 GB/s on MI355X,
    // scripts/probes/gather_engines_probe.hip split, profiles/r04/gather_engines_probe.txt).
    // Every stream shares the 4 hardware queues, though: in the world-1 flow 2 streams beat 1
    // (0.790 vs 0.798 ms/frame) and 8 stalled the renders (1.17; profiles/r04/dist_flow_ab.txt)
    hipStream_t xstream[8] = {};
    hipEvent_t xgo = nullptr, xdone[8] = {};
    // ---- staging: ranks sending to another rank's root (copy engines); every rank (RCCL) ----
    size_t stage_bytes = 0;
    void* stage[2] = {};                      // this rank's packed bands
    void* parts[2] = {};                      // RCCL root: nranks x stage_bytes received bands
    hipEvent_t packed[2] = {}, sent[2] = {}, unpacked[2] = {};
    bool sent_valid[2] = {}, unpacked_valid[2] = {};
    int slot = 0;
    double* scratch = nullptr;  // reductions
    // shared worlds (rtCommInitShared): no RCCL; setup exchanges, reductions and barriers go
    // through files in `fdir` (exchange number fseq), the gathers over the copy engines
    std::string fdir;
    uint64_t fseq = 0;
    uint64_t fnonce = 0;  // the world's id (rank 0's, from fdir/world): part of every exchange file name
};

namespace {

// a shared world's exchange file: x<world>_<exchange>_r<rank>
std::string xname(const rt_comm c, uint64_t seq, int q) {
    char w[17];
    std::snprintf(w, sizeof(w), "%016llx", (unsigned long long)c->fnonce);
    return c->fdir + "/x" + w + "_" + std::to_string(seq) + "_r" + std::to_string(q);
}

// A shared world's id.  Rank 0 publishes it in fdir/world (written aside, then linked into place:
// a directory that already holds one -- an earlier world's -- is refused); the other ranks wait up
// to a minute for it.  Exchange files carry it, so files an earlier world left are never read.
int shared_world_id(rt_comm c) {
    const std::string path = c->fdir + "/world";
    if (c->rank == 0) {
        uint64_t id = (uint64_t)std::chrono::steady_clock::now().time_since_epoch().count() * 0x9e3779b97f4a7c15ull ^
                      (uint64_t)getpid() << 32;
        if (id == 0) id = 1;
        const std::string tmp = path + ".tmp" + std::to_string(getpid());
        std::FILE* f = std::fopen(tmp.c_str(), "wb");
        if (!f) return RT_FILE_NOT_FOUND;
        const bool ok = std::fwrite(&id, sizeof(id), 1, f) == 1;
        if (std::fclose(f) != 0 || !ok) {
            (void)std::remove(tmp.c_str());
            return RT_OUT_OF_RESOURCES;
        }
        const int linked = link(tmp.c_str(), path.c_str());
        (void)std::remove(tmp.c_str());
        if (linked != 0) return errno == EEXIST ? RT_INVALID_VALUE : RT_OUT_OF_RESOURCES;
        c->fnonce = id;
        return RT_SUCCESS;
    }
    const auto deadline = std::chrono::steady_clock::now() + std::chrono::seconds(60);
    for (;;) {
        if (std::FILE* f = std::fopen(path.c_str(), "rb")) {
            uint64_t id = 0;
            const bool ok = std::fread(&id, sizeof(id), 1, f) == 1;
            std::fclose(f);
            if (ok && id != 0) {
                c->fnonce = id;
                return RT_SUCCESS;
            }
        }
        if (std::chrono::steady_clock::now() > deadline) return RT_OUT_OF_RESOURCES;
        std::this_thread::sleep_for(std::chrono::milliseconds(1));
    }
}

// The communicator's streams (transfer, root, and the extra transfer streams) run at the device's
// greatest stream priority.  Read off a kernel trace of the world-1 flow
// (profiles/r04/dist_flow_ab.txt): HIP maps streams onto a few hardware queues (GPU_MAX_HW_QUEUES
// 4); at normal priority the communicator's streams shared the main stream's and a render stream's
// queue, so the next fused render sat behind the previous step's gather.  High-priority streams
// get queues of their own.  (Reserving CUs per XCD for RCCL's transfer kernel let it run at once
// but cost the renders more than it saved -- 0.85 vs 0.82 ms/frame in the same flow; removed in
// round 5.)
int comm_events(rt_comm c, hipError_t e);
int comm_streams(rt_comm c) {
    int least = 0, greatest = 0;
    hipError_t e = hipDeviceGetStreamPriorityRange(&least, &greatest);
    if (e == hipSuccess) e = hipStreamCreateWithPriority(&c->cstream, hipStreamNonBlocking, greatest);
    if (e == hipSuccess) e = hipStreamCreateWithPriority(&c->ustream, hipStreamNonBlocking, greatest);
    return comm_events(c, e);
}

#ifndef RT_COMM_XFER_STREAMS
#define RT_COMM_XFER_STREAMS 2  // 1: the copies on the communicator stream itself
#endif
static_assert(RT_COMM_XFER_STREAMS >= 1 && RT_COMM_XFER_STREAMS <= 8, "copy streams");
int comm_events(rt_comm c, hipError_t e) {
    int least = 0, greatest = 0;
    if (e == hipSuccess) e = hipDeviceGetStreamPriorityRange(&least, &greatest);
    for (int i = 0; RT_COMM_XFER_STREAMS > 1 && i < RT_COMM_XFER_STREAMS && e == hipSuccess; ++i) {
        e = hipStreamCreateWithPriority(&c->xstream[i], hipStreamNonBlocking, greatest);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&c->xdone[i], hipEventDisableTiming);
    }
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->xgo, hipEventDisableTiming);
    for (hipEvent_t* ev : {&c->ready, &c->dsent, &c->released})
        if (e == hipSuccess) e = hipEventCreateWithFlags(ev, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreate(&c->xt0);
    if (e == hipSuccess) e = hipEventCreate(&c->xt1);
    for (int s = 0; s < 2 && e == hipSuccess; ++s) {
        e = hipEventCreateWithFlags(&c->packed[s], hipEventDisableTiming);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&c->sent[s], hipEventDisableTiming);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&c->unpacked[s], hipEventDisableTiming);
    }
    if (e == hipSuccess) e = hipMalloc(&c->scratch, 64 * sizeof(double));
    return map_hip(e);
}

// staging slots (a rank sending to another rank's root; every rank of an RCCL plan) and, for an
// RCCL root, its receive slots
int stage_buffers(rt_comm c, bool rccl) {
    hipError_t e = hipSuccess;
    for (int s = 0; s < 2 && e == hipSuccess; ++s) {
        if (!c->stage[s]) e = hipMalloc(&c->stage[s], std::max<size_t>(c->stage_bytes, 16));
        if (e == hipSuccess && rccl && c->rank == c->root && !c->parts[s])
            e = hipMalloc(&c->parts[s], std::max<size_t>(c->stage_bytes * c->nranks, 16));
    }
    return map_hip(e);
}
int rccl_buffers(rt_comm c) { return stage_buffers(c, true); }

// the flag values' source array, once per communicator
int flag_values(rt_comm c) {
    if (c->vals) return RT_SUCCESS;
    std::vector<uint64_t> v;
    try {
        v.resize(kFlagValues);
    } catch (const std::bad_alloc&) {
        return RT_OUT_OF_HOST_MEMORY;
    }
    for (uint64_t i = 0; i < kFlagValues; ++i) v[i] = i;
    hipError_t e = hipMalloc(reinterpret_cast<void**>(&c->vals), kFlagValues * sizeof(uint64_t));
    if (e == hipSuccess) e = hipMemcpy(c->vals, v.data(), kFlagValues * sizeof(uint64_t), hipMemcpyHostToDevice);
    if (e != hipSuccess && c->vals) {
        (void)hipFree(c->vals);
        c->vals = nullptr;
    }
    return map_hip(e);
}

// A system-scope acquire on the CU each workgroup runs on: its L1 and its XCD's L2 drop what they
// cached of memory that another device may have written (buffer_inv sc0 sc1 on gfx950).  One
// workgroup per CU: the dispatcher deals workgroups round-robin over the 8 XCDs, so every XCD's L2
// sees at least one (the kernel itself reads and writes nothing).
__global__ void system_acquire_kernel() {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the invalidate has completed when the wave ends
}

// a flag word (another device's, or this one's) := v, on the copy engine of stream s
hipError_t flag_copy(rt_comm c, uint64_t* dst, uint64_t v, hipStream_t s) {
    return hipMemcpyAsync(dst, c->vals + v, sizeof(uint64_t), hipMemcpyDeviceToDeviceNoCU, s);
}

void free_buffers(rt_comm c) {
    for (void* p : c->ipc_opened) (void)hipIpcCloseMemHandle(p);
    c->ipc_opened.clear();
    for (int s = 0; s < 2; ++s) {
        if (c->stage[s]) (void)hipFree(c->stage[s]);
        if (c->parts[s]) (void)hipFree(c->parts[s]);
        c->stage[s] = c->parts[s] = nullptr;
        c->sent_valid[s] = c->unpacked_valid[s] = false;
    }
    for (uint64_t** f : {&c->sflags, &c->rflags})
        if (*f) (void)hipFree(*f);
    if (c->probe) (void)hipFree(c->probe);
    c->sflags = c->rflags = c->peer_rflags = nullptr;
    c->probe = c->peer_probe = c->peer_target = nullptr;
    c->peer_sflags.clear();
    if (c->target) rti::unpin(c->target);
    c->target = nullptr;
    c->runs.clear();
    c->ce = c->ipc_linked = c->sends = c->remote_writers = false;
    c->fallback_reason = RT_COMM_FALLBACK_NONE;
    c->seq = c->join_seq = 0;
    c->xt_valid = false;
    c->slot = 0;
    c->W = c->H = 0;
    c->root = -1;
    if (c->ctx->oread_ev == c->dsent) c->ctx->oread = false;
    if (c->ctx->gjoin == c) c->ctx->gjoin = nullptr;
}

void release(rt_comm c) {
    if (c->ctx) (void)hipSetDevice(c->ctx->device);
    for (hipStream_t s : {c->cstream, c->ustream})
        if (s) (void)hipStreamSynchronize(s);
    for (hipStream_t s : c->xstream)
        if (s) (void)hipStreamSynchronize(s);
    if (c->members) {  // (its transfers have drained: nobody needs to wait for its events)
        auto& m = *c->members;
        m.erase(std::remove(m.begin(), m.end(), c), m.end());
        for (rt_comm o : m)
            o->join_events.erase(std::remove_if(o->join_events.begin(), o->join_events.end(),
                                                [&](hipEvent_t ev) { return ev == c->sent[0] || ev == c->sent[1]; }),
                                 o->join_events.end());
    }
    free_buffers(c);
    if (c->ctx->oread_ev == c->dsent) c->ctx->oread_ev = nullptr;
    for (int s = 0; s < 2; ++s)
        for (hipEvent_t ev : {c->packed[s], c->sent[s], c->unpacked[s]})
            if (ev) (void)hipEventDestroy(ev);
    for (hipEvent_t ev : {c->ready, c->dsent, c->released, c->xt0, c->xt1, c->xgo})
        if (ev) (void)hipEventDestroy(ev);
    for (int i = 0; i < 8; ++i) {
        if (c->xstream[i]) (void)hipStreamDestroy(c->xstream[i]);
        if (c->xdone[i]) (void)hipEventDestroy(c->xdone[i]);
    }
    if (c->vals) (void)hipFree(c->vals);
    if (c->scratch) (void)hipFree(c->scratch);
    if (c->nc) (void)ncclCommDestroy(c->nc);
    if (c->cstream) (void)hipStreamDestroy(c->cstream);
    if (c->ustream) (void)hipStreamDestroy(c->ustream);
    // a shared world's rank removes its own exchange files but the last: every rank wrote its file
    // of exchange k only after reading all files of exchange k - 1, so those have all been read;
    // the last one may still be awaited by a slower rank (the caller removes the directory)
    for (uint64_t q = 1; !c->fdir.empty() && q < c->fseq; ++q)
        (void)std::remove(xname(c, q, c->rank).c_str());
    delete c;
}

// Every stream of the communicator (and the context's accumulation stream, whose accumulations
// a gather may follow) idle: a plan can be torn down.
void quiesce(rt_comm c) {
    for (hipStream_t s : {c->cstream, c->ustream, c->ctx->astream})
        (void)hipStreamSynchronize(s);
    for (hipStream_t s : c->xstream)
        if (s) (void)hipStreamSynchronize(s);
}

// The plan of a W x H gather into `dst` (the root's destination; ranks other than the root pass
// nullptr) from `out` -- all earlier gathers of this comm have completed when it is rebuilt.  A
// copy-engine plan writes into the destination it was linked to, so a new one rebuilds it (the
// RCCL transport unpacks into whatever the call names); so does a gather count about to run past
// the flag values (every rank of the world at the same gather).
int ensure_plan(rt_comm c, unsigned W, unsigned H, int root, rt_mem dst, rt_mem out, bool* built) {
    *built = false;
    if (c->W == W && c->H == H && c->root == root && (c->rank != root || !c->ce || dst == c->target) &&
        c->seq < c->replan_after)
        return RT_SUCCESS;
    *built = true;
    quiesce(c);
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
    c->W = W;
    c->H = H;
    c->root = root;
    if (c->rank == root) {
        c->target = dst;
        rti::pin(dst);
    }
    // the root gathering into its own output has its bands in place already
    c->sends = c->rank != root || dst != out;
    if (c->transport == RT_COMM_TRANSPORT_RCCL) return rccl_buffers(c);
    // copy engines: the release and arrival flags and the probe are fine-grained memory (written
    // by other devices' engines, read coherently by the waits and the host), each its own
    // allocation (an IPC handle maps a whole allocation)
    c->runs = band_runs(c->plans[c->rank]);
    if (c->rank != root) {
        const int rc = stage_buffers(c, false);
        if (rc) return rc;
    }
    hipError_t e = hipExtMallocWithFlags(reinterpret_cast<void**>(&c->sflags), sizeof(uint64_t), hipDeviceMallocFinegrained);
    if (e == hipSuccess && c->rank == root)
        e = hipExtMallocWithFlags(reinterpret_cast<void**>(&c->rflags), sizeof(uint64_t) * c->nranks,
                                  hipDeviceMallocFinegrained);
    if (e == hipSuccess && c->rank == root)
        e = hipExtMallocWithFlags(reinterpret_cast<void**>(&c->probe), kProbeBytes * c->nranks, hipDeviceMallocFinegrained);
    if (e == hipSuccess) e = hipMemset(c->sflags, 0, sizeof(uint64_t));
    if (e == hipSuccess && c->rflags) e = hipMemset(c->rflags, 0, sizeof(uint64_t) * c->nranks);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    return map_hip(e);
}

// Copy-engine links of a plan whose members are all in this call (loopback worlds, and RCCL
// worlds driven by one process): the root's destination by address, the steps ordered by events.
// Between devices the copy engines reach peer memory once peer access is on.
int link_direct(const rt_comm* comms, int n_local, int root) {
    rt_comm R = nullptr;
    for (int i = 0; i < n_local; ++i)
        if (comms[i]->rank == root) R = comms[i];
    if (!R) return RT_INVALID_VALUE;
    for (int i = 0; i < n_local; ++i) {
        rt_comm c = comms[i];
        if (c->ctx->device != R->ctx->device) {
            int can = 0;
            hipError_t e = hipDeviceCanAccessPeer(&can, c->ctx->device, R->ctx->device);
            if (e != hipSuccess || !can) return RT_INVALID_OPERATION;
            for (auto [a, b] : {std::pair<int, int>{c->ctx->device, R->ctx->device}, {R->ctx->device, c->ctx->device}}) {
                (void)hipSetDevice(a);
                e = hipDeviceEnablePeerAccess(b, 0);
                if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) return map_hip(e);
                (void)hipGetLastError();
            }
        }
    }
    for (int i = 0; i < n_local; ++i) {
        comms[i]->peer_target = static_cast<uint8_t*>(R->target->dptr);
        comms[i]->ce = true;
        if (comms[i]->ctx->device != R->ctx->device) R->remote_writers = true;
    }
    return RT_SUCCESS;
}

// The same links across processes: every rank publishes IPC handles of its allocations (the
// root: destination, arrival flags and probe; everyone: release flag) with one ncclAllGather, maps
// the ones it needs, and the world agrees (ncclAllReduce, max) whether every rank could -- if
// one could not, the whole world keeps the RCCL transport for this plan.
// Shared worlds: an all-gather of `n` bytes per rank through files -- each rank writes
// x<seq>_r<rank> (written to a temporary name, then renamed, so a reader never sees half a file)
// and reads everyone's, waiting up to a minute for the slowest rank.
int file_allgather(rt_comm c, const void* mine, size_t n, void* all) {
    const uint64_t seq = ++c->fseq;
    auto name = [&](int q) { return xname(c, seq, q); };
    {
        const std::string tmp = name(c->rank) + ".tmp";
        std::FILE* f = std::fopen(tmp.c_str(), "wb");
        if (!f) return RT_FILE_NOT_FOUND;
        const bool ok = std::fwrite(mine, 1, n, f) == n;
        if (std::fclose(f) != 0 || !ok || std::rename(tmp.c_str(), name(c->rank).c_str()) != 0) return RT_OUT_OF_RESOURCES;
    }
    const auto deadline = std::chrono::steady_clock::now() + std::chrono::seconds(60);
    for (int q = 0; q < c->nranks; ++q) {
        for (;;) {
            std::FILE* f = std::fopen(name(q).c_str(), "rb");
            if (f) {
                const bool ok = std::fread(static_cast<uint8_t*>(all) + (size_t)q * n, 1, n, f) == n;
                std::fclose(f);
                if (!ok) return RT_PARSE_ERROR;
                break;
            }
            if (std::chrono::steady_clock::now() > deadline) return RT_OUT_OF_RESOURCES;
            std::this_thread::sleep_for(std::chrono::milliseconds(1));
        }
    }
    return RT_SUCCESS;
}

// the world's maximum of v (RCCL, or files in a shared world)
int world_max(rt_comm c, int v, int* out) {
    if (!c->fdir.empty()) {
        std::vector<int> all(c->nranks);
        int rc = file_allgather(c, &v, sizeof(v), all.data());
        if (rc) return rc;
        *out = *std::max_element(all.begin(), all.end());
        return RT_SUCCESS;
    }
    int* d = nullptr;
    hipError_t e = hipMalloc(reinterpret_cast<void**>(&d), 2 * sizeof(int));
    if (e != hipSuccess) return map_hip(e);
    e = hipMemcpy(d, &v, sizeof(int), hipMemcpyHostToDevice);
    int rc = map_hip(e);
    if (!rc) rc = map_nccl(ncclAllReduce(d, d + 1, 1, ncclInt32, ncclMax, c->nc, c->cstream));
    if (!rc) rc = map_hip(hipStreamSynchronize(c->cstream));
    if (!rc) rc = map_hip(hipMemcpy(out, d + 1, sizeof(int), hipMemcpyDeviceToHost));
    (void)hipFree(d);
    return rc;
}

struct IpcBlob {
    hipIpcMemHandle_t target, rflags, probe, sflags;
};

// the host waits for `s` until `deadline` (no hang: a stream stuck on a flag is reported)
bool wait_until(hipStream_t s, std::chrono::steady_clock::time_point deadline) {
    for (;;) {
        const hipError_t q = hipStreamQuery(s);
        if (q == hipSuccess) return true;
        if (q != hipErrorNotReady || std::chrono::steady_clock::now() > deadline) return false;
        std::this_thread::sleep_for(std::chrono::microseconds(200));
    }
}

// reads `n` u64 words of device memory until every word equals `v` or the deadline passes
bool poll_words(const uint64_t* dev, size_t n, uint64_t v, std::chrono::steady_clock::time_point deadline) {
    std::vector<uint64_t> h(n);
    for (;;) {
        if (hipMemcpy(h.data(), dev, h.size() * sizeof(uint64_t), hipMemcpyDeviceToHost) != hipSuccess) return false;
        bool all = true;
        for (size_t i = 0; i < n; ++i) all &= h[i] == v;
        if (all) return true;
        if (std::chrono::steady_clock::now() > deadline) return false;
        std::this_thread::sleep_for(std::chrono::microseconds(200));
    }
}

// One trial round over fresh IPC links, with the production signalling: every rank copies a 4-KB
// pattern into its part of the root's probe and its arrival flag := 1 (copy engines); the root
// waits for every flag (from the host, then -- once they are in memory -- with the stream waits a
// read of the image uses), checks every pattern, copies release := 1 into every rank's flag; each
// rank waits for its own the same two ways; all flags go back to 0.  Returns 1 when anything
// failed or timed out.
int ipc_handshake(rt_comm c) {
    const auto deadline = std::chrono::steady_clock::now() + std::chrono::seconds(20);
    uint8_t* src = nullptr;
    hipError_t e = hipMalloc(reinterpret_cast<void**>(&src), kProbeBytes);
    if (e == hipSuccess) e = hipMemsetAsync(src, (c->rank + 1) & 0xff, kProbeBytes, c->cstream);
    if (e == hipSuccess)
        e = hipMemcpyAsync(c->peer_probe + (size_t)c->rank * kProbeBytes, src, kProbeBytes,
                           hipMemcpyDeviceToDeviceNoCU, c->cstream);
    if (e == hipSuccess) e = flag_copy(c, c->peer_rflags + c->rank, 1, c->cstream);
    const bool sent_ok = e == hipSuccess && wait_until(c->cstream, deadline);
    if (src) (void)hipFree(src);
    if (!sent_ok) return 1;
    if (c->rank == c->root) {
        if (!poll_words(c->rflags, (size_t)c->nranks, 1, deadline)) return 1;
        for (int q = 0; q < c->nranks && e == hipSuccess; ++q)
            e = hipStreamWaitValue64(c->ustream, c->rflags + q, 1, hipStreamWaitValueGte, ~0ull);
        if (e != hipSuccess || !wait_until(c->ustream, deadline)) return 1;
        std::vector<uint8_t> got(kProbeBytes);
        for (int q = 0; q < c->nranks; ++q) {
            if (hipMemcpy(got.data(), c->probe + (size_t)q * kProbeBytes, kProbeBytes, hipMemcpyDeviceToHost) != hipSuccess)
                return 1;
            for (uint8_t b : got)
                if (b != (uint8_t)((q + 1) & 0xff)) return 1;
        }
        for (int q = 0; q < c->nranks && e == hipSuccess; ++q) e = flag_copy(c, c->peer_sflags[q], 1, c->ustream);
        if (e == hipSuccess) e = hipMemsetAsync(c->rflags, 0, sizeof(uint64_t) * c->nranks, c->ustream);
        if (e != hipSuccess || !wait_until(c->ustream, deadline)) return 1;
    }
    if (!poll_words(c->sflags, 1, 1, deadline)) return 1;
    e = hipStreamWaitValue64(c->cstream, c->sflags, 1, hipStreamWaitValueGte, ~0ull);
    if (e != hipSuccess || !wait_until(c->cstream, deadline)) return 1;
    e = hipMemset(c->sflags, 0, sizeof(uint64_t));
    if (e == hipSuccess) e = hipDeviceSynchronize();
    return e == hipSuccess ? 0 : 1;
}

int link_ipc(rt_comm c) {
    hipError_t e = hipSetDevice(c->ctx->device);
    IpcBlob mine{};
    // 0: links hold; RT_COMM_FALLBACK_IPC_MAP / _HANDSHAKE: why not (the world agrees on the max)
    int bad = c->fail_links ? RT_COMM_FALLBACK_HANDSHAKE : 0;
    if (e == hipSuccess && flag_values(c) != RT_SUCCESS) bad = RT_COMM_FALLBACK_HANDSHAKE;
    if (e == hipSuccess) e = hipIpcGetMemHandle(&mine.sflags, c->sflags);
    if (e == hipSuccess && c->rank == c->root) {
        e = hipIpcGetMemHandle(&mine.target, c->target->dptr);
        if (e == hipSuccess) e = hipIpcGetMemHandle(&mine.rflags, c->rflags);
        if (e == hipSuccess) e = hipIpcGetMemHandle(&mine.probe, c->probe);
    }
    if (e != hipSuccess) bad = std::max(bad, (int)RT_COMM_FALLBACK_IPC_MAP);
    std::vector<IpcBlob> all(c->nranks);
    auto exchange = [&]() -> int {
        if (!c->fdir.empty()) return file_allgather(c, &mine, sizeof(mine), all.data());
        void* dev = nullptr;
        hipError_t he = hipMalloc(&dev, sizeof(IpcBlob) * (c->nranks + 1));
        if (he != hipSuccess) return map_hip(he);
        uint8_t* d = static_cast<uint8_t*>(dev);
        he = hipMemcpy(d, &mine, sizeof(mine), hipMemcpyHostToDevice);
        int rc = map_hip(he);
        if (!rc) rc = map_nccl(ncclAllGather(d, d + sizeof(IpcBlob), sizeof(IpcBlob), ncclUint8, c->nc, c->cstream));
        if (!rc) rc = map_hip(hipStreamSynchronize(c->cstream));
        if (!rc)
            rc = map_hip(hipMemcpy(all.data(), d + sizeof(IpcBlob), sizeof(IpcBlob) * c->nranks, hipMemcpyDeviceToHost));
        (void)hipFree(dev);
        return rc;
    };
    auto open = [&](const hipIpcMemHandle_t& h, void** p) {
        *p = nullptr;
        if (bad) return;
        if (hipIpcOpenMemHandle(p, h, hipIpcMemLazyEnablePeerAccess) != hipSuccess) {
            bad = RT_COMM_FALLBACK_IPC_MAP;
            *p = nullptr;
            return;
        }
        c->ipc_opened.push_back(*p);
    };
    int rc = exchange();
    if (!rc) {
        if (c->rank == c->root) {
            c->peer_target = static_cast<uint8_t*>(c->target->dptr);
            c->peer_rflags = c->rflags;
            c->peer_probe = c->probe;
            c->peer_sflags.assign(c->nranks, nullptr);
            for (int q = 0; q < c->nranks; ++q) {
                if (q == c->rank) {
                    c->peer_sflags[q] = c->sflags;
                } else {
                    void* p = nullptr;
                    open(all[q].sflags, &p);
                    c->peer_sflags[q] = static_cast<uint64_t*>(p);
                }
            }
        } else {
            void* p[3] = {};
            open(all[c->root].target, &p[0]);
            open(all[c->root].rflags, &p[1]);
            open(all[c->root].probe, &p[2]);
            c->peer_target = static_cast<uint8_t*>(p[0]);
            c->peer_rflags = static_cast<uint64_t*>(p[1]);
            c->peer_probe = static_cast<uint8_t*>(p[2]);
        }
        // does every rank hold its links?
        rc = world_max(c, bad, &bad);
    }
    // the links hold: one small transfer and both flags across the world, polled from the host
    // with a deadline, before any gather relies on them (a world whose first real gather waited on
    // a flag that never arrives would hang instead of falling back)
    if (!rc && !bad) {
        bad = ipc_handshake(c) ? RT_COMM_FALLBACK_HANDSHAKE : 0;
        rc = world_max(c, bad, &bad);
    }
    if (rc) return rc;
    if (bad && !c->nc) return RT_INVALID_OPERATION;  // a shared world has no RCCL to fall back to
    if (bad) {  // the world falls back to RCCL transfers for this plan
        for (void* p : c->ipc_opened) (void)hipIpcCloseMemHandle(p);
        c->ipc_opened.clear();
        c->peer_target = c->peer_probe = nullptr;
        c->peer_rflags = nullptr;
        c->peer_sflags.clear();
        c->ce = false;
        c->fallback_reason = bad;
        return rccl_buffers(c);
    }
    c->ce = c->ipc_linked = true;
    // one process per GPU (an RCCL world): the other ranks' copy engines write the root's image
    // from other devices (a shared world's ranks all run on one)
    c->remote_writers = c->rank == c->root && c->nranks > 1 && c->fdir.empty();
    return RT_SUCCESS;
}

// pack / unpack copies of the RCCL transport (the runtime runs 2-D device copies as blit kernels)
hipError_t copy_rects(const std::vector<rt_rect>& plan, uint8_t* img, uint8_t* stage, bool to_stage, hipStream_t s) {
    for (const rt_rect& r : plan) {
        hipError_t e = to_stage
            ? hipMemcpy2DAsync(stage + r.stage_offset, r.width, img + r.img_offset, r.img_pitch, r.width, r.rows,
                               hipMemcpyDeviceToDevice, s)
            : hipMemcpy2DAsync(img + r.img_offset, r.img_pitch, stage + r.stage_offset, r.width, r.width, r.rows,
                               hipMemcpyDeviceToDevice, s);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

int rccl_transfer(const rt_comm* comms, int n_local, int root);
// the members of a one-process world know each other (rt_comm_s::members)
void link_members(rt_comm* comms, int n) {
    try {
        auto m = std::make_shared<std::vector<rt_comm>>(comms, comms + n);
        for (int i = 0; i < n; ++i) comms[i]->members = m;
    } catch (const std::bad_alloc&) {  // (no exception crosses the C ABI; a join then waits at once)
        for (int i = 0; i < n; ++i) comms[i]->members.reset();
    }
}
int finish_gather(const rt_comm* comms, int n_local, int root, rt_mem root_dst, const rt_mem* outs);
int ce_gather(const rt_comm* comms, int n_local, int root, const rt_mem* outs);
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
    if (!rc) rc = comm_streams(c);
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
            rc = comm_streams(c);
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
    link_members(comms_out, n);
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
            rc = e == hipSuccess ? comm_streams(c) : map_hip(e);
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
    link_members(comms_out, n);
    return RT_SUCCESS;
}

int rtCommInitShared(rt_context ctx, int nranks, int rank, const char* dir, rt_comm* out) {
    if (!out) return RT_INVALID_VALUE;
    *out = nullptr;
    if (!ctx) return RT_INVALID_CONTEXT;
    if (!dir || !*dir || nranks < 1 || rank < 0 || rank >= nranks) return RT_INVALID_VALUE;
    hipError_t he = hipSetDevice(ctx->device);
    if (he != hipSuccess) return map_hip(he);
    rt_comm c = new (std::nothrow) rt_comm_s();
    if (!c) return RT_OUT_OF_HOST_MEMORY;
    c->ctx = ctx;
    c->rank = rank;
    c->nranks = nranks;
    try {
        c->fdir = dir;
    } catch (const std::bad_alloc&) {
        delete c;
        return RT_OUT_OF_HOST_MEMORY;
    }
    int rc = shared_world_id(c);
    if (rc) {
        delete c;
        return rc;
    }
    rc = comm_streams(c);
    if (rc) {
        release(c);
        return rc;
    }
    *out = c;
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

int rtCommSetTransport(rt_comm c, int transport) {
    if (!c) return RT_INVALID_VALUE;
    if (transport != RT_COMM_TRANSPORT_COPY_ENGINES && transport != RT_COMM_TRANSPORT_RCCL &&
        transport != RT_COMM_TRANSPORT_COPY_ENGINES_IPC)
        return RT_INVALID_VALUE;
    if (c->group && transport != RT_COMM_TRANSPORT_COPY_ENGINES) return RT_INVALID_OPERATION;
    if (!c->nc && transport == RT_COMM_TRANSPORT_RCCL) return RT_INVALID_OPERATION;  // shared worlds
    (void)hipSetDevice(c->ctx->device);
    quiesce(c);
    c->transport = transport;
    free_buffers(c);  // the next gather builds the plan for it (also: a new destination)
    return RT_SUCCESS;
}

int rtCommGetTransport(rt_comm c, int* transport, int* active) {
    if (!c) return RT_INVALID_VALUE;
    if (transport) *transport = c->transport;
    // the transport the current plan uses (-1: no plan yet)
    if (active) *active = c->W == 0 ? -1 : !c->ce ? RT_COMM_TRANSPORT_RCCL : c->ipc_linked ? RT_COMM_TRANSPORT_COPY_ENGINES_IPC
                                                                                   : RT_COMM_TRANSPORT_COPY_ENGINES;
    return RT_SUCCESS;
}

int rtCommGetStatus(rt_comm c, rt_comm_status* out) {
    if (!c || !out) return RT_INVALID_VALUE;
    std::memset(out, 0, sizeof(*out));
    out->rank = c->rank;
    out->nranks = c->nranks;
    (void)rtCommGetTransport(c, &out->transport, &out->active);
    out->fallback = c->fallback_reason != RT_COMM_FALLBACK_NONE;
    out->fallback_reason = c->fallback_reason;
    out->gathers = c->seq;
    if (c->W != 0 && c->ce) {
        if (c->sends)
            for (const auto& r : c->runs) out->bytes_per_gather += r.second;
        // the root: its own bands straight into the destination; the others: pack + transfer + flag
        const unsigned n = (unsigned)c->runs.size();
        out->copies_per_gather = !c->sends ? 0u : c->rank == c->root ? n : 2u * n + (c->ipc_linked ? 1u : 0u);
    } else if (c->W != 0) {
        out->bytes_per_gather = c->stage_bytes;
        out->copies_per_gather = 1;
    }
    out->last_xfer_ms = -1.0;
    float ms = 0.0f;
    if (c->xt_valid && hipEventQuery(c->xt1) == hipSuccess && hipEventElapsedTime(&ms, c->xt0, c->xt1) == hipSuccess)
        out->last_xfer_ms = ms;
    return RT_SUCCESS;
}

int rtCommSetOption(rt_comm c, int option, int value) {
    if (!c) return RT_INVALID_VALUE;
    if (option == RT_COMM_OPT_FAIL_LINKS) {
        c->fail_links = value != 0;
        return RT_SUCCESS;
    }
    if (option == RT_COMM_OPT_REPLAN_PERIOD) {
        if (value < 1 || (uint64_t)value > kFlagValues - 2) return RT_INVALID_VALUE;
        c->replan_after = (uint64_t)value;
        return RT_SUCCESS;
    }
    if (option == RT_COMM_OPT_SYSTEM_ACQUIRE) {
        c->force_acquire = value != 0;
        return RT_SUCCESS;
    }
    return RT_INVALID_VALUE;
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
        if (!c || !outs[i] || outs[i]->released) return RT_INVALID_VALUE;
        if (root < 0 || root >= c->nranks) return RT_INVALID_VALUE;
        if (outs[i]->ctx != c->ctx || outs[i]->size < img_bytes) return RT_INVALID_MEM_OBJECT;
        if (c->rank == root && root_dst &&
            (root_dst->released || root_dst->ctx != c->ctx || root_dst->size < img_bytes))
            return RT_INVALID_MEM_OBJECT;
    }
    if (int rc = check_loopback(comms, n_local)) return rc;
    for (int i = 0; i < n_local; ++i)  // coalesced per-frame launches first: the gather reads their output
        if (comms[i]->ctx->pend_k) (void)rti::flush_frames(comms[i]->ctx);
    // the plans (rebuilt, by every rank alike, when the size, the root or the transport changes).
    // The root's destination is part of a copy-engine plan: linked by address (every rank in this
    // call) a new one rebuilds it; linked by IPC handles the root cannot tell the other processes,
    // so it refuses a new destination until a collective re-plan
    const bool whole_world = n_local == comms[0]->nranks;
    bool fresh = false;
    for (int i = 0; i < n_local; ++i) {
        rt_comm c = comms[i];
        hipError_t e = hipSetDevice(c->ctx->device);
        if (e != hipSuccess) return map_hip(e);
        rt_mem dst = c->rank == root ? (root_dst ? root_dst : outs[i]) : nullptr;
        if (c->ipc_linked && c->rank == root && c->W == W && c->H == H && c->root == root && c->target != dst)
            return RT_INVALID_OPERATION;
        bool built = false;
        int rc = ensure_plan(c, W, H, root, dst, outs[i], &built);
        if (rc) return rc;
        fresh |= built;
    }
    if (fresh && comms[0]->transport != RT_COMM_TRANSPORT_RCCL) {
        int rc = RT_SUCCESS;
        if (comms[0]->transport == RT_COMM_TRANSPORT_COPY_ENGINES_IPC) {
            if (n_local != 1 || (!comms[0]->nc && comms[0]->fdir.empty())) return RT_INVALID_OPERATION;
            rc = link_ipc(comms[0]);
        } else if (whole_world) {
            rc = link_direct(comms, n_local, root);  // every member is in this call
            if (rc && !comms[0]->group) {            // (RCCL world: keep RCCL's transfers)
                rc = RT_SUCCESS;
                for (int i = 0; i < n_local && !rc; ++i) {
                    comms[i]->ce = false;
                    comms[i]->fallback_reason = RT_COMM_FALLBACK_NO_PEER_ACCESS;
                    rc = rccl_buffers(comms[i]);
                }
            }
        } else if (n_local == 1 && (comms[0]->nc || !comms[0]->fdir.empty())) {
            rc = link_ipc(comms[0]);
        }
        if (rc) return rc;
    }
    // only a copy-engine plan writes into the destination it was built with: an RCCL plan (asked
    // for, or a fallback) unpacks into whatever each call names, so it keeps no pin on the first one
    for (int i = 0; fresh && i < n_local; ++i)
        if (!comms[i]->ce && comms[i]->target) {
            rti::unpin(comms[i]->target);
            comms[i]->target = nullptr;
        }
    bool ce = true;
    for (int i = 0; i < n_local; ++i) ce &= comms[i]->ce;
    // loopback and shared worlds move bytes on the copy engines only
    if ((comms[0]->group || !comms[0]->fdir.empty()) && !ce) return RT_INVALID_OPERATION;
    if (ce) return ce_gather(comms, n_local, root, outs);
    // RCCL transport.  Phase 1: every rank (the root too) packs its bands on its context's
    // accumulation stream
    for (int i = 0; i < n_local; ++i) {
        rt_comm c = comms[i];
        rt_context ctx = c->ctx;
        hipError_t e = hipSetDevice(ctx->device);
        if (e != hipSuccess) return map_hip(e);
        if (int rc = rccl_buffers(c)) return rc;
        const int s = c->slot;
        ++c->seq;
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
        if (e == hipSuccess) e = hipEventRecord(c->xt0, c->cstream);
        if (e != hipSuccess) return map_hip(e);
        ctx->apending = true;
    }
    // phase 2: the transfers, one group over every local rank (required when one thread drives
    // several GPUs).  The root posts one receive per rank, so all its links carry data at once;
    // its own bands take the same path (a send to itself, a device-local copy) -- one uniform
    // unpack, and a world of one still runs the whole RCCL flow.
    int rc = rccl_transfer(comms, n_local, root);
    if (rc) return rc;
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

// Copies of this rank's band runs on the copy engines: run i (image offset o_i, n_i bytes, dense
// offset d_i -- its place in the staging slot) from src + (src_dense ? d_i : o_i) to
// dst + (dst_dense ? d_i : o_i).  On stream `s` alone, or (split) dealt out over the transfer
// streams in image order in pieces of at least 1 MiB, after and before everything on `s`.
hipError_t copy_runs(rt_comm c, hipStream_t s, bool split, uint8_t* dst, bool dst_dense, const uint8_t* src,
                     bool src_dense) {
    uint64_t total = 0;
    for (const auto& r : c->runs) total += r.second;
    const size_t k = split ? std::max<size_t>(1, std::min<uint64_t>(RT_COMM_XFER_STREAMS, total >> 20)) : 1;
    auto copy = [&](size_t run, uint64_t dense, uint64_t at, uint64_t n, hipStream_t st) {
        const uint64_t o = c->runs[run].first + at, d = dense + at;
        return hipMemcpyAsync(dst + (dst_dense ? d : o), src + (src_dense ? d : o), n, hipMemcpyDeviceToDeviceNoCU, st);
    };
    if (k == 1) {
        uint64_t dense = 0;
        for (size_t i = 0; i < c->runs.size(); ++i) {
            if (hipError_t e = copy(i, dense, 0, c->runs[i].second, s)) return e;
            dense += c->runs[i].second;
        }
        return hipSuccess;
    }
    hipError_t e = hipEventRecord(c->xgo, s);
    const uint64_t share = ((total + k - 1) / k + 255) & ~(uint64_t)255;
    size_t run = 0;
    uint64_t run_done = 0, dense = 0;  // bytes of runs[run] already dealt out; its dense offset
    for (size_t i = 0; i < k && e == hipSuccess && run < c->runs.size(); ++i) {
        e = hipStreamWaitEvent(c->xstream[i], c->xgo, 0);
        uint64_t left = share;
        while (e == hipSuccess && left > 0 && run < c->runs.size()) {
            const uint64_t n = std::min(left, c->runs[run].second - run_done);
            e = copy(run, dense, run_done, n, c->xstream[i]);
            left -= n;
            run_done += n;
            if (run_done == c->runs[run].second) {
                dense += run_done;
                ++run;
                run_done = 0;
            }
        }
        if (e == hipSuccess) e = hipEventRecord(c->xdone[i], c->xstream[i]);
        if (e == hipSuccess) e = hipStreamWaitEvent(s, c->xdone[i], 0);
    }
    return e;
}

// Copy-engine gather (see the top of the file).  Flags carry the gather's sequence number seq
// (1, 2, ... within a plan): rflags[q] = seq when rank q's bands of image seq are in the root's
// destination, sflags = seq when the root has released image seq (everything its context queued
// before gather seq + 1 has run) -- a rank's transfer of image seq + 1 waits for it.  Ranks driven
// by this process (loopback worlds, rtCommInitAll) order the same steps with events instead (the
// root's `released`, the ranks' `sent`), joined by the root at once (events wait without a
// kernel).
int ce_gather(const rt_comm* comms, int n_local, int root, const rt_mem* outs) {
    rt_comm R = nullptr;  // the root, when it is driven by this call
    rt_mem Rout = nullptr;
    for (int i = 0; i < n_local; ++i)
        if (comms[i]->rank == root) {
            R = comms[i];
            Rout = outs[i];
        }
    // 1. the root releases the previous image once everything its context queued so far has run
    if (R) {
        hipError_t e = hipSetDevice(R->ctx->device);
        const uint64_t prev = R->seq;
        if (e == hipSuccess) e = rti::main_tail_wait(R->ctx, R->ustream);
        // (reads on the accumulation stream: rtContextSetReadbackOnAccumStream)
        if (e == hipSuccess && R->ctx->readback_on_astream) e = hipStreamWaitEvent(R->ustream, R->ctx->atail, 0);
        for (int q = 0; R->ipc_linked && prev > 0 && q < R->nranks && e == hipSuccess; ++q)
            if (q != root) e = flag_copy(R, R->peer_sflags[q], prev, R->ustream);
        if (e == hipSuccess) e = hipEventRecord(R->released, R->ustream);
        // 1b. gathering into another buffer, the root copies its own bands there straight from its
        // output: after the accumulations and per-frame launches that wrote them, after the reads
        // of the previous image; the next accumulation waits for the copies (out_read_wait)
        if (e == hipSuccess && R->sends) {
            rt_context ctx = R->ctx;
            ++R->seq;
            e = rti::main_tail_wait(ctx, ctx->astream);
            if (e == hipSuccess) e = hipEventRecord(R->ready, ctx->astream);
            if (e == hipSuccess) e = hipStreamWaitEvent(R->cstream, R->ready, 0);
            if (e == hipSuccess) e = hipStreamWaitEvent(R->cstream, R->released, 0);
            if (e == hipSuccess) e = hipEventRecord(R->xt0, R->cstream);
            if (e == hipSuccess)
                e = copy_runs(R, R->cstream, true, static_cast<uint8_t*>(R->target->dptr), false,
                              static_cast<const uint8_t*>(Rout->dptr), false);
            if (e == hipSuccess) e = hipEventRecord(R->xt1, R->cstream);
            if (e == hipSuccess) e = hipEventRecord(R->dsent, R->cstream);
            if (e == hipSuccess) {
                R->xt_valid = true;
                ctx->oread_ev = R->dsent;
                ctx->oread = true;
            }
        } else if (e == hipSuccess) {
            ++R->seq;
        }
        if (e != hipSuccess) return map_hip(e);
    }
    // 2. every other rank: pack its bands into a staging slot right after the accumulation
    // (accumulation stream: the next accumulation never waits across GPUs), then -- once the root
    // has released the previous image -- transfer them into the root's destination and raise its
    // arrival flag, all on the copy engines
    for (int i = 0; i < n_local; ++i) {
        rt_comm c = comms[i];
        if (c == R) continue;
        rt_context ctx = c->ctx;
        const uint64_t seq = ++c->seq;
        const int s = c->slot;
        hipError_t e = hipSetDevice(ctx->device);
        if (e == hipSuccess) e = rti::main_tail_wait(ctx, ctx->astream);
        if (e == hipSuccess && c->sent_valid[s]) e = hipStreamWaitEvent(ctx->astream, c->sent[s], 0);  // slot free
        if (e == hipSuccess)
            e = copy_runs(c, ctx->astream, false, static_cast<uint8_t*>(c->stage[s]), true,
                          static_cast<const uint8_t*>(outs[i]->dptr), false);
        if (e == hipSuccess) e = hipEventRecord(c->packed[s], ctx->astream);
        if (e == hipSuccess) e = hipEventRecord(ctx->atail, ctx->astream);
        if (e == hipSuccess) ctx->apending = true;
        if (e == hipSuccess) e = hipStreamWaitEvent(c->cstream, c->packed[s], 0);
        if (e == hipSuccess && seq > 1) {  // the root is done with the previous image
            e = c->ipc_linked ? hipStreamWaitValue64(c->cstream, c->sflags, seq - 1, hipStreamWaitValueGte, ~0ull)
                              : hipStreamWaitEvent(c->cstream, R->released, 0);
        }
        if (e == hipSuccess) e = hipEventRecord(c->xt0, c->cstream);
        if (e == hipSuccess)
            e = copy_runs(c, c->cstream, !(!c->ipc_linked && c->nranks > 1), c->peer_target, false,
                          static_cast<const uint8_t*>(c->stage[s]), true);
        if (e == hipSuccess) e = hipEventRecord(c->xt1, c->cstream);
        if (e == hipSuccess && c->ipc_linked) e = flag_copy(c, c->peer_rflags + c->rank, seq, c->cstream);
        if (e == hipSuccess) e = hipEventRecord(c->sent[s], c->cstream);
        // reads on this rank's context wait for its transfer (qs)
        if (e == hipSuccess) e = hipEventRecord(ctx->gtail, c->cstream);
        if (e != hipSuccess) return map_hip(e);
        c->sent_valid[s] = true;
        c->xt_valid = true;
        ctx->gpending = true;
        c->slot ^= 1;
    }
    // 3. the root's context joins the arrivals when the image is next read (join_gather): flag
    // waits between processes, the ranks' events within one.  Nothing waits at gather time: even
    // an event wait on the root's stream cost the world-1 flow 2 % (0.804 vs 0.788 ms/frame,
    // profiles/r05/gather_world1_ab.txt)
    if (R) {
        R->join_seq = R->seq;
        R->join_events.clear();
        if (!R->ipc_linked && !R->members && n_local > 1) {  // (no member list: join now, on the root's stream)
            hipError_t e = hipSetDevice(R->ctx->device);
            for (int j = 0; j < n_local && e == hipSuccess; ++j)
                if (comms[j] != R) e = hipStreamWaitEvent(R->ustream, comms[j]->sent[comms[j]->slot ^ 1], 0);
            if (e == hipSuccess && R->sends) e = hipStreamWaitEvent(R->ustream, R->dsent, 0);
            if (e == hipSuccess && (R->remote_writers || R->force_acquire)) {  // (see join_gather)
                hipLaunchKernelGGL(system_acquire_kernel, dim3(R->ctx->num_cus > 0 ? R->ctx->num_cus : 256), dim3(64), 0,
                                   R->ustream);
                e = hipGetLastError();
            }
            if (e == hipSuccess) e = hipEventRecord(R->ctx->gtail, R->ustream);
            if (e != hipSuccess) return map_hip(e);
            R->ctx->gpending = true;
            return RT_SUCCESS;
        }
        for (int j = 0; !R->ipc_linked && j < n_local; ++j)
            if (comms[j] != R) R->join_events.push_back(comms[j]->sent[comms[j]->slot ^ 1]);
        R->ctx->gjoin = R;
        R->ctx->gpending = false;
    }
    return RT_SUCCESS;
}

// phase 3 of the RCCL transport: the root unpacks every rank's bands into the destination
int finish_gather(const rt_comm* comms, int n_local, int root, rt_mem root_dst, const rt_mem* outs) {
    for (int i = 0; i < n_local; ++i) {
        rt_comm c = comms[i];
        rt_context ctx = c->ctx;
        const int s = c->slot;
        hipError_t e = hipSetDevice(ctx->device);
        if (e == hipSuccess) e = hipEventRecord(c->xt1, c->cstream);
        if (e == hipSuccess) e = hipEventRecord(c->sent[s], c->cstream);
        if (e != hipSuccess) return map_hip(e);
        c->xt_valid = true;
        c->sent_valid[s] = true;
        if (c->rank == root) {
            // Gathering into the root's own output: its own bands are in place already and are
            // not unpacked, so the unpack writes only other ranks' rows, which no later render,
            // accumulation or pack of this context touches -- nothing on the context waits for
            // it.  (An unpack that the next accumulation had to wait for chained that
            // accumulation, and the render after it, to the transfer: RCCL's kernel gets CUs only
            // as a persistent render drains, so every second render started a step late --
            // world-1 0.90 vs 0.77 ms/frame, profiles/r04/dist_flow_ab.txt.)  Reads of the
            // image wait for it through the context's queue (gtail, qs()); the unpack waits for
            // the reads queued before this gather.
            const bool into_out = !root_dst || root_dst == outs[i];
            uint8_t* dst = static_cast<uint8_t*>((root_dst ? root_dst : outs[i])->dptr);
            e = rti::main_tail_wait(ctx, c->ustream);
            if (e == hipSuccess) e = hipStreamWaitEvent(c->ustream, c->sent[s], 0);
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

}  // namespace

// The root's first read of a gathered image: `s` waits for every rank's arrival (flags between
// processes, events within one; and the root's own copies), and the context's gather tail
// becomes that point of `s`.  Where other devices' copy engines wrote the image (remote_writers),
// the root's caches may still hold lines of the previous image that the root read before (its
// blits, kernels): a system-scope acquire on every XCD follows the waits, before any read.
// (Multi-GPU byte parity of the direct-write gather has not been verified on hardware: every run
// so far wrote from one device; RT_COMM_OPT_SYSTEM_ACQUIRE runs the acquire there, tests/test_comm.py.)
hipError_t rti::join_gather(rt_comm c, hipStream_t s) {
    hipError_t e = hipSetDevice(c->ctx->device);
    for (int q = 0; c->ipc_linked && q < c->nranks && e == hipSuccess; ++q)
        if (q != c->root) e = hipStreamWaitValue64(s, c->rflags + q, c->join_seq, hipStreamWaitValueGte, ~0ull);
    for (size_t j = 0; j < c->join_events.size() && e == hipSuccess; ++j) e = hipStreamWaitEvent(s, c->join_events[j], 0);
    if (e == hipSuccess && c->sends) e = hipStreamWaitEvent(s, c->dsent, 0);
    if (e == hipSuccess && (c->remote_writers || c->force_acquire)) {
        hipLaunchKernelGGL(system_acquire_kernel, dim3(c->ctx->num_cus > 0 ? c->ctx->num_cus : 256), dim3(64), 0, s);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipEventRecord(c->ctx->gtail, s);
    return e;
}

namespace {

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
    if (!comms[0]->fdir.empty()) {
        // shared world: one rank per call, the reduction through the exchange files, after this
        // rank's earlier gathers have drained (as RCCL's stream order would have it)
        if (n_local != 1) return RT_INVALID_VALUE;
        rt_comm c = comms[0];
        hipError_t e = hipSetDevice(c->ctx->device);
        if (e == hipSuccess) e = hipStreamSynchronize(c->cstream);
        if (e == hipSuccess) e = hipStreamSynchronize(c->ustream);
        if (e != hipSuccess) return map_hip(e);
        std::vector<double> all((size_t)c->nranks * count);
        int rc = file_allgather(c, values, sizeof(double) * count, all.data());
        if (rc) return rc;
        for (int j = 0; j < count; ++j) {
            double acc = all[j];
            for (int q = 1; q < c->nranks; ++q) {
                const double v = all[(size_t)q * count + j];
                acc = op == RT_COMM_SUM ? acc + v : std::max(acc, v);
            }
            values[j] = acc;
        }
        return RT_SUCCESS;
    }
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

int rtBandPackPlan(unsigned width, unsigned height, unsigned period, unsigned phase, rt_rect* rects,
                   int capacity, int* n_rects, size_t* staging_bytes) {
    return band_plan(width, height, period, phase, rects, capacity, n_rects, staging_bytes);
}

}  // extern "C"
