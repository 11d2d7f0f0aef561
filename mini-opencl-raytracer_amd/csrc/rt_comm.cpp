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
//   communicator stream         :                 (wait pack) [transfer k -> root slot s] [flag]
//   root unpack stream          :                      (wait flags k) [unpack k -> dst] [free s]
//   context render streams      : [render k+1 ........................................]
//
// Two staging slots alternate, so step k's transfer runs under step k+1's render.
//
// Transport (rtCommSetTransport).  A persistent render holds every CU slot until it drains, and
// RCCL's transfer kernel (64 workgroups, 248 VGPRs, 37 KB LDS each on gfx950) fits beside it
// nowhere: in the world-1 flow its transfer waited for renders to drain (19 ms for a 0.12-ms
// copy) and every second step stalled on it (profiles/r04/dist_flow_ab.txt).  So by default the
// bytes move on the COPY ENGINES (SDMA, hipMemcpyDeviceToDeviceNoCU; over xGMI between GPUs):
// every rank copies its staging slot straight into the root's receive slot (an IPC-mapped
// pointer to the root's memory, exchanged once per plan with one ncclAllGather), then raises its
// arrival flag in the root's memory (hipStreamWriteValue64); the root's unpack stream waits for
// the flags (hipStreamWaitValue64) and, after the unpack, raises each rank's slot-free flag,
// which that rank's next copy into the slot waits for.  No compute unit is needed for the
// transfer, no host round trip for the synchronisation.  RCCL stays for the setup, reductions
// and barriers, and as the grouped ncclSend/ncclRecv transport (RT_COMM_TRANSPORT_RCCL; also
// the fallback when a rank cannot map the root's memory).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
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
    // members), whose gathers always run on the copy engines with the members linked by address
    const void* group = nullptr;
    hipEvent_t xfer = nullptr;  // (unused since the copy-engine transport; kept for the ABI of the struct's users)
    bool reserved = false;      // holds a CU reservation on ctx (rti::reserve_cus)
    int rank = 0, nranks = 1;
    hipStream_t cstream = nullptr;  // transfers (copy engines or RCCL), RCCL setup and reductions
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
    // copy-engine transport (see the top of the file)
    int transport = RT_COMM_TRANSPORT_COPY_ENGINES;  // requested (rtCommSetTransport)
    bool ce = false;                 // this plan moves bytes on the copy engines
    bool ipc_linked = false;         // ... with its links exchanged as IPC handles (link_ipc)
    uint64_t seq = 0;                // gathers enqueued with this plan (1, 2, ...)
    uint64_t* sflags = nullptr;      // [2] (fine-grained, this rank's memory): slot s freed by the root up to seq
    uint64_t* rflags = nullptr;      // root, [nranks][2] (fine-grained): rank q's bytes for slot s arrived, seq
    uint8_t* peer_parts[2] = {};     // the root's receive slots, as this rank addresses them
    uint64_t* peer_rflags = nullptr; // the root's arrival flags, as this rank addresses them
    std::vector<uint64_t*> peer_sflags;  // root: every rank's slot-free flags
    std::vector<void*> ipc_opened;       // IPC mappings to close with the plan
    // the copy-engine transfer split over streams of its own, which the runtime spreads over
    // several SDMA engines (one engine: 61 GB/s; 2 streams 120, 8 streams 154 GB/s on MI355X,
    // scripts/probes/gather_engines_probe.hip split, profiles/r04/gather_engines_probe.txt).
    // Every stream shares the 4 hardware queues, though: in the world-1 flow 2 streams beat 1
    // (0.790 vs 0.798 ms/frame) and 8 stalled the renders (1.17; profiles/r04/dist_flow_ab.txt)
    hipStream_t xstream[8] = {};
    hipEvent_t xgo = nullptr, xdone[8] = {};
    // shared worlds (rtCommInitShared): no RCCL; setup exchanges, reductions and barriers go
    // through files in `fdir` (exchange number fseq), the gathers over the copy engines
    std::string fdir;
    uint64_t fseq = 0;
};

namespace {

// The communicator's transfer and unpack streams run at the device's greatest stream priority.
// Two reasons, both read off a kernel trace of the world-1 flow (profiles/r04/dist_flow_ab.txt):
// * HIP maps streams onto a few hardware queues (GPU_MAX_HW_QUEUES 4); at normal priority these two
//   shared the main stream's and a render stream's queue, so the next fused render sat behind the
//   previous step's unpack, which sat behind its transfer.  High-priority streams get queues of
//   their own.
// * RCCL's transfer kernel needs CU slots, and a persistent render holds them all until it
//   drains; at high priority its workgroups are dispatched first -- which still leaves it waiting
//   for a drain (hence the copy-engine transport).
#ifndef RT_COMM_STREAM_PRIO
#define RT_COMM_STREAM_PRIO 1
#endif
// RCCL communicators: CUs of every XCD kept for the communicator's streams (rti::reserve_cus),
// an A/B knob of the RCCL transport.  RCCL's transfer kernel (64 workgroups of 256 threads, 37 KB
// of LDS and 248 VGPRs each on gfx950) fits beside a persistent render on no CU; with a
// reservation it runs at once on its own CUs, but the renders lose those CUs' share and the
// world-1 flow measured slower than without (0.85 vs 0.82 ms/frame, profiles/r04/dist_flow_ab.txt).
// 0 = none (default).
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

#ifndef RT_COMM_XFER_STREAMS
#define RT_COMM_XFER_STREAMS 2  // 1: the copy on the communicator stream itself
#endif
#ifndef RT_COMM_XFER_PRIO
#define RT_COMM_XFER_PRIO 1     // extra transfer streams at the greatest priority (own hardware queues)
#endif
static_assert(RT_COMM_XFER_STREAMS >= 1 && RT_COMM_XFER_STREAMS <= 8, "copy streams");
int comm_events(rt_comm c, hipError_t e) {
    int least = 0, greatest = 0;
    if (e == hipSuccess) e = hipDeviceGetStreamPriorityRange(&least, &greatest);
    for (int i = 0; RT_COMM_XFER_STREAMS > 1 && i < RT_COMM_XFER_STREAMS && e == hipSuccess; ++i) {
        e = hipStreamCreateWithPriority(&c->xstream[i], hipStreamNonBlocking, RT_COMM_XFER_PRIO ? greatest : least);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&c->xdone[i], hipEventDisableTiming);
    }
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->xgo, hipEventDisableTiming);
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
    for (void* p : c->ipc_opened) (void)hipIpcCloseMemHandle(p);
    c->ipc_opened.clear();
    for (int s = 0; s < 2; ++s) {
        if (c->stage[s]) (void)hipFree(c->stage[s]);
        if (c->parts[s]) (void)hipFree(c->parts[s]);
        c->stage[s] = c->parts[s] = nullptr;
        c->peer_parts[s] = nullptr;
        c->sent_valid[s] = c->unpacked_valid[s] = false;
    }
    if (c->sflags) (void)hipFree(c->sflags);
    if (c->rflags) (void)hipFree(c->rflags);
    c->sflags = c->rflags = c->peer_rflags = nullptr;
    c->peer_sflags.clear();
    c->ce = c->ipc_linked = false;
    c->seq = 0;
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
    for (int i = 0; i < 8; ++i) {
        if (c->xstream[i]) (void)hipStreamSynchronize(c->xstream[i]);
        if (c->xstream[i]) (void)hipStreamDestroy(c->xstream[i]);
        if (c->xdone[i]) (void)hipEventDestroy(c->xdone[i]);
    }
    if (c->xgo) (void)hipEventDestroy(c->xgo);
    if (c->scratch) (void)hipFree(c->scratch);
    if (c->nc) (void)ncclCommDestroy(c->nc);
    if (c->cstream) (void)hipStreamDestroy(c->cstream);
    if (c->ustream) (void)hipStreamDestroy(c->ustream);
    // the last communicator of the context gives its CUs back to the renders
    if (c->reserved && --c->ctx->reserve_refs == 0) (void)rti::reserve_cus(c->ctx, 0, nullptr);
    // a shared world's rank removes its own exchange files but the last: every rank wrote its file
    // of exchange k only after reading all files of exchange k - 1, so those have all been read;
    // the last one may still be awaited by a slower rank (the caller removes the directory)
    for (uint64_t q = 1; !c->fdir.empty() && q < c->fseq; ++q)
        (void)std::remove((c->fdir + "/x" + std::to_string(q) + "_r" + std::to_string(c->rank)).c_str());
    delete c;
}

// buffers and plans for a W x H gather (all earlier gathers of this comm have completed)
int ensure_plan(rt_comm c, unsigned W, unsigned H, int root, bool* built) {
    *built = false;
    if (c->W == W && c->H == H && c->root == root) return RT_SUCCESS;
    *built = true;
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
    // copy engines: the root's receive slots and every flag word are fine-grained memory (the
    // copies and flag writes come from other devices' engines; the unpack and the waits read
    // them coherently), each its own allocation (an IPC handle maps a whole allocation)
    const bool ce = c->transport != RT_COMM_TRANSPORT_RCCL;
    auto alloc = [&](void** p, size_t n, bool fine) {
        return fine ? hipExtMallocWithFlags(p, n, hipDeviceMallocFinegrained) : hipMalloc(p, n);
    };
    hipError_t e = hipSuccess;
    for (int s = 0; s < 2 && e == hipSuccess; ++s) {
        e = hipMalloc(&c->stage[s], std::max<size_t>(sb, 16));
        if (e == hipSuccess && c->rank == root) e = alloc(&c->parts[s], std::max<size_t>(sb * c->nranks, 16), ce);
    }
    if (ce && e == hipSuccess) e = alloc(reinterpret_cast<void**>(&c->sflags), 2 * sizeof(uint64_t), true);
    if (ce && e == hipSuccess && c->rank == root)
        e = alloc(reinterpret_cast<void**>(&c->rflags), 2 * sizeof(uint64_t) * c->nranks, true);
    if (ce && e == hipSuccess) e = hipMemset(c->sflags, 0, 2 * sizeof(uint64_t));
    if (ce && e == hipSuccess && c->rflags) e = hipMemset(c->rflags, 0, 2 * sizeof(uint64_t) * c->nranks);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e != hipSuccess) {
        free_buffers(c);
        return map_hip(e);
    }
    c->W = W;
    c->H = H;
    c->root = root;
    return RT_SUCCESS;
}

// Copy-engine links of a plan whose members are all in this call (loopback worlds, and RCCL
// worlds driven by one process): the root's slots and flags by address.  Between devices the
// copy engines reach peer memory once peer access is on.
int link_direct(const rt_comm* comms, int n_local, int root) {
    rt_comm R = nullptr;
    for (int i = 0; i < n_local; ++i)
        if (comms[i]->rank == root) R = comms[i];
    if (!R) return RT_INVALID_VALUE;
    R->peer_sflags.assign(R->nranks, nullptr);
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
        for (int s = 0; s < 2; ++s) c->peer_parts[s] = static_cast<uint8_t*>(R->parts[s]);
        c->peer_rflags = R->rflags;
        R->peer_sflags[c->rank] = c->sflags;
        c->ce = true;
    }
    return RT_SUCCESS;
}

// The same links across processes: every rank publishes IPC handles of its allocations (the
// root: receive slots and arrival flags; everyone: slot-free flags) with one ncclAllGather, maps
// the ones it needs, and the world agrees (ncclAllReduce, max) whether every rank could -- if
// one could not, the whole world keeps the RCCL transport for this plan.
// Shared worlds: an all-gather of `n` bytes per rank through files -- each rank writes
// x<seq>_r<rank> (written to a temporary name, then renamed, so a reader never sees half a file)
// and reads everyone's, waiting up to a minute for the slowest rank.
int file_allgather(rt_comm c, const void* mine, size_t n, void* all) {
    const uint64_t seq = ++c->fseq;
    auto name = [&](int q) { return c->fdir + "/x" + std::to_string(seq) + "_r" + std::to_string(q); };
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
    hipIpcMemHandle_t parts[2], rflags, sflags;
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
bool poll_words(const uint64_t* dev, size_t n, size_t stride, uint64_t v, std::chrono::steady_clock::time_point deadline) {
    std::vector<uint64_t> h(n * stride);
    for (;;) {
        if (hipMemcpy(h.data(), dev, h.size() * sizeof(uint64_t), hipMemcpyDeviceToHost) != hipSuccess) return false;
        bool all = true;
        for (size_t i = 0; i < n; ++i) all &= h[i * stride] == v;
        if (all) return true;
        if (std::chrono::steady_clock::now() > deadline) return false;
        std::this_thread::sleep_for(std::chrono::microseconds(200));
    }
}

// One trial round over fresh IPC links: every rank copies a 4-KB pattern into its part of the
// root's slot 0 on the copy engines and raises its arrival flag; the root waits for every flag
// (from the host, then -- once they are in memory -- with the stream waits gathers use), checks
// every pattern, raises every rank's slot-free flag; each rank waits for its own the same two
// ways; all flags go back to 0.  Returns 1 when anything failed or timed out.
int ipc_handshake(rt_comm c) {
    constexpr uint64_t kMagic = 0x52545f4c494e4b31ull;
    const auto deadline = std::chrono::steady_clock::now() + std::chrono::seconds(20);
    const size_t n = std::min<size_t>(c->stage_bytes, 4096);
    hipError_t e = hipMemsetAsync(c->stage[0], (c->rank + 1) & 0xff, n, c->cstream);
    if (e == hipSuccess)
        e = hipMemcpyAsync(c->peer_parts[0] + (size_t)c->rank * c->stage_bytes, c->stage[0], n,
                           hipMemcpyDeviceToDeviceNoCU, c->cstream);
    if (e == hipSuccess) e = hipStreamWriteValue64(c->cstream, c->peer_rflags + 2 * c->rank, kMagic, 0);
    if (e != hipSuccess || !wait_until(c->cstream, deadline)) return 1;
    if (c->rank == c->root) {
        if (!poll_words(c->rflags, (size_t)c->nranks, 2, kMagic, deadline)) return 1;
        // the flags are in memory; the unpack stream's waits must see them too (the production path)
        for (int q = 0; q < c->nranks && e == hipSuccess; ++q)
            e = hipStreamWaitValue64(c->ustream, c->rflags + 2 * q, kMagic, hipStreamWaitValueGte, ~0ull);
        if (e != hipSuccess || !wait_until(c->ustream, deadline)) return 1;
        std::vector<uint8_t> got(n);
        for (int q = 0; q < c->nranks; ++q) {
            if (hipMemcpy(got.data(), static_cast<uint8_t*>(c->parts[0]) + (size_t)q * c->stage_bytes, n,
                          hipMemcpyDeviceToHost) != hipSuccess)
                return 1;
            for (uint8_t b : got)
                if (b != (uint8_t)((q + 1) & 0xff)) return 1;
        }
        for (int q = 0; q < c->nranks && e == hipSuccess; ++q)
            e = hipStreamWriteValue64(c->ustream, c->peer_sflags[q], kMagic, 0);
        if (e == hipSuccess) e = hipMemsetAsync(c->rflags, 0, 2 * sizeof(uint64_t) * c->nranks, c->ustream);
        if (e != hipSuccess || !wait_until(c->ustream, deadline)) return 1;
    }
    if (!poll_words(c->sflags, 1, 1, kMagic, deadline)) return 1;
    e = hipStreamWaitValue64(c->cstream, c->sflags, kMagic, hipStreamWaitValueGte, ~0ull);
    if (e != hipSuccess || !wait_until(c->cstream, deadline)) return 1;
    e = hipMemset(c->sflags, 0, 2 * sizeof(uint64_t));
    if (e == hipSuccess) e = hipDeviceSynchronize();
    return e == hipSuccess ? 0 : 1;
}
int link_ipc(rt_comm c) {
    hipError_t e = hipSetDevice(c->ctx->device);
    IpcBlob mine{};
    int bad = 0;
    if (e == hipSuccess) e = hipIpcGetMemHandle(&mine.sflags, c->sflags);
    if (e == hipSuccess && c->rank == c->root) {
        e = hipIpcGetMemHandle(&mine.parts[0], c->parts[0]);
        if (e == hipSuccess) e = hipIpcGetMemHandle(&mine.parts[1], c->parts[1]);
        if (e == hipSuccess) e = hipIpcGetMemHandle(&mine.rflags, c->rflags);
    }
    if (e != hipSuccess) bad = 1;
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
        if (bad) return;
        if (hipIpcOpenMemHandle(p, h, hipIpcMemLazyEnablePeerAccess) != hipSuccess) {
            bad = 1;
            *p = nullptr;
            return;
        }
        c->ipc_opened.push_back(*p);
    };
    int rc = exchange();
    if (!rc) {
        if (c->rank == c->root) {
            c->peer_parts[0] = static_cast<uint8_t*>(c->parts[0]);
            c->peer_parts[1] = static_cast<uint8_t*>(c->parts[1]);
            c->peer_rflags = c->rflags;
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
            open(all[c->root].parts[0], &p[0]);
            open(all[c->root].parts[1], &p[1]);
            open(all[c->root].rflags, &p[2]);
            c->peer_parts[0] = static_cast<uint8_t*>(p[0]);
            c->peer_parts[1] = static_cast<uint8_t*>(p[1]);
            c->peer_rflags = static_cast<uint64_t*>(p[2]);
        }
        // does every rank hold its links?
        rc = world_max(c, bad, &bad);
    }
    // the links hold: one small transfer and both flags across the world, polled from the host
    // with a deadline, before any gather relies on them (a world whose first real gather waited on
    // a flag that never arrives would hang instead of falling back)
    if (!rc && !bad) {
        bad = ipc_handshake(c);
        rc = world_max(c, bad, &bad);
    }
    if (rc) return rc;
    if (bad && !c->nc) return RT_INVALID_OPERATION;  // a shared world has no RCCL to fall back to
    if (bad) {  // the world falls back to RCCL transfers for this plan
        for (void* p : c->ipc_opened) (void)hipIpcCloseMemHandle(p);
        c->ipc_opened.clear();
        c->peer_parts[0] = c->peer_parts[1] = nullptr;
        c->peer_rflags = nullptr;
        c->peer_sflags.clear();
        c->ce = false;
        return RT_SUCCESS;
    }
    c->ce = c->ipc_linked = true;
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
int finish_gather(const rt_comm* comms, int n_local, int root, rt_mem root_dst, const rt_mem* outs);
int ce_gather(const rt_comm* comms, int n_local, int root, rt_mem root_dst, const rt_mem* outs);
int link_direct(const rt_comm* comms, int n_local, int root);
int link_ipc(rt_comm c);
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
    const int rc = comm_streams(c, false);
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
    if (transport == c->transport) return RT_SUCCESS;
    (void)hipSetDevice(c->ctx->device);
    (void)hipStreamSynchronize(c->cstream);
    (void)hipStreamSynchronize(c->ustream);
    (void)hipStreamSynchronize(c->ctx->astream);
    c->transport = transport;
    free_buffers(c);  // the next gather builds the plan for it
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
    for (int i = 0; i < n_local; ++i)  // coalesced per-frame launches first: the gather reads their output
        if (comms[i]->ctx->pend_k) (void)rti::flush_frames(comms[i]->ctx);
    // the plans (rebuilt, by every rank alike, when the size, the root or the transport changes)
    bool fresh = false;
    for (int i = 0; i < n_local; ++i) {
        hipError_t e = hipSetDevice(comms[i]->ctx->device);
        if (e != hipSuccess) return map_hip(e);
        bool built = false;
        int rc = ensure_plan(comms[i], W, H, root, &built);
        if (rc) return rc;
        fresh |= built;
    }
    if (fresh && comms[0]->transport != RT_COMM_TRANSPORT_RCCL) {
        int rc = RT_SUCCESS;
        if (comms[0]->transport == RT_COMM_TRANSPORT_COPY_ENGINES_IPC) {
            if (n_local != 1 || (!comms[0]->nc && comms[0]->fdir.empty())) return RT_INVALID_OPERATION;
            rc = link_ipc(comms[0]);
        } else if (n_local == comms[0]->nranks) {
            rc = link_direct(comms, n_local, root);  // every member is in this call
            if (rc && !comms[0]->group) {            // (RCCL world: keep RCCL's transfers)
                for (int i = 0; i < n_local; ++i) comms[i]->ce = false;
                rc = RT_SUCCESS;
            }
        } else if (n_local == 1 && (comms[0]->nc || !comms[0]->fdir.empty())) {
            rc = link_ipc(comms[0]);
        }
        if (rc) return rc;
    }
    bool ce = true;
    for (int i = 0; i < n_local; ++i) ce &= comms[i]->ce;
    // loopback and shared worlds move bytes on the copy engines only
    if ((comms[0]->group || !comms[0]->fdir.empty()) && !ce) return RT_INVALID_OPERATION;
    if (ce) return ce_gather(comms, n_local, root, root_dst, outs);
    // RCCL transport.  Phase 1: every rank (the root too) packs its bands on its context's
    // accumulation stream
    for (int i = 0; i < n_local; ++i) {
        rt_comm c = comms[i];
        rt_context ctx = c->ctx;
        hipError_t e = hipSetDevice(ctx->device);
        if (e != hipSuccess) return map_hip(e);
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

// `n` bytes on the copy engines, after and before everything on the communicator stream:
// chunks of at least 1 MiB over the transfer streams (several ranks driven by one process share
// its hardware queues, so they copy on the one stream)
hipError_t copy_engines(rt_comm c, uint8_t* dst, const uint8_t* src, size_t n) {
    const bool shared = !c->ipc_linked && c->nranks > 1;
    const size_t k = shared ? 1 : std::max<size_t>(1, std::min<size_t>(RT_COMM_XFER_STREAMS, n >> 20));
    if (k == 1) return hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToDeviceNoCU, c->cstream);
    const size_t chunk = ((n + k - 1) / k + 255) & ~(size_t)255;
    hipError_t e = hipEventRecord(c->xgo, c->cstream);
    for (size_t i = 0; i < k && e == hipSuccess; ++i) {
        const size_t off = i * chunk;
        if (off >= n) break;
        e = hipStreamWaitEvent(c->xstream[i], c->xgo, 0);
        if (e == hipSuccess)
            e = hipMemcpyAsync(dst + off, src + off, std::min(chunk, n - off), hipMemcpyDeviceToDeviceNoCU,
                               c->xstream[i]);
        if (e == hipSuccess) e = hipEventRecord(c->xdone[i], c->xstream[i]);
        if (e == hipSuccess) e = hipStreamWaitEvent(c->cstream, c->xdone[i], 0);
    }
    return e;
}

// Copy-engine gather (see the top of the file).  Between processes (IPC links), flags carry the
// gather's sequence number seq (1, 2, ... within a plan): rflags[q][s] = seq when rank q's bytes
// for slot s have landed in the root's receive slot, sflags[s] = seq when the root has unpacked
// slot s -- the next copy into that slot (gather seq + 2) waits for it.  Ranks driven by this
// process (loopback worlds, rtCommInitAll) order the same steps with events instead (the
// sender's `sent`, the root's `unpacked`): no waiting kernel on a hardware queue their other
// streams share.  Gathering into the root's own output, its own bands are in place: it neither
// packs nor sends them.
int ce_gather(const rt_comm* comms, int n_local, int root, rt_mem root_dst, const rt_mem* outs) {
    rt_comm R = nullptr;  // the root, when it is driven by this call
    for (int i = 0; i < n_local; ++i)
        if (comms[i]->rank == root) R = comms[i];
    for (int i = 0; i < n_local; ++i) {
        rt_comm c = comms[i];
        rt_context ctx = c->ctx;
        const int s = c->slot;
        const uint64_t seq = ++c->seq;
        const bool into_out = c->rank == root && (!root_dst || root_dst == outs[i]);
        hipError_t e = hipSetDevice(ctx->device);
        if (e == hipSuccess && !into_out) {
            // pack on the accumulation stream, after the accumulations (and main-stream work)
            // that write `out`, once the copy engine has read the slot's previous contents
            e = rti::main_tail_wait(ctx, ctx->astream);
            if (e == hipSuccess && c->sent_valid[s]) e = hipStreamWaitEvent(ctx->astream, c->sent[s], 0);
            if (e == hipSuccess)
                e = copy_rects(c->plans[c->rank], static_cast<uint8_t*>(outs[i]->dptr),
                               static_cast<uint8_t*>(c->stage[s]), true, ctx->astream);
            if (e == hipSuccess) e = hipEventRecord(c->packed[s], ctx->astream);
            if (e == hipSuccess) e = hipEventRecord(ctx->atail, ctx->astream);
            if (e == hipSuccess) ctx->apending = true;
            // transfer on the communicator stream: into the root's slot once the root has
            // unpacked what the slot held two gathers ago, then the arrival flag
            if (e == hipSuccess) e = hipStreamWaitEvent(c->cstream, c->packed[s], 0);
            if (c->ipc_linked) {
                if (e == hipSuccess && seq > 2)
                    e = hipStreamWaitValue64(c->cstream, c->sflags + s, seq - 2, hipStreamWaitValueGte, ~0ull);
            } else if (e == hipSuccess && R->unpacked_valid[s]) {
                e = hipStreamWaitEvent(c->cstream, R->unpacked[s], 0);
            }
            if (e == hipSuccess) e = copy_engines(c, c->peer_parts[s] + (size_t)c->rank * c->stage_bytes,
                                                  static_cast<const uint8_t*>(c->stage[s]), c->stage_bytes);
            if (e == hipSuccess && c->ipc_linked)
                e = hipStreamWriteValue64(c->cstream, c->peer_rflags + 2 * c->rank + s, seq, 0);
            if (e == hipSuccess) e = hipEventRecord(c->sent[s], c->cstream);
            if (e == hipSuccess) c->sent_valid[s] = true;
        }
        if (e != hipSuccess) return map_hip(e);
    }
    for (int i = 0; i < n_local; ++i) {
        rt_comm c = comms[i];
        rt_context ctx = c->ctx;
        const int s = c->slot;
        const uint64_t seq = c->seq;
        hipError_t e = hipSetDevice(ctx->device);
        hipStream_t tail = c->cstream;
        if (e == hipSuccess && c->rank == root) {
            // the root: wait for every sender's bytes, unpack them, free the slot for each sender
            const bool into_out = !root_dst || root_dst == outs[i];
            uint8_t* dst = static_cast<uint8_t*>((root_dst ? root_dst : outs[i])->dptr);
            if (c->ipc_linked) {
                for (int q = 0; q < c->nranks && e == hipSuccess; ++q)
                    if (!(into_out && q == c->rank))
                        e = hipStreamWaitValue64(c->ustream, c->rflags + 2 * q + s, seq, hipStreamWaitValueGte, ~0ull);
            } else {
                for (int j = 0; j < n_local && e == hipSuccess; ++j)
                    if (!(into_out && comms[j] == c)) e = hipStreamWaitEvent(c->ustream, comms[j]->sent[s], 0);
            }
            for (int q = 0; q < c->nranks && e == hipSuccess; ++q)
                if (!(into_out && q == c->rank))
                    e = copy_rects(c->plans[q], dst, static_cast<uint8_t*>(c->parts[s]) + (size_t)q * c->stage_bytes,
                                   false, c->ustream);
            for (int q = 0; c->ipc_linked && q < c->nranks && e == hipSuccess; ++q)
                if (!(into_out && q == c->rank)) e = hipStreamWriteValue64(c->ustream, c->peer_sflags[q] + s, seq, 0);
            if (e == hipSuccess) e = hipEventRecord(c->unpacked[s], c->ustream);
            if (e == hipSuccess) c->unpacked_valid[s] = true;
            tail = c->ustream;
        }
        // reads on this context wait for its part of the gather (qs)
        if (e == hipSuccess) e = hipEventRecord(ctx->gtail, tail);
        if (e != hipSuccess) return map_hip(e);
        ctx->gpending = true;
        c->slot ^= 1;
    }
    return RT_SUCCESS;
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
            // world-1 0.90 vs 0.77 ms/frame, profiles/r04/dist_flow_ab.txt.)  Reads of the
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

int rtBandPackPlan(unsigned width, unsigned height, unsigned period, unsigned phase, rt_rect* rects, int capacity,
                   int* n_rects, size_t* staging_bytes) {
    return band_plan(width, height, period, phase, rects, capacity, n_rects, staging_bytes);
}

}  // extern "C"
