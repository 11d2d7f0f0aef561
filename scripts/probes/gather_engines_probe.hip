// Probe: can the band gather move its bytes without compute units while a render holds them all?
//  1. a 132.7-MB device copy as hipMemcpyDeviceToDeviceNoCU (copy engine?) vs a plain D2D copy,
//     alone and beside a kernel that fills every CU slot for ~30 ms (does the copy finish first?);
//  2. hipStreamWriteValue64 / hipStreamWaitValue64 as cross-stream signals beside that kernel;
//  3. two processes on the one GPU: the child opens the parent's buffers by IPC handle, copies
//     its bytes into them with a no-CU copy and raises a flag there (hipStreamWriteValue64); the
//     parent's stream waits for the flag (hipStreamWaitValue64) and checks the bytes.
// usage: gather_engines_probe [ipc|split]   (prints one line per measurement; exits non-zero on a mismatch)
// The processes fork before either touches the GPU.
#include <hip/hip_runtime.h>
#include <signal.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/wait.h>
#include <unistd.h>

#define CK(x)                                                                            \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess) {                                                          \
            fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(2);                                                                     \
        }                                                                                \
    } while (0)

// fills every slot: 256 threads x many workgroups, fixed arithmetic per thread (bounded time)
__global__ __launch_bounds__(256) void busy(float* out, int iters) {
    float a = threadIdx.x * 1e-3f, b = 1.0001f;
    for (int i = 0; i < iters; ++i) a = a * b + 1e-7f;
    if (a == 12345.0f) out[blockIdx.x] = a;  // never true; keeps the loop
}

__global__ void fill_u32(uint32_t* p, size_t n, uint32_t v) {
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i < n) p[i] = v + (uint32_t)i;
}

static const size_t kBytes = 3840ull * 2160ull * 16ull;

static float ms_between(hipEvent_t a, hipEvent_t b) {
    float m = 0;
    CK(hipEventElapsedTime(&m, a, b));
    return m;
}

static int single_process() {
    CK(hipSetDevice(0));
    int can_wait = 0;
    (void)hipDeviceGetAttribute(&can_wait, hipDeviceAttributeCanUseStreamWaitValue, 0);
    printf("hipDeviceAttributeCanUseStreamWaitValue %d\n", can_wait);
    void *A, *B;
    float* junk;
    uint64_t* flag;
    CK(hipMalloc(&A, kBytes));
    CK(hipMalloc(&B, kBytes));
    CK(hipMalloc(&junk, 4096 * sizeof(float)));
    CK(hipMalloc(&flag, 64));
    CK(hipMemset(flag, 0, 64));
    fill_u32<<<(kBytes / 4 + 255) / 256, 256>>>((uint32_t*)A, kBytes / 4, 7u);
    CK(hipDeviceSynchronize());
    hipStream_t s1, s2;
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    hipEvent_t e0, e1, e2, e3;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventCreate(&e2));
    CK(hipEventCreate(&e3));
    // 1a. copies alone
    for (int kind = 0; kind < 2; ++kind) {
        const hipMemcpyKind k = kind ? hipMemcpyDeviceToDeviceNoCU : hipMemcpyDeviceToDevice;
        for (int rep = 0; rep < 3; ++rep) {
            CK(hipEventRecord(e0, s2));
            CK(hipMemcpyAsync(B, A, kBytes, k, s2));
            CK(hipEventRecord(e1, s2));
            CK(hipStreamSynchronize(s2));
        }
        printf("copy alone %-6s %.3f ms (%.1f GB/s)\n", kind ? "NoCU" : "D2D", ms_between(e0, e1),
               kBytes / (ms_between(e0, e1) * 1e-3) / 1e9);
    }
    // 1b. copies beside a kernel holding every slot
    int iters = 200000;
    for (int kind = 0; kind < 2; ++kind) {
        const hipMemcpyKind k = kind ? hipMemcpyDeviceToDeviceNoCU : hipMemcpyDeviceToDevice;
        CK(hipMemset(B, 0, kBytes));
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0, s1));
        busy<<<256 * 8 * 4, 256, 0, s1>>>(junk, iters);
        CK(hipEventRecord(e1, s1));
        usleep(2000);  // the busy kernel is resident
        CK(hipEventRecord(e2, s2));
        CK(hipMemcpyAsync(B, A, kBytes, k, s2));
        CK(hipEventRecord(e3, s2));
        CK(hipDeviceSynchronize());
        printf("beside busy %-6s busy %.3f ms, copy %.3f ms, copy ended %.3f ms after busy began (%s)\n",
               kind ? "NoCU" : "D2D", ms_between(e0, e1), ms_between(e2, e3), ms_between(e0, e3),
               ms_between(e0, e3) < ms_between(e0, e1) ? "before busy ended" : "after busy ended");
        if (memcmp("", "", 0)) return 3;
    }
    // 2. signals beside the busy kernel: s2 waits for flag >= 1, s1 (after a short kernel) writes it
    {
        CK(hipMemset(flag, 0, 64));
        CK(hipDeviceSynchronize());
        hipStream_t s3;
        CK(hipStreamCreateWithFlags(&s3, hipStreamNonBlocking));
        CK(hipEventRecord(e0, s1));
        busy<<<256 * 8 * 4, 256, 0, s1>>>(junk, iters);
        CK(hipEventRecord(e1, s1));
        usleep(2000);
        CK(hipStreamWaitValue64(s2, flag, 1, hipStreamWaitValueGte, ~0ull));
        CK(hipEventRecord(e2, s2));
        CK(hipMemcpyAsync(B, A, 4096, hipMemcpyDeviceToDeviceNoCU, s3));
        CK(hipStreamWriteValue64(s3, flag, 1, 0));
        CK(hipEventRecord(e3, s3));
        CK(hipDeviceSynchronize());
        printf("signal beside busy: writer done %.3f ms, waiter released %.3f ms after busy began; busy %.3f ms\n",
               ms_between(e0, e3), ms_between(e0, e2), ms_between(e0, e1));
    }
    return 0;
}

static int two_processes() {
    int to_child[2], to_parent[2];
    if (pipe(to_child) || pipe(to_parent)) return 4;
    pid_t pid = fork();
    if (pid < 0) return 4;
    if (pid == 0) {  // child: opens the parent's buffers, copies into them, raises the flag
        alarm(60);
        hipIpcMemHandle_t hb, hf;
        if (read(to_child[0], &hb, sizeof(hb)) != sizeof(hb) || read(to_child[0], &hf, sizeof(hf)) != sizeof(hf))
            _exit(5);
        CK(hipSetDevice(0));
        void *rb = nullptr, *rf = nullptr;
        CK(hipIpcOpenMemHandle(&rb, hb, hipIpcMemLazyEnablePeerAccess));
        CK(hipIpcOpenMemHandle(&rf, hf, hipIpcMemLazyEnablePeerAccess));
        void* A;
        CK(hipMalloc(&A, kBytes));
        fill_u32<<<(kBytes / 4 + 255) / 256, 256>>>((uint32_t*)A, kBytes / 4, 99u);
        hipStream_t s;
        CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        CK(hipDeviceSynchronize());
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        CK(hipEventRecord(e0, s));
        CK(hipMemcpyAsync(rb, A, kBytes, hipMemcpyDeviceToDeviceNoCU, s));
        CK(hipStreamWriteValue64(s, rf, 1, 0));
        CK(hipEventRecord(e1, s));
        CK(hipStreamSynchronize(s));
        printf("child: IPC no-CU copy + flag %.3f ms\n", ms_between(e0, e1));
        fflush(stdout);
        char ok = 1;
        if (read(to_child[0], &ok, 1) != 1) _exit(6);  // parent done before unmapping
        CK(hipIpcCloseMemHandle(rb));
        CK(hipIpcCloseMemHandle(rf));
        _exit(0);
    }
    alarm(60);
    CK(hipSetDevice(0));
    void* B;
    uint64_t* flag;
    CK(hipMalloc(&B, kBytes));
    // the flag word as fine-grained device memory when the runtime exports it by IPC (else plain)
    const bool fine = getenv("PROBE_FINE") != nullptr;
    if (fine)
        CK(hipExtMallocWithFlags((void**)&flag, 64, hipDeviceMallocFinegrained));
    else
        CK(hipMalloc(&flag, 64));
    printf("parent: flag memory %s\n", fine ? "fine-grained" : "hipMalloc");
    CK(hipMemset(B, 0, kBytes));
    CK(hipMemset(flag, 0, 64));
    CK(hipDeviceSynchronize());
    hipIpcMemHandle_t hb, hf;
    CK(hipIpcGetMemHandle(&hb, B));
    CK(hipIpcGetMemHandle(&hf, flag));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    // the wait is queued before the child has even started copying
    CK(hipStreamWaitValue64(s, flag, 1, hipStreamWaitValueGte, ~0ull));
    uint32_t* host = nullptr;
    CK(hipHostMalloc((void**)&host, kBytes, 0));
    CK(hipMemcpyAsync(host, B, kBytes, hipMemcpyDeviceToHost, s));
    if (write(to_child[1], &hb, sizeof(hb)) != sizeof(hb) || write(to_child[1], &hf, sizeof(hf)) != sizeof(hf)) return 4;
    CK(hipStreamSynchronize(s));
    size_t bad = 0;
    for (size_t i = 0; i < kBytes / 4; ++i) bad += host[i] != 99u + (uint32_t)i;
    printf("parent: waited on the child's flag, %zu of %zu words differ\n", bad, kBytes / 4);
    char ok = 1;
    if (write(to_child[1], &ok, 1) != 1) return 4;
    int st = 0;
    waitpid(pid, &st, 0);
    printf("child exit status %d\n", WIFEXITED(st) ? WEXITSTATUS(st) : -1);
    return bad ? 1 : (WIFEXITED(st) ? WEXITSTATUS(st) : 7);
}

// 4. one 132.7-MB no-CU copy split into k chunks on k streams: do the streams reach k engines?
static int split_copies() {
    CK(hipSetDevice(0));
    void *A, *B;
    CK(hipMalloc(&A, kBytes));
    CK(hipMalloc(&B, kBytes));
    hipStream_t st[16];
    for (int i = 0; i < 16; ++i) CK(hipStreamCreateWithFlags(&st[i], hipStreamNonBlocking));
    hipEvent_t e0, e1, ev[16];
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int i = 0; i < 16; ++i) CK(hipEventCreateWithFlags(&ev[i], hipEventDisableTiming));
    for (int k : {1, 2, 4, 8, 16}) {
        float best = 1e9f;
        for (int rep = 0; rep < 3; ++rep) {
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(e0, st[0]));
            const size_t chunk = (kBytes / k + 255) & ~(size_t)255;
            for (int i = 0; i < k; ++i) {
                if (i) CK(hipStreamWaitEvent(st[i], e0, 0));
                const size_t off = chunk * i, n = off >= kBytes ? 0 : (off + chunk > kBytes ? kBytes - off : chunk);
                if (n) CK(hipMemcpyAsync((char*)B + off, (char*)A + off, n, hipMemcpyDeviceToDeviceNoCU, st[i]));
                if (i) {
                    CK(hipEventRecord(ev[i], st[i]));
                    CK(hipStreamWaitEvent(st[0], ev[i], 0));
                }
            }
            CK(hipEventRecord(e1, st[0]));
            CK(hipEventSynchronize(e1));
            best = fminf(best, ms_between(e0, e1));
        }
        printf("no-CU copy in %2d chunks on %2d streams: %.3f ms (%.1f GB/s)\n", k, k, best, kBytes / (best * 1e-3) / 1e9);
    }
    return 0;
}

int main(int argc, char** argv) {
    if (argc > 1 && !strcmp(argv[1], "ipc")) return two_processes();
    if (argc > 1 && !strcmp(argv[1], "split")) return split_copies();
    return single_process();
}
