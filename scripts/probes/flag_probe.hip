// Probe: which cross-stream signalling forms complete while a kernel holds every CU slot?
// (The copy-engine gather must order copies and reads between processes without compute units.)
//  a. hipStreamWriteValue64 (ROCclr runs it as a kernel, __amd_rocclr_streamOpsWrite?)
//  b. an 8-byte hipMemcpyAsync NoCU from pinned host memory into fine-grained device memory
//  c. an 8-byte hipMemcpyAsync NoCU from device memory into fine-grained device memory
//  d. hipStreamWaitEvent on an event of another stream (a barrier packet?)
//  e. hipStreamWaitValue64 satisfied by (c) on another stream
// Each form runs on a high-priority stream beside `busy` (every slot, ~40 ms); the host timestamps
// when its completion event fires: before busy ends = no compute unit needed.
// usage: flag_probe   (one line per form)
#include <hip/hip_runtime.h>
#include <chrono>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x)                                                                            \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess) {                                                          \
            fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(2);                                                                     \
        }                                                                                \
    } while (0)

__global__ __launch_bounds__(256) void busy(float* out, int iters) {
    float a = threadIdx.x * 1e-3f, b = 1.0001f;
    for (int i = 0; i < iters; ++i) a = a * b + 1e-7f;
    if (a == 12345.0f) out[blockIdx.x] = a;
}

static double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// ms from t0 until `ev` completes (host polling)
static double wait_ms(hipEvent_t ev, double t0) {
    for (;;) {
        hipError_t q = hipEventQuery(ev);
        if (q == hipSuccess) return now_ms() - t0;
        if (q != hipErrorNotReady) {
            fprintf(stderr, "query %s\n", hipGetErrorString(q));
            exit(2);
        }
    }
}

int main() {
    CK(hipSetDevice(0));
    int least = 0, greatest = 0;
    CK(hipDeviceGetStreamPriorityRange(&least, &greatest));
    hipStream_t sb, s1, s2;
    CK(hipStreamCreateWithFlags(&sb, hipStreamNonBlocking));
    CK(hipStreamCreateWithPriority(&s1, hipStreamNonBlocking, greatest));
    CK(hipStreamCreateWithPriority(&s2, hipStreamNonBlocking, greatest));
    float* junk;
    uint64_t *fine, *dev, *host;
    CK(hipMalloc(&junk, 1 << 20));
    CK(hipExtMallocWithFlags(reinterpret_cast<void**>(&fine), 64, hipDeviceMallocFinegrained));
    CK(hipMalloc(&dev, 64));
    CK(hipHostMalloc(reinterpret_cast<void**>(&host), 64, 0));
    hipDeviceProp_t p;
    CK(hipGetDeviceProperties(&p, 0));
    const int grid = p.multiProcessorCount * 8;  // 8 x 256 threads per CU: every wave slot
    hipEvent_t eb, e1, e2;
    CK(hipEventCreate(&eb));
    CK(hipEventCreate(&e1));
    CK(hipEventCreate(&e2));
    const uint64_t v = 7;
    CK(hipMemcpy(dev, &v, 8, hipMemcpyHostToDevice));
    host[0] = 9;
    // warm every path once
    hipLaunchKernelGGL(busy, dim3(1), dim3(64), 0, sb, junk, 10);
    CK(hipStreamWriteValue64(s1, fine, 1, 0));
    CK(hipMemcpyAsync(fine, host, 8, hipMemcpyDeviceToDeviceNoCU, s1));
    CK(hipMemcpyAsync(fine, dev, 8, hipMemcpyDeviceToDeviceNoCU, s1));
    CK(hipDeviceSynchronize());
    const int iters = 400000;
    for (int form = 0; form < 5; ++form) {
        CK(hipMemset(fine, 0, 64));
        CK(hipDeviceSynchronize());
        hipLaunchKernelGGL(busy, dim3(grid), dim3(256), 0, sb, junk, iters);
        CK(hipEventRecord(eb, sb));
        const double t0 = now_ms();
        // give the busy kernel time to take every slot
        while (now_ms() - t0 < 2.0) {
        }
        const char* name = "";
        switch (form) {
            case 0: name = "hipStreamWriteValue64"; CK(hipStreamWriteValue64(s1, fine, 1, 0)); break;
            case 1: name = "8-B NoCU copy, pinned host -> fine-grained"; CK(hipMemcpyAsync(fine, host, 8, hipMemcpyDeviceToDeviceNoCU, s1)); break;
            case 2: name = "8-B NoCU copy, device -> fine-grained"; CK(hipMemcpyAsync(fine, dev, 8, hipMemcpyDeviceToDeviceNoCU, s1)); break;
            case 3: {
                name = "hipStreamWaitEvent on another high-priority stream's event";
                CK(hipMemcpyAsync(fine, dev, 8, hipMemcpyDeviceToDeviceNoCU, s2));
                CK(hipEventRecord(e2, s2));
                CK(hipStreamWaitEvent(s1, e2, 0));
                break;
            }
            case 4: {
                name = "hipStreamWaitValue64 met by an 8-B NoCU copy on another stream";
                CK(hipStreamWaitValue64(s1, fine, 7, hipStreamWaitValueGte, ~0ull));
                CK(hipMemcpyAsync(fine, dev, 8, hipMemcpyDeviceToDeviceNoCU, s2));
                break;
            }
        }
        CK(hipEventRecord(e1, s1));
        const double done = wait_ms(e1, t0);
        const double bend = wait_ms(eb, t0);
        uint64_t got = 0;
        CK(hipMemcpy(&got, fine, 8, hipMemcpyDeviceToHost));
        printf("%-64s done %8.3f ms, busy ended %8.3f ms -> %s (flag %llu)\n", name, done, bend,
               done < bend - 1.0 ? "NO CU NEEDED" : "waited for the busy kernel", (unsigned long long)got);
        CK(hipDeviceSynchronize());
    }
    return 0;
}
