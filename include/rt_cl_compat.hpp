// rt_cl_compat.hpp -- header-only C++ face of librt_hip.so with the reference's shapes.
//
// A host written against the reference's device wrapper (CLutils.h:11-145) keeps its
// calls: CLContext::{ReadBuffer, ExecuteKernel, Finish, GetContext},
// CLKernel::SetArgument, RenderKernelArgument_t, CLException("msg (CL_NAME)").
// cl::Buffer becomes rtcl::Buffer (RAII over rt_mem); cl::Platform disappears (the
// context takes a GPU index).  Nothing here allocates device memory on its own.
#pragma once

#include <cstddef>
#include <cstdint>
#include <memory>
#include <stdexcept>
#include <string>

#include "rt_hip.h"
#include "rt_status.h"

namespace rtcl {

// CLutils.h:11-27
enum class RenderKernelArgument_t : unsigned int {
    BUFFER_OUT,
    BUFFER_SCENE,
    BUFFER_NODE,
    BUFFER_MATERIAL,
    WIDTH,
    HEIGHT,
    FRAME_COUNT,
    FRAME_SEED,
    LIGHT_BOUNCES,
    LIGHT_TYPE,
    SKYBOX_INTENSITY,
    CAMERA_POS,
    CAMERA_FRONT,
    CAMERA_UP
};

// CLutils.h:107-114
class CLException : public std::runtime_error {
public:
    CLException(const std::string& message, int errorCode)
        : std::runtime_error(message + " (" + rtGetErrorString(errorCode) + ")"), code(errorCode) {}
    int code;
};

inline void check(int rc, const char* what) {
    if (rc != RT_SUCCESS) throw CLException(what, rc);
}

class Buffer {
public:
    Buffer() = default;
    Buffer(rt_context ctx, uint64_t flags, size_t size, const void* host = nullptr) {
        check(rtCreateBuffer(ctx, flags, size, host, &mem_), "Failed to create buffer");
    }
    ~Buffer() { reset(); }
    Buffer(const Buffer&) = delete;
    Buffer& operator=(const Buffer&) = delete;
    Buffer(Buffer&& o) noexcept : mem_(o.mem_) { o.mem_ = nullptr; }
    Buffer& operator=(Buffer&& o) noexcept {
        if (this != &o) {
            reset();
            mem_ = o.mem_;
            o.mem_ = nullptr;
        }
        return *this;
    }
    rt_mem get() const { return mem_; }
    void reset() {
        if (mem_) rtReleaseBuffer(mem_);
        mem_ = nullptr;
    }

private:
    rt_mem mem_ = nullptr;
};

class CLKernel;

// CLutils.h:116-133
class CLContext {
public:
    explicit CLContext(int device = 0) { check(rtCreateContext(device, &ctx_), "Failed to create context"); }
    ~CLContext() {
        if (ctx_) rtReleaseContext(ctx_);
    }
    CLContext(const CLContext&) = delete;
    CLContext& operator=(const CLContext&) = delete;

    void ReadBuffer(const Buffer& buffer, void* ptr, size_t size) const {
        check(rtEnqueueReadBuffer(ctx_, buffer.get(), 0, 0, size, ptr), "Failed to read buffer");
    }
    inline void ExecuteKernel(std::shared_ptr<CLKernel> kernel, size_t workSize) const;
    void Finish() const { check(rtFinish(ctx_), "Failed to finish queue"); }
    rt_context GetContext() const { return ctx_; }

private:
    rt_context ctx_ = nullptr;
};

// CLutils.h:135-145
class CLKernel {
public:
    CLKernel(const CLContext& ctx, const char* name = "KernelEntry") {
        check(rtCreateKernel(ctx.GetContext(), name, &k_), "Failed to create kernel");
    }
    ~CLKernel() {
        if (k_) rtReleaseKernel(k_);
    }
    CLKernel(const CLKernel&) = delete;
    CLKernel& operator=(const CLKernel&) = delete;

    // Same contract as the reference: throws on failure, returns true otherwise.
    bool SetArgument(RenderKernelArgument_t argIndex, const void* data, size_t size) {
        check(rtSetKernelArg(k_, static_cast<unsigned>(argIndex), size, data),
              "Failed to set kernel argument");
        return true;
    }
    bool SetBuffer(RenderKernelArgument_t argIndex, const Buffer& b) {
        rt_mem m = b.get();
        return SetArgument(argIndex, &m, sizeof(m));
    }
    rt_kernel GetKernel() const { return k_; }

private:
    rt_kernel k_ = nullptr;
};

inline void CLContext::ExecuteKernel(std::shared_ptr<CLKernel> kernel, size_t workSize) const {
    check(rtEnqueueKernel(ctx_, kernel->GetKernel(), workSize), "Failed to enqueue kernel");
}

}  // namespace rtcl
