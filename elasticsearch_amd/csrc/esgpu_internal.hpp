// esgpu_internal.hpp — pieces shared by the translation units of libesgpu.so (runtime, comm): the error model of the
// C-ABI, the device context with its HBM budget, and device / pinned buffers.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <mutex>
#include <stdexcept>
#include <string>

#include "../../include/esgpu.h"

// ------------------------------------------------------------------------------------------------------------
// errors
// ------------------------------------------------------------------------------------------------------------
inline thread_local std::string g_err;

struct EsError : std::runtime_error {
    int code;
    EsError(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

#define HIPX(expr)                                                                                            \
    do {                                                                                                      \
        hipError_t e_ = (expr);                                                                               \
        if (e_ != hipSuccess)                                                                                 \
            throw EsError(e_ == hipErrorOutOfMemory ? ESGPU_ERR_OOM : ESGPU_ERR_DEVICE,                       \
                          std::string(#expr) + ": " + hipGetErrorString(e_));                                \
    } while (0)

template <class F>
inline int guarded(F&& f) {
    try {
        f();
        return ESGPU_OK;
    } catch (const EsError& e) {
        g_err = e.what();
        return e.code;
    } catch (const std::bad_alloc&) {
        g_err = "host out of memory";
        return ESGPU_ERR_OOM;
    } catch (const std::exception& e) {
        g_err = e.what();
        return ESGPU_ERR_INVALID;
    }
}

inline void require(bool c, int code, const std::string& msg) {
    if (!c) throw EsError(code, msg);
}

// Shard results and reduces allocate multi-MB columnar arrays per request (57,700 buckets x 9 arrays for a north-star
// shard at 8 shards).  glibc serves those from fresh mmap'd pages (above its mmap threshold) or returns them to the OS
// by heap trimming, so every request paid a page fault per 4 KB touched: 2.1 ms to copy one shard's arrays into new
// vectors against 0.37 ms into recycled heap memory (measured on this build host).  The first context / reduce raises
// M_MMAP_THRESHOLD (32 MB, glibc's maximum) and M_TRIM_THRESHOLD (256 MB) once for the process, so freed result
// memory is reused; ESGPU_MALLOC_TUNE=0 leaves the host process's allocator settings alone.
void tune_host_heap();

// ------------------------------------------------------------------------------------------------------------
// context + HBM accounting (the REQUEST/FIELDDATA circuit breakers' analogue, BigArrays.java:393-395)
// ------------------------------------------------------------------------------------------------------------
struct esgpu_ctx {
    int device = 0;
    int cus = 256;
    uint64_t budget = 0;
    std::atomic<uint64_t> used{0};
    hipStream_t stream = nullptr;  // upload / generation stream
    std::mutex mu;
    // layout options (esgpu_ctx_set_option): compact columns, packed integer metric cells
    std::atomic<int> opt_compact{1}, opt_pi{1}, opt_hll_fs{1}, opt_b16{1};
    // synthetic tables (device copies)
    double* d_host_cdf = nullptr;
    double* d_rt_cdf = nullptr;
    double* d_url_cdf = nullptr;
};

struct DevBuf {
    esgpu_ctx* ctx = nullptr;
    void* p = nullptr;
    size_t bytes = 0;
    DevBuf() = default;
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
    DevBuf(DevBuf&& o) noexcept : ctx(o.ctx), p(o.p), bytes(o.bytes) { o.p = nullptr; o.bytes = 0; }
    DevBuf& operator=(DevBuf&& o) noexcept {
        if (this != &o) {
            release();
            ctx = o.ctx; p = o.p; bytes = o.bytes;
            o.p = nullptr; o.bytes = 0;
        }
        return *this;
    }
    ~DevBuf() { release(); }
    void release() {
        if (p) {
            (void)hipSetDevice(ctx->device);
            (void)hipFree(p);
            ctx->used -= bytes;
            p = nullptr;
            bytes = 0;
        }
    }
    void alloc(esgpu_ctx* c, size_t n) {
        release();
        ctx = c;
        if (n == 0) return;
        if (c->used + n > c->budget)
            throw EsError(ESGPU_ERR_OOM, "[request] Data too large: HBM budget of " + std::to_string(c->budget) +
                                             " bytes would be exceeded by " + std::to_string(n) + " bytes");
        HIPX(hipSetDevice(c->device));
        HIPX(hipMalloc(&p, n));
        bytes = n;
        c->used += n;
    }
    template <class T> T* as() const { return reinterpret_cast<T*>(p); }
};

// pinned host staging buffer (D2H of build results without a pageable bounce)
struct PinnedBuf {
    void* p = nullptr;
    void* dp = nullptr;  // the same memory as the device addresses it (kernels write build results straight into it)
    size_t bytes = 0;
    PinnedBuf() = default;
    PinnedBuf(const PinnedBuf&) = delete;
    PinnedBuf& operator=(const PinnedBuf&) = delete;
    PinnedBuf(PinnedBuf&& o) noexcept : p(o.p), dp(o.dp), bytes(o.bytes) { o.p = nullptr; o.dp = nullptr; o.bytes = 0; }
    PinnedBuf& operator=(PinnedBuf&& o) noexcept {
        if (this != &o) {
            if (p) (void)hipHostFree(p);
            p = o.p; dp = o.dp; bytes = o.bytes;
            o.p = nullptr; o.dp = nullptr; o.bytes = 0;
        }
        return *this;
    }
    ~PinnedBuf() { if (p) (void)hipHostFree(p); }
    void* ensure(size_t n) {
        if (n <= bytes) return p;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        dp = nullptr;
        bytes = 0;
        HIPX(hipHostMalloc(&p, n, hipHostMallocDefault));
        bytes = n;
        return p;
    }
    void* dev() {
        if (!dp && p) HIPX(hipHostGetDevicePointer(&dp, p, 0));
        return dp;
    }
    void release() {
        if (p) (void)hipHostFree(p);
        p = nullptr;
        dp = nullptr;
        bytes = 0;
    }
    template <class T> T* as() const { return reinterpret_cast<T*>(p); }
};

// device scratch that only grows: no hipMalloc/hipFree (and their implicit syncs) on the per-request path
struct Scratch {
    DevBuf buf;
    void* ensure(esgpu_ctx* c, size_t n) {
        if (n > buf.bytes) buf.alloc(c, n + n / 4);
        return buf.p;
    }
    template <class T> T* as() const { return buf.as<T>(); }
};


// the collectives of a communicator (esgpu_comm.cpp), for the device-resident reduce across ranks in the runtime
namespace esgpu {
struct Collective;
Collective& comm_collective(esgpu_comm* c);
}  // namespace esgpu
