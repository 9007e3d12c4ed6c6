// Shared host/device helpers for libska_sdp_hip: error plumbing across the
// C ABI, the per-device scratch cache and small device utilities.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <stdexcept>
#include <string>

#include "ska_sdp_hip.h"

namespace sdp {

struct Error : std::runtime_error {
    int code;
    Error(int c, const std::string &m) : std::runtime_error(m), code(c) {}
};

#define SDP_HIP_CHECK(expr)                                                    \
    do {                                                                       \
        hipError_t e_ = (expr);                                                \
        if (e_ != hipSuccess)                                                  \
            throw ::sdp::Error(e_ == hipErrorOutOfMemory ? SDP_HIP_ERR_MEMORY  \
                                                         : SDP_HIP_ERR_RUNTIME,\
                               std::string(#expr) + ": " +                     \
                                   hipGetErrorString(e_));                     \
    } while (0)

#define SDP_REQUIRE(cond, msg)                                                 \
    do {                                                                       \
        if (!(cond))                                                           \
            throw ::sdp::Error(SDP_HIP_ERR_INVALID_ARG, std::string(msg));     \
    } while (0)

inline void write_err(char *buf, size_t len, const char *msg) {
    if (!buf || len == 0) return;
    std::snprintf(buf, len, "%s", msg);
}

// Run `fn` and translate exceptions into a status code + message.
template <class F>
int guarded(char *errbuf, size_t errlen, F &&fn) {
    try {
        fn();
        if (errbuf && errlen) errbuf[0] = 0;
        return SDP_HIP_OK;
    } catch (const Error &e) {
        write_err(errbuf, errlen, e.what());
        return e.code;
    } catch (const std::bad_alloc &) {
        write_err(errbuf, errlen, "host allocation failed");
        return SDP_HIP_ERR_MEMORY;
    } catch (const std::exception &e) {
        write_err(errbuf, errlen, e.what());
        return SDP_HIP_ERR_RUNTIME;
    }
}

// Per-device named scratch buffers that only ever grow.  Not used
// concurrently from several host threads on one device.
class Workspace {
   public:
    static Workspace &get() {
        static Workspace ws;
        return ws;
    }
    void *buffer(const std::string &name, size_t bytes) {
        int dev = 0;
        SDP_HIP_CHECK(hipGetDevice(&dev));
        std::lock_guard<std::mutex> lk(mu_);
        auto &b = bufs_[{dev, name}];
        if (b.bytes < bytes) {
            if (b.ptr) {
                ++gen_;  // an existing buffer moves
                SDP_HIP_CHECK(hipDeviceSynchronize());
                SDP_HIP_CHECK(hipFree(b.ptr));
                b.ptr = nullptr;
                b.bytes = 0;
            }
            // headroom against regrowth, capped so that the large plane and
            // record buffers do not take memory the call has budgeted elsewhere
            size_t want = bytes + std::min<size_t>(bytes / 8, (size_t)1 << 30) + 256;
            hipError_t e = hipMalloc(&b.ptr, want);
            if (e != hipSuccess) {
                (void)hipGetLastError();
                e = hipMalloc(&b.ptr, bytes);
                want = bytes;
            }
            if (e != hipSuccess) {
                (void)hipGetLastError();
                b.ptr = nullptr;
                throw Error(SDP_HIP_ERR_MEMORY,
                            "workspace '" + name + "': cannot allocate " +
                                std::to_string(bytes) + " bytes");
            }
            b.bytes = want;
            b.epoch = ++epoch_;
        }
        return b.ptr;
    }
    // identity of the allocation currently held under `name` (0: none): it
    // changes whenever that buffer is (re)allocated or released, so data a
    // caller left in it is known to be intact while the epoch is unchanged
    uint64_t epoch(const std::string &name) {
        int dev = 0;
        SDP_HIP_CHECK(hipGetDevice(&dev));
        std::lock_guard<std::mutex> lk(mu_);
        auto it = bufs_.find({dev, name});
        return it == bufs_.end() ? 0 : it->second.epoch;
    }
    // bytes currently held under `name` on the current device (0 if none)
    size_t held(const std::string &name) {
        int dev = 0;
        SDP_HIP_CHECK(hipGetDevice(&dev));
        std::lock_guard<std::mutex> lk(mu_);
        auto it = bufs_.find({dev, name});
        return it == bufs_.end() ? 0 : it->second.bytes;
    }
    // bumped whenever a buffer handed out before is freed (regrowth, release):
    // pointers kept across calls are valid while it is unchanged
    uint64_t generation() {
        std::lock_guard<std::mutex> lk(mu_);
        return gen_;
    }
    // free the buffer held under `name` on the current device (if any), so
    // that memory a plan does not use is not counted as reusable
    void drop(const std::string &name) {
        int dev = 0;
        SDP_HIP_CHECK(hipGetDevice(&dev));
        std::lock_guard<std::mutex> lk(mu_);
        auto it = bufs_.find({dev, name});
        if (it == bufs_.end() || !it->second.ptr) return;
        ++gen_;
        SDP_HIP_CHECK(hipDeviceSynchronize());
        SDP_HIP_CHECK(hipFree(it->second.ptr));
        bufs_.erase(it);
    }
    void release() {
        std::lock_guard<std::mutex> lk(mu_);
        ++gen_;
        if (!bufs_.empty()) (void)hipDeviceSynchronize();
        for (auto &kv : bufs_)
            if (kv.second.ptr) (void)hipFree(kv.second.ptr);
        bufs_.clear();
    }

   private:
    struct Buf {
        void *ptr = nullptr;
        size_t bytes = 0;
        uint64_t epoch = 0;
    };
    std::mutex mu_;
    uint64_t gen_ = 0;
    uint64_t epoch_ = 0;
    std::map<std::pair<int, std::string>, Buf> bufs_;
};

// Workspace slot of the calling NUFFT (0, or 1 under SDP_HIP_SLOT1): a second
// set of every named buffer, so that two inverts issued on two streams can
// run overlapped without sharing scratch memory.
inline int &ws_slot() {
    static thread_local int s = 0;
    return s;
}
inline std::string ws_name(const std::string &name) { return ws_slot() ? name + "#1" : name; }

template <class T>
T *scratch(const std::string &name, size_t count) {
    return static_cast<T *>(Workspace::get().buffer(ws_name(name), count * sizeof(T)));
}

inline hipStream_t as_stream(void *s) { return static_cast<hipStream_t>(s); }

inline unsigned grid1d(int64_t n, int block) {
    int64_t g = (n + block - 1) / block;
    return (unsigned)(g < 1 ? 1 : g);
}

}  // namespace sdp
