// cached_ws.h — a per-device workspace that several streams / host threads may use in
// turn: a mutex serialises the host side, and every user's stream waits for the previous
// user's completion event before touching the buffer (so a buffer is never rewritten or
// freed while an earlier launch on another stream still reads it).
#pragma once
#include <hip/hip_runtime.h>

#include <mutex>
#include <string>

#include "epp_internal.h"

namespace epp {

struct CachedWs {
    std::mutex mu;
    void* buf = nullptr;
    size_t cap = 0;
    hipEvent_t done = nullptr;
    bool used = false;

    // Caller holds `mu`.  Orders `s` after the previous user and grows the buffer.
    hipError_t acquire(hipStream_t s, size_t bytes) {
        hipError_t e = hipSuccess;
        if (!done) e = hipEventCreateWithFlags(&done, hipEventDisableTiming);
        if (e == hipSuccess && used) e = hipStreamWaitEvent(s, done, 0);
        if (e == hipSuccess && bytes > cap) {
            // the previous user's kernels may still read the old buffer: wait for them
            if (used) e = hipEventSynchronize(done);
            if (e == hipSuccess && buf) e = hipFree(buf);
            buf = nullptr;
            cap = 0;
            if (e == hipSuccess) e = hipMalloc(&buf, bytes);
            if (e == hipSuccess) cap = bytes;
        }
        return e;
    }
    // Caller holds `mu`: marks the end of this user's work on `s`.
    void release(hipStream_t s) {
        if (hipEventRecord(done, s) == hipSuccess) used = true;
    }
};

}  // namespace epp
