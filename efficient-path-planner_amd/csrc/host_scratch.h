// host_scratch.h — per-host-thread device staging used by the C++ API shims: one
// non-blocking stream and one growable HBM buffer per thread, so host-array calls
// from several threads (the reference plans two segments concurrently,
// src/OnlineTrajGenerator.cpp:324-340) never share a stream or a buffer.
#pragma once
#include <algorithm>
#include <cstddef>
#include <cstdint>
#include <stdexcept>
#include <string>

#include <hip/hip_runtime_api.h>

#include "epp.h"

namespace epp {

inline void check(epp_status rc, const char* what) {
    if (rc != EPP_OK) {
        const std::string msg = std::string(what) + ": " + epp_last_error();
        if (rc == EPP_ERR_INVALID_ARGUMENT) throw std::invalid_argument(msg);
        throw std::runtime_error(msg);
    }
}

class ThreadScratch {
public:
    static ThreadScratch& get() {
        thread_local ThreadScratch s;
        return s;
    }
    void* stream() {
        if (!stream_) check(epp_stream_create(&stream_), "stream");
        return stream_;
    }
    // A second stream for copies that overlap the first stream's kernels.
    void* copy_stream() {
        if (!cstream_) check(epp_stream_create(&cstream_), "stream");
        return cstream_;
    }
    // Device buffer of at least `bytes`, 256-byte aligned sub-allocations handed out
    // by `carve` until the next reset().
    void reset(size_t bytes) {
        bytes = (bytes + 255) & ~size_t(255);
        if (bytes > cap_) {  // (x2, at least 4 MB: freeing device memory synchronises the device)
            bytes = std::max(bytes, std::max<size_t>(2 * cap_, size_t(4) << 20));
            if (buf_) epp_free(buf_);
            buf_ = nullptr;
            cap_ = 0;
            check(epp_malloc(&buf_, bytes), "device scratch");
            cap_ = bytes;
        }
        used_ = 0;
    }
    void* carve(size_t bytes) {
        bytes = (bytes + 255) & ~size_t(255);
        if (used_ + bytes > cap_) throw std::runtime_error("device scratch overflow");
        void* p = static_cast<char*>(buf_) + used_;
        used_ += bytes;
        return p;
    }
    static size_t rounded(size_t bytes) { return (bytes + 255) & ~size_t(255); }
    // Pinned (page-locked) host staging of at least `bytes`, slot 0, 1 or 2: device-to-host
    // copies into it run at DMA speed instead of through a pageable bounce buffer.
    // Grows geometrically (x1.5) from 1 MB -- what the zero-copy path of a World query needs
    // at its largest (16,384 rays: 2 x 384 KB + 16 KB), so that path never reallocates:
    // reallocating pinned memory takes ~0.3 ms and synchronises the device (the second plan
    // of a generator paid it in its shortcut's checks).
    void* pinned(int slot, size_t bytes) {
        if (bytes > pcap_[slot]) {
            bytes = std::max(bytes, std::max<size_t>(pcap_[slot] + pcap_[slot] / 2, size_t(1) << 20));
            if (pin_[slot]) (void)hipHostFree(pin_[slot]);
            pin_[slot] = nullptr;
            pcap_[slot] = 0;
            if (hipHostMalloc(&pin_[slot], bytes, hipHostMallocDefault) != hipSuccess) {
                pin_[slot] = nullptr;
                throw std::runtime_error("pinned host staging: hipHostMalloc failed");
            }
            pcap_[slot] = bytes;
        }
        return pin_[slot];
    }
    ~ThreadScratch() {
        if (buf_) epp_free(buf_);
        for (void* p : pin_)
            if (p) (void)hipHostFree(p);
        if (stream_) epp_stream_destroy(stream_);
        if (cstream_) epp_stream_destroy(cstream_);
    }

private:
    void* stream_ = nullptr;
    void* cstream_ = nullptr;
    void* buf_ = nullptr;
    size_t cap_ = 0, used_ = 0;
    void* pin_[3] = {nullptr, nullptr, nullptr};
    size_t pcap_[3] = {0, 0, 0};
};

}  // namespace epp
