// comm.cpp — the multi-track path's one exchange step over RCCL (xGMI): every rank plans
// its own track, then the final waypoint sets are all-gathered (the
// reference has no multi-GPU code).  RCCL is opened at first use (dlopen of the
// librccl next to the HIP runtime this library runs on), so the library does not depend
// on it unless the exchange is used.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "epp_internal.h"

namespace epp {
namespace {

struct Rccl {
    void* h = nullptr;
    decltype(&ncclGetUniqueId) getUniqueId = nullptr;
    decltype(&ncclCommInitRank) commInitRank = nullptr;
    decltype(&ncclCommInitAll) commInitAll = nullptr;
    decltype(&ncclCommDestroy) commDestroy = nullptr;
    decltype(&ncclAllGather) allGather = nullptr;
    decltype(&ncclAllReduce) allReduce = nullptr;
    decltype(&ncclGetErrorString) errorString = nullptr;
    decltype(&ncclCommGetAsyncError) getAsyncError = nullptr;
    decltype(&ncclCommAbort) commAbort = nullptr;
};

const Rccl* rccl() {
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        // The RCCL that belongs to the HIP runtime this library is bound to: the one in the
        // directory of the loaded libamdhip64 (ROCm's librccl.so.1, or PyTorch's bundled
        // librccl.so when PyTorch's runtime came first).  A process may hold both runtimes
        // (this library loaded before PyTorch): a bare dlopen("librccl.so.1") would then
        // return PyTorch's RCCL, whose runtime does not know this library's buffers
        // ("no ROCm-capable device").  RTLD_LOCAL: no symbol interposition either way.
        std::vector<std::string> names;
        Dl_info info;
        if (dladdr(reinterpret_cast<void*>(&hipGetDevice), &info) && info.dli_fname) {
            std::string dir(info.dli_fname);
            const size_t slash = dir.rfind('/');
            if (slash != std::string::npos) {
                dir.resize(slash + 1);
                names.push_back(dir + "librccl.so.1");
                names.push_back(dir + "librccl.so");
            }
        }
        for (const char* name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"}) names.push_back(name);
        for (const std::string& name : names) {
            r.h = dlopen(name.c_str(), RTLD_NOW | RTLD_LOCAL);
            if (r.h) break;
        }
        if (!r.h) return;
        r.getUniqueId = reinterpret_cast<decltype(r.getUniqueId)>(dlsym(r.h, "ncclGetUniqueId"));
        r.commInitRank = reinterpret_cast<decltype(r.commInitRank)>(dlsym(r.h, "ncclCommInitRank"));
        r.commInitAll = reinterpret_cast<decltype(r.commInitAll)>(dlsym(r.h, "ncclCommInitAll"));
        r.commDestroy = reinterpret_cast<decltype(r.commDestroy)>(dlsym(r.h, "ncclCommDestroy"));
        r.allGather = reinterpret_cast<decltype(r.allGather)>(dlsym(r.h, "ncclAllGather"));
        r.allReduce = reinterpret_cast<decltype(r.allReduce)>(dlsym(r.h, "ncclAllReduce"));
        r.errorString = reinterpret_cast<decltype(r.errorString)>(dlsym(r.h, "ncclGetErrorString"));
        r.getAsyncError = reinterpret_cast<decltype(r.getAsyncError)>(dlsym(r.h, "ncclCommGetAsyncError"));
        r.commAbort = reinterpret_cast<decltype(r.commAbort)>(dlsym(r.h, "ncclCommAbort"));
    });
    if (!r.h || !r.getUniqueId || !r.commInitRank || !r.commInitAll || !r.commDestroy || !r.allGather ||
        !r.allReduce || !r.errorString || !r.getAsyncError || !r.commAbort) {
        set_error("epp_comm: RCCL (librccl.so.1) is not available");
        return nullptr;
    }
    return &r;
}

epp_status nccl_error(const Rccl* r, ncclResult_t e, const char* what) {
    set_error(std::string(what) + ": " + r->errorString(e));
    return EPP_ERR_RUNTIME;
}

}  // namespace
}  // namespace epp

struct epp_comm {
    ncclComm_t comm = nullptr;
    int n_ranks = 0, rank = 0, device = 0;
    char* d_buf = nullptr;  // counts (n_ranks + 1 int32, padded) | send set | gathered sets
    size_t cap = 0;
    hipStream_t stream = nullptr;
    double timeout_s = 120.0;              // epp_comm_set_timeout
    std::atomic<bool> abort_req{false};    // epp_comm_abort (any thread)
    bool aborted = false;                  // ncclCommAbort ran: every later call fails
};

using namespace epp;

#ifdef EPP_TEST_HOOKS
namespace epp {
hipError_t test_stall(hipStream_t stream, double ms);  // csrc/test_stall.hip
}
#endif

namespace {

// EPP_TEST_COMM_STALL_MS (test builds only, -DEPP_TEST_HOOKS: testhooks/): a bounded
// stall queued on the communicator's stream just before each collective, so the
// collective is still in flight when the deadline passes or an abort is requested
// (tests/comm_stall_case.py).  The product build has no such hook.
hipError_t stall_hook(hipStream_t stream) {
#ifdef EPP_TEST_HOOKS
    if (const char* s = std::getenv("EPP_TEST_COMM_STALL_MS")) return test_stall(stream, std::atof(s));
#endif
    (void)stream;
    return hipSuccess;
}

// Binds the communicator's device and stream for one call (restores the caller's device).
struct CommScope {
    int prev = 0;
    hipError_t he = hipSuccess;
    explicit CommScope(epp_comm* c) {
        (void)hipGetDevice(&prev);
        (void)hipSetDevice(c->device);
        if (!c->stream) he = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    }
    ~CommScope() { (void)hipSetDevice(prev); }
};

hipError_t comm_grow(epp_comm* c, size_t need) {
    if (need <= c->cap) return hipSuccess;
    if (c->d_buf) (void)hipFree(c->d_buf);
    c->d_buf = nullptr;
    c->cap = 0;
    const hipError_t he = hipMalloc(&c->d_buf, need);
    if (he == hipSuccess) c->cap = need;
    return he;
}

epp_status hip_fail(const char* what, hipError_t he) {
    set_error(std::string(what) + ": " + hipGetErrorString(he));
    return EPP_ERR_HIP;
}

// Tears the communicator down without waiting for its peers: RCCL's kernels and proxy
// leave their collectives, the comm is unusable afterwards (epp_comm_destroy still frees
// the rest).
void do_abort(const Rccl* r, epp_comm* c) {
    if (c->aborted) return;
    if (c->comm) r->commAbort(c->comm);
    c->comm = nullptr;
    c->aborted = true;
}

epp_status aborted_error(const char* what) {
    set_error(std::string(what) + ": the communicator was aborted (a peer failed or timed out)");
    return EPP_ERR_PEER;
}

// Waits for the communicator's stream WITHOUT blocking in the runtime: the collective
// queued on it completes only if every peer takes part.  While it runs, RCCL's
// asynchronous error state (a peer process died, a broken connection) and an abort
// requested from another thread (epp_comm_abort) are polled; either, or the deadline
// (epp_comm_set_timeout), aborts the communicator, and the call returns an error instead
// of leaving this rank inside the collective.
epp_status comm_wait(const Rccl* r, epp_comm* c, const char* what) {
    const auto t0 = std::chrono::steady_clock::now();
    for (uint64_t spin = 0;; ++spin) {
        const hipError_t q = hipStreamQuery(c->stream);
        if (q == hipSuccess) return EPP_OK;
        if (q != hipErrorNotReady) return hip_fail(what, q);
        if ((spin & 63) != 63) {  // (a short spin first: the exchange is normally quick)
            std::this_thread::yield();
            continue;
        }
        ncclResult_t ae = ncclSuccess;
        if (c->comm) (void)r->getAsyncError(c->comm, &ae);
        if (ae != ncclSuccess && ae != ncclInProgress) {
            const std::string why = r->errorString(ae);
            do_abort(r, c);
            set_error(std::string(what) + ": RCCL asynchronous error (" + why + "): communicator aborted");
            return EPP_ERR_PEER;
        }
        if (c->abort_req.load()) {
            do_abort(r, c);
            return aborted_error(what);
        }
        const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (el > c->timeout_s) {
            do_abort(r, c);
            set_error(std::string(what) + ": no completion within " + std::to_string(c->timeout_s) +
                      " s (a peer did not take part): communicator aborted");
            return EPP_ERR_TIMEOUT;
        }
        std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
}

// A result copied to the caller's memory once its collective has completed (comm_wait):
// nothing is queued ahead of it on the stream, so the copy cannot wait on a peer, and no
// copy is left in flight into the caller's buffer when the call returns (an aborted
// collective returns before any copy is queued).
hipError_t copy_out(epp_comm* c, void* dst, const void* src, size_t bytes) {
    hipError_t he = hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, c->stream);
    if (he == hipSuccess) he = hipStreamSynchronize(c->stream);
    return he;
}

// Entry check of every collective: an aborted communicator (or one whose abort was
// requested before the call) fails at once.
epp_status comm_usable(const Rccl* r, epp_comm* c, const char* what) {
    if (!c->aborted && c->abort_req.load()) do_abort(r, c);
    return c->aborted ? aborted_error(what) : EPP_OK;
}

}  // namespace

extern "C" {

epp_status epp_comm_available(void) { return rccl() ? EPP_OK : EPP_ERR_UNSUPPORTED; }

epp_status epp_comm_unique_id(uint8_t id[128]) {
    if (!id) {
        set_error("epp_comm_unique_id: invalid argument");
        return EPP_ERR_INVALID_ARGUMENT;
    }
    const Rccl* r = rccl();
    if (!r) return EPP_ERR_UNSUPPORTED;
    ncclUniqueId u;
    const ncclResult_t e = r->getUniqueId(&u);
    if (e != ncclSuccess) return nccl_error(r, e, "ncclGetUniqueId");
    static_assert(sizeof(u) == 128, "ncclUniqueId is 128 bytes");
    std::memcpy(id, &u, 128);
    return EPP_OK;
}

epp_status epp_comm_init(const uint8_t id[128], int32_t n_ranks, int32_t rank, epp_comm** out) {
    if (!id || !out || n_ranks < 1 || rank < 0 || rank >= n_ranks) {
        set_error("epp_comm_init: invalid argument");
        return EPP_ERR_INVALID_ARGUMENT;
    }
    const Rccl* r = rccl();
    if (!r) return EPP_ERR_UNSUPPORTED;
    ncclUniqueId u;
    std::memcpy(&u, id, 128);
    epp_comm* c = new epp_comm();
    c->n_ranks = n_ranks;
    c->rank = rank;
    (void)hipGetDevice(&c->device);
    const ncclResult_t e = r->commInitRank(&c->comm, n_ranks, u, rank);
    if (e != ncclSuccess) {
        delete c;
        return nccl_error(r, e, "ncclCommInitRank");
    }
    *out = c;
    return EPP_OK;
}

epp_status epp_comm_init_all(int32_t n_devices, const int32_t* devices, epp_comm** out) {
    if (n_devices < 1 || !devices || !out) {
        set_error("epp_comm_init_all: invalid argument");
        return EPP_ERR_INVALID_ARGUMENT;
    }
    const Rccl* r = rccl();
    if (!r) return EPP_ERR_UNSUPPORTED;
    std::vector<ncclComm_t> comms(n_devices);
    std::vector<int> devs(devices, devices + n_devices);
    const ncclResult_t e = r->commInitAll(comms.data(), n_devices, devs.data());
    if (e != ncclSuccess) return nccl_error(r, e, "ncclCommInitAll");
    for (int i = 0; i < n_devices; ++i) {
        out[i] = new epp_comm();
        out[i]->comm = comms[i];
        out[i]->n_ranks = n_devices;
        out[i]->rank = i;
        out[i]->device = devices[i];
    }
    return EPP_OK;
}

epp_status epp_comm_destroy(epp_comm* c) {
    if (!c) return EPP_OK;
    int prev = 0;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(c->device);
    if (c->d_buf) (void)hipFree(c->d_buf);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    const Rccl* r = rccl();
    if (r && c->comm && !c->aborted) r->commDestroy(c->comm);
    (void)hipSetDevice(prev);
    delete c;
    return EPP_OK;
}

epp_status epp_comm_rank(const epp_comm* c, int32_t* rank, int32_t* n_ranks) {
    if (!c || !rank || !n_ranks) return EPP_ERR_INVALID_ARGUMENT;
    *rank = c->rank;
    *n_ranks = c->n_ranks;
    return EPP_OK;
}

epp_status epp_comm_set_timeout(epp_comm* c, double seconds) {
    if (!c || !(seconds > 0.0)) {
        set_error("epp_comm_set_timeout: invalid argument");
        return EPP_ERR_INVALID_ARGUMENT;
    }
    c->timeout_s = seconds;
    return EPP_OK;
}

epp_status epp_comm_abort(epp_comm* c) {
    if (!c) {
        set_error("epp_comm_abort: invalid argument");
        return EPP_ERR_INVALID_ARGUMENT;
    }
    c->abort_req.store(true);
    return EPP_OK;
}

epp_status epp_comm_allgather_waypoints(epp_comm* c, const double* wp, int32_t n, int32_t cap, double* out,
                                        int32_t* counts) {
    if (!c || n < -1 || cap < 0 || (n > 0 && !wp) || !counts || (cap > 0 && !out)) {
        set_error("epp_comm_allgather_waypoints: invalid argument");
        return EPP_ERR_INVALID_ARGUMENT;
    }
    const Rccl* r = rccl();
    if (!r) return EPP_ERR_UNSUPPORTED;
    if (const epp_status us = comm_usable(r, c, "epp_comm_allgather_waypoints")) return us;
    CommScope scope(c);
    hipError_t he = scope.he;
    const int R = c->n_ranks;
    const size_t cnt_b = ((size_t)(R + 1) * 4 + 255) & ~size_t(255);
    if (he == hipSuccess) he = comm_grow(c, cnt_b);
    // 1. the counts (-1: that rank failed before it had a set; every rank then stops here)
    if (he == hipSuccess) he = hipMemcpyAsync(c->d_buf, &n, 4, hipMemcpyHostToDevice, c->stream);
    if (he == hipSuccess) he = stall_hook(c->stream);
    if (he != hipSuccess) return hip_fail("epp_comm_allgather_waypoints", he);
    ncclResult_t e = r->allGather(c->d_buf, c->d_buf + 4, 1, ncclInt32, c->comm, c->stream);
    if (e != ncclSuccess) return nccl_error(r, e, "ncclAllGather (counts)");
    // the collective is waited for (polled, see comm_wait) BEFORE anything is copied to the
    // caller's memory: a device-to-host copy into pageable memory queued behind a hung
    // collective would block this thread inside the runtime, out of comm_wait's reach
    if (const epp_status ws = comm_wait(r, c, "ncclAllGather (counts)")) return ws;
    if ((he = copy_out(c, counts, c->d_buf + 4, (size_t)R * 4)) != hipSuccess)
        return hip_fail("epp_comm_allgather_waypoints", he);
    // every rank holds the same counts, so every rank takes the same branch below
    int32_t maxw = 0, failed = -1, n_failed = 0;
    for (int i = 0; i < R; ++i) {
        maxw = std::max(maxw, counts[i]);
        if (counts[i] < 0 && n_failed++ == 0) failed = i;
    }
    if (n_failed) {
        set_error("epp_comm_allgather_waypoints: " + std::to_string(n_failed) + " rank(s) reported a failure (first: rank " +
                  std::to_string(failed) + "; counts filled, -1 marks them)");
        return EPP_ERR_PEER;
    }
    if (maxw > cap) {
        set_error("epp_comm_allgather_waypoints: a rank has more waypoints than cap (counts filled)");
        return EPP_ERR_CAPACITY;
    }
    if (maxw == 0) return EPP_OK;
    // 2. the sets, padded to the longest (zeros after a rank's own points)
    const size_t set_b = (size_t)maxw * 24;
    he = comm_grow(c, cnt_b + set_b * (R + 1));
    char* d_send = c->d_buf + cnt_b;
    char* d_recv = d_send + set_b;
    if (he == hipSuccess) he = hipMemsetAsync(d_send, 0, set_b, c->stream);
    if (he == hipSuccess && n > 0) he = hipMemcpyAsync(d_send, wp, (size_t)n * 24, hipMemcpyHostToDevice, c->stream);
    if (he == hipSuccess) he = stall_hook(c->stream);
    if (he != hipSuccess) return hip_fail("epp_comm_allgather_waypoints", he);
    e = r->allGather(d_send, d_recv, (size_t)maxw * 3, ncclFloat64, c->comm, c->stream);
    if (e != ncclSuccess) return nccl_error(r, e, "ncclAllGather (waypoints)");
    if (const epp_status ws = comm_wait(r, c, "ncclAllGather (waypoints)")) return ws;
    for (int i = 0; i < R && he == hipSuccess; ++i)
        if (counts[i] > 0) he = copy_out(c, out + (size_t)i * cap * 3, d_recv + (size_t)i * set_b, (size_t)counts[i] * 24);
    if (he != hipSuccess) return hip_fail("epp_comm_allgather_waypoints", he);
    return EPP_OK;
}

epp_status epp_comm_allreduce_f64(epp_comm* c, double* x, int32_t n, int32_t op) {
    if (!c || n < 0 || (n > 0 && !x) || op < EPP_REDUCE_SUM || op > EPP_REDUCE_MIN) {
        set_error("epp_comm_allreduce_f64: invalid argument");
        return EPP_ERR_INVALID_ARGUMENT;
    }
    const Rccl* r = rccl();
    if (!r) return EPP_ERR_UNSUPPORTED;
    if (n == 0) return EPP_OK;
    if (const epp_status us = comm_usable(r, c, "epp_comm_allreduce_f64")) return us;
    CommScope scope(c);
    hipError_t he = scope.he;
    const size_t bytes = ((size_t)n * 8 + 255) & ~size_t(255);
    if (he == hipSuccess) he = comm_grow(c, bytes);
    if (he == hipSuccess) he = hipMemcpyAsync(c->d_buf, x, (size_t)n * 8, hipMemcpyHostToDevice, c->stream);
    if (he == hipSuccess) he = stall_hook(c->stream);
    if (he != hipSuccess) return hip_fail("epp_comm_allreduce_f64", he);
    const ncclRedOp_t rop = op == EPP_REDUCE_SUM ? ncclSum : op == EPP_REDUCE_MAX ? ncclMax : ncclMin;
    const ncclResult_t e = r->allReduce(c->d_buf, c->d_buf, (size_t)n, ncclFloat64, rop, c->comm, c->stream);
    if (e != ncclSuccess) return nccl_error(r, e, "ncclAllReduce");
    if (const epp_status ws = comm_wait(r, c, "ncclAllReduce")) return ws;
    if ((he = copy_out(c, x, c->d_buf, (size_t)n * 8)) != hipSuccess) return hip_fail("epp_comm_allreduce_f64", he);
    return EPP_OK;
}

epp_status epp_comm_barrier(epp_comm* c) {
    double x = 0.0;
    return epp_comm_allreduce_f64(c, &x, 1, EPP_REDUCE_SUM);
}

}  // extern "C"
