// runtime.cpp — error state and thin HIP runtime wrappers of the C ABI (include/epp.h).
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>
#include <string>

#include "epp_internal.h"

namespace epp {
namespace {
thread_local std::string g_last_error;
}
void set_error(const std::string& msg) { g_last_error = msg; }
}  // namespace epp

#define EPP_HIP_RET(call)                                                            \
    do {                                                                             \
        hipError_t e_ = (call);                                                      \
        if (e_ != hipSuccess) {                                                      \
            epp::set_error(std::string(#call) + ": " + hipGetErrorString(e_));       \
            (void)hipGetLastError(); /* reported here: not again at the next launch */ \
            return EPP_ERR_HIP;                                                      \
        }                                                                            \
    } while (0)

extern "C" {

const char* epp_last_error(void) { return epp::g_last_error.c_str(); }
const char* epp_version(void) { return "epp-mi355x 0.1 (gfx950)"; }

epp_status epp_device_count(int* count) {
    EPP_HIP_RET(hipGetDeviceCount(count));
    return EPP_OK;
}
epp_status epp_set_device(int device) {
    EPP_HIP_RET(hipSetDevice(device));
    return EPP_OK;
}
epp_status epp_malloc(void** ptr, uint64_t bytes) {
    EPP_HIP_RET(hipMalloc(ptr, bytes ? bytes : 16));
    return EPP_OK;
}
epp_status epp_free(void* ptr) {
    if (ptr) EPP_HIP_RET(hipFree(ptr));
    return EPP_OK;
}
epp_status epp_memcpy_h2d(void* dst, const void* src, uint64_t bytes, void* stream) {
    if (!bytes) return EPP_OK;
    EPP_HIP_RET(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, (hipStream_t)stream));
    EPP_HIP_RET(hipStreamSynchronize((hipStream_t)stream));
    return EPP_OK;
}
epp_status epp_memcpy_d2h(void* dst, const void* src, uint64_t bytes, void* stream) {
    if (!bytes) return EPP_OK;
    EPP_HIP_RET(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, (hipStream_t)stream));
    EPP_HIP_RET(hipStreamSynchronize((hipStream_t)stream));
    return EPP_OK;
}
epp_status epp_memcpy_h2d_async(void* dst, const void* src, uint64_t bytes, void* stream) {
    if (!bytes) return EPP_OK;
    EPP_HIP_RET(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, (hipStream_t)stream));
    return EPP_OK;
}
epp_status epp_memcpy_d2h_async(void* dst, const void* src, uint64_t bytes, void* stream) {
    if (!bytes) return EPP_OK;
    EPP_HIP_RET(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, (hipStream_t)stream));
    return EPP_OK;
}
epp_status epp_memset(void* dst, int value, uint64_t bytes, void* stream) {
    if (!bytes) return EPP_OK;
    EPP_HIP_RET(hipMemsetAsync(dst, value, bytes, (hipStream_t)stream));
    return EPP_OK;
}
epp_status epp_stream_create(void** stream) {
    hipStream_t s;
    EPP_HIP_RET(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    *stream = s;
    return EPP_OK;
}
epp_status epp_stream_destroy(void* stream) {
    if (stream) EPP_HIP_RET(hipStreamDestroy((hipStream_t)stream));
    return EPP_OK;
}
epp_status epp_stream_sync(void* stream) {
    EPP_HIP_RET(hipStreamSynchronize((hipStream_t)stream));
    return EPP_OK;
}
epp_status epp_device_sync(void) {
    EPP_HIP_RET(hipDeviceSynchronize());
    return EPP_OK;
}
epp_status epp_event_create(void** event) {
    hipEvent_t e;
    EPP_HIP_RET(hipEventCreate(&e));
    *event = e;
    return EPP_OK;
}
epp_status epp_event_destroy(void* event) {
    if (event) EPP_HIP_RET(hipEventDestroy((hipEvent_t)event));
    return EPP_OK;
}
epp_status epp_event_record(void* event, void* stream) {
    EPP_HIP_RET(hipEventRecord((hipEvent_t)event, (hipStream_t)stream));
    return EPP_OK;
}
epp_status epp_event_elapsed_ms(void* start, void* stop, float* ms) {
    EPP_HIP_RET(hipEventSynchronize((hipEvent_t)stop));
    EPP_HIP_RET(hipEventElapsedTime(ms, (hipEvent_t)start, (hipEvent_t)stop));
    return EPP_OK;
}
void epp_host_free(void* p) { std::free(p); }

// Stream capture into a HIP graph: a captured sequence of stream-ordered epp_* calls is
// replayed with one host call (the kernels dispatch back to back, no per-launch host
// work in between).  Relaxed mode keeps the launchers' host-side queries legal.
epp_status epp_graph_begin(void* stream) {
    EPP_HIP_RET(hipStreamBeginCapture((hipStream_t)stream, hipStreamCaptureModeRelaxed));
    return EPP_OK;
}
epp_status epp_graph_end(void* stream, void** exec) {
    if (!exec) return EPP_ERR_INVALID_ARGUMENT;
    hipGraph_t g = nullptr;
    EPP_HIP_RET(hipStreamEndCapture((hipStream_t)stream, &g));
    hipGraphExec_t e = nullptr;
    const hipError_t err = hipGraphInstantiate(&e, g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    EPP_HIP_RET(err);
    EPP_HIP_RET(hipGraphUpload(e, (hipStream_t)stream));
    *exec = e;
    return EPP_OK;
}
epp_status epp_graph_launch(void* exec, void* stream) {
    EPP_HIP_RET(hipGraphLaunch((hipGraphExec_t)exec, (hipStream_t)stream));
    return EPP_OK;
}
epp_status epp_graph_destroy(void* exec) {
    if (exec) EPP_HIP_RET(hipGraphExecDestroy((hipGraphExec_t)exec));
    return EPP_OK;
}

}  // extern "C"
