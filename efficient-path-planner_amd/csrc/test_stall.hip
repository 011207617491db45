// Test-hooks build only (testhooks/libepp.so, -DEPP_TEST_HOOKS): a kernel that holds a
// stream for a bounded time, so a collective queued behind it is "in flight" long enough
// for the communicator's deadline and abort paths (comm.cpp comm_wait) to be exercised on
// a one-GPU box.  The wait is bounded by the device's constant-rate wall clock: every
// launch ends by itself.
#include <hip/hip_runtime.h>

namespace epp {

__global__ void k_test_stall(unsigned long long ticks) {
    const unsigned long long t0 = wall_clock64();
    while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(127);
}

// Queues a stall of `ms` milliseconds (at most 10 s) on `stream`.
hipError_t test_stall(hipStream_t stream, double ms) {
    if (!(ms > 0.0)) return hipSuccess;
    if (ms > 10000.0) ms = 10000.0;
    int dev = 0, khz = 0;
    hipError_t he = hipGetDevice(&dev);
    if (he == hipSuccess) he = hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev);
    if (he != hipSuccess) return he;
    if (khz <= 0) khz = 100000;  // gfx9 constant clock: 100 MHz
    const unsigned long long ticks = (unsigned long long)(ms * (double)khz);
    hipLaunchKernelGGL(k_test_stall, dim3(1), dim3(64), 0, stream, ticks);
    return hipGetLastError();
}

}  // namespace epp
