// world_create_probe.cpp — where the cold cost of a fresh PathPlanner goes (diagnostics):
// times the HIP allocations epp_world_create makes (pinned records, pinned staging, the
// device blob, a stream) and whole epp_world_create / epp_world_destroy cycles of the C2
// world.  Build: hipcc -O2 -I include scripts/world_create_probe.cpp -Lefficient-path-planner_amd -lepp
//   -Wl,-rpath,$PWD/efficient-path-planner_amd -o scripts/world_create_probe
#include <hip/hip_runtime_api.h>

#include <chrono>
#include <cstdio>
#include <vector>

#include "epp.h"

static double us_since(std::chrono::steady_clock::time_point t0) {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
}

int main() {
    (void)hipSetDevice(0);
    (void)hipFree(nullptr);  // runtime init outside the timings
    auto t = std::chrono::steady_clock::now();
    for (int r = 0; r < 3; ++r) {
        void* p = nullptr;
        t = std::chrono::steady_clock::now();
        (void)hipHostMalloc(&p, 17408 * 2, hipHostMallocDefault);
        const double a = us_since(t);
        t = std::chrono::steady_clock::now();
        (void)hipHostFree(p);
        const double b = us_since(t);
        void* d = nullptr;
        t = std::chrono::steady_clock::now();
        (void)hipMalloc(&d, 100000);
        const double c = us_since(t);
        t = std::chrono::steady_clock::now();
        (void)hipFree(d);
        const double dd = us_since(t);
        hipStream_t s;
        t = std::chrono::steady_clock::now();
        (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
        const double e = us_since(t);
        t = std::chrono::steady_clock::now();
        (void)hipStreamDestroy(s);
        const double f = us_since(t);
        std::printf("hipHostMalloc %.1f us, hipHostFree %.1f, hipMalloc %.1f, hipFree %.1f, hipStreamCreate %.1f, "
                    "hipStreamDestroy %.1f\n", a, b, c, dd, e, f);
    }
    // a 64-box world of unit boxes
    std::vector<epp_obb> obbs(64);
    for (int i = 0; i < 64; ++i) {
        epp_obb& o = obbs[i];
        o = epp_obb{};
        o.center[0] = -5.0 + (i % 8) * 1.3;
        o.center[1] = -5.0 + (i / 8) * 1.3;
        o.center[2] = 1.0;
        o.half[0] = o.half[1] = 0.1;
        o.half[2] = 1.0;
        o.rot[0] = o.rot[4] = o.rot[8] = 1.0;
    }
    for (int r = 0; r < 4; ++r) {
        epp_world* w = nullptr;
        t = std::chrono::steady_clock::now();
        const epp_status rc = epp_world_create(obbs.data(), 64, 0.2, 0.2, &w);
        const double a = us_since(t);
        t = std::chrono::steady_clock::now();
        epp_world_destroy(w);
        std::printf("epp_world_create %.1f us (rc %d), epp_world_destroy %.1f us\n", a, (int)rc, us_since(t));
    }
    return 0;
}
