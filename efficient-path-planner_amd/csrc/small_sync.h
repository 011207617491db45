// small_sync.h — synchronous small queries for the host shims (host_world.cpp): the
// brute-force kernels of small.hip on pinned host arrays, waited for by polling the
// workgroups' completion flags instead of synchronising the stream.  *handled = false
// (nothing launched) when the query is not small (too many queries or OBBs).
#pragma once
#include <cstdint>

#include <hip/hip_runtime_api.h>

#include "epp.h"

namespace epp {
// can_pass of motions_small_sync / k_motions_small (mode 0; internal, never from the C ABI,
// which takes 0 / 1): each ray's flag byte holds both answers, bit 0 canPassGate = false,
// bit 1 true (World::checkRaysBoth)
constexpr int32_t kCanPassBoth = 2;
epp_status states_small_sync(const epp_world* world, bool mindist, const double* xyz, int64_t n, int32_t can_pass,
                             double md, uint8_t* valid, hipStream_t st, bool* handled);
epp_status motions_small_sync(const epp_world* world, int32_t mode, const double* s1, const double* s2, int64_t n,
                              int32_t can_pass, uint8_t* valid, hipStream_t st, bool* handled);
}  // namespace epp
