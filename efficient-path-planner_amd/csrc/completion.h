// completion.h — device side of the completion slots the synchronous host paths poll
// (small.hip, the refit kernels of minsnap.hip, k_pb_emit of planner.hip).
#pragma once
#include <hip/hip_runtime.h>

namespace epp {

// Before lane 0 of a workgroup publishes its completion with a system-scope release store:
// every wave waits until its own stores are acknowledged by the memory system
// (s_waitcnt vmcnt(0)), and the barrier orders them before that store, whose release (an
// L2 write-back of the XCD, then the store) covers them.  One system-scope release per
// workgroup instead of a __threadfence_system() per wave: k_motions_small at 1,024 edges
// (64 workgroups) 11.3 -> 7.5 us, one edge 5.4 -> 4.7 us (scripts/gpu_small_rays.sh).
__device__ __forceinline__ void wg_stores_settled() {
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
}

}  // namespace epp
