/*
 * epp.h — C ABI of the MI355X-native Efficient-Path-Planner hot path.
 *
 * Plain pointers and sizes only; no torch / Eigen / OMPL types.  Every compute
 * entry point is stream-ordered on the hipStream_t passed as `void* stream`
 * (NULL = the null stream) and takes DEVICE pointers for bulk data (pinned host memory
 * from hipHostMalloc also works: the kernels then read / write it over the bus, which
 * the host-array paths use for small batches).  All
 * functions return an epp_status (0 = ok, < 0 = error); the message of the last
 * error on the calling thread is available from epp_last_error().
 *
 * Reference interfaces each entry point replaces (paths relative to the
 * reference repository root):
 *
 *   epp_world_create / epp_world_update
 *       World::addGate / addObstacle / updateGatePosition / resetWorld
 *       (include/World.h:27-56, src/World.cpp:13-78) — OBB table + AABB index
 *       (the Boost rtree `index`, include/World.h:109) uploaded to HBM.
 *   epp_check_states
 *       StateValidator::isValid (include/StateValidator.h:31, src/StateValidator.cpp:7-13)
 *       -> World::checkPointValidity(p, canPassGate) (src/World.cpp:80-104), batched.
 *   epp_check_states_mindist
 *       World::checkPointValidity(p, minDistance) (src/World.cpp:106-128) as used by
 *       PathPlanner::checkTrajectoryValidity (src/PathPlanner.cpp:267-280).
 *   epp_check_motions
 *       MotionValidator::checkMotion (include/MotionValidator.h:26, src/MotionValidator.cpp:8-17)
 *       -> World::checkRayValid (src/World.cpp:130-162), batched; mode 1 adds the
 *       32-step discretised check of BASELINE config 3.
 *   epp_minsnap_batch / epp_sample_count / epp_sample_batch
 *       poly_traj::generateTrajectory (external/poly_traj/include/poly_traj/trajectory_generator.h:20,
 *       external/poly_traj/src/trajectory_generator.cpp:12-100), batched over tracks.
 */
#ifndef EPP_H_
#define EPP_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef int32_t epp_status;
#define EPP_OK 0
#define EPP_ERR_INVALID_ARGUMENT (-1) /* std::invalid_argument in the reference */
#define EPP_ERR_RUNTIME (-2)          /* std::runtime_error in the reference */
#define EPP_ERR_HIP (-3)              /* HIP runtime error */
#define EPP_ERR_UNSUPPORTED (-4)      /* rotation other than about z (src/Object.cpp:38-47) */
#define EPP_ERR_CAPACITY (-5)         /* an output buffer was too small */
#define EPP_ERR_PEER (-6)             /* another rank of a collective reported a failure */
#define EPP_ERR_TIMEOUT (-7)          /* a collective did not complete within the communicator's timeout */

/* An oriented bounding box after the world build (reference class OBB,
 * include/OBB.h:19-57).  rot is the row-major rotation matrix; the reference only
 * produces rotations about z (src/Object.cpp:61-85) and so does this ABI. */
typedef struct epp_obb {
    double center[3];
    double half[3];
    double rot[9];
    int32_t filling; /* OBB::type == "filling" (else "collision") */
    int32_t is_gate; /* World key contains "gate": selects the gate inflate radius */
} epp_obb;

/* One OBB of a component's geometry (config `component_geometry.<comp>.<obb>`,
 * src/ConfigParserYAML.cpp:54-73): position relative to the component origin and
 * full size (the half size is size / 2). */
typedef struct epp_obb_desc {
    double pos[3];
    double size[3];
    int32_t filling; /* "filling" (1) or "collision" (0) */
    int32_t pad;
} epp_obb_desc;

typedef struct epp_world epp_world; /* opaque, bound to one device */

/* ---- runtime ---------------------------------------------------------------------- */
const char* epp_last_error(void);
const char* epp_version(void);
epp_status epp_device_count(int* count);
epp_status epp_set_device(int device);
epp_status epp_malloc(void** ptr, uint64_t bytes);
epp_status epp_free(void* ptr);
epp_status epp_memcpy_h2d(void* dst, const void* src, uint64_t bytes, void* stream);
epp_status epp_memcpy_d2h(void* dst, const void* src, uint64_t bytes, void* stream);
/* Stream-ordered copies that return without waiting (epp_memcpy_* above synchronise the
 * stream); the host side should be pinned (page-locked) memory and must stay
 * untouched until the stream is synchronised. */
epp_status epp_memcpy_h2d_async(void* dst, const void* src, uint64_t bytes, void* stream);
epp_status epp_memcpy_d2h_async(void* dst, const void* src, uint64_t bytes, void* stream);
epp_status epp_memset(void* dst, int value, uint64_t bytes, void* stream);
epp_status epp_stream_create(void** stream);
epp_status epp_stream_destroy(void* stream);
epp_status epp_stream_sync(void* stream);
epp_status epp_device_sync(void);
epp_status epp_event_create(void** event);
epp_status epp_event_destroy(void* event);
epp_status epp_event_record(void* event, void* stream);
epp_status epp_event_elapsed_ms(void* start, void* stop, float* ms);
/* Stream capture of stream-ordered epp_* calls into an instantiated HIP graph and its
 * replay (no counterpart in the reference: launch-overhead tool for batched callers,
 * e.g. bench.py's timed steps). */
epp_status epp_graph_begin(void* stream);
epp_status epp_graph_end(void* stream, void** exec);
epp_status epp_graph_launch(void* exec, void* stream);
epp_status epp_graph_destroy(void* exec);

/* ---- world ------------------------------------------------------------------------ */
/* World::addGate / World::addObstacle (src/World.cpp:13-55) via
 * Object::createFromDescription (src/Object.cpp:26-85), on the host.
 * gates: n_gates x 7 row-major (x, y, z, roll, pitch, yaw, type) — z is forced to 0
 * (src/PathPlanner.cpp:68); obstacles: n_obstacles x 6 (x, y, z, roll, pitch, yaw).
 * Gate type t uses gate_desc[gate_desc_off[t] .. gate_desc_off[t+1]).  Errors:
 * EPP_ERR_UNSUPPORTED for |roll| or |pitch| > 1e-6, EPP_ERR_RUNTIME for an object
 * centre z > 1e-6 or an unknown gate type, EPP_ERR_CAPACITY if out is too small
 * (*n_out then holds the required count). */
epp_status epp_build_obbs(const epp_obb_desc* gate_desc, const int32_t* gate_desc_off,
                          int32_t n_gate_types, const epp_obb_desc* obst_desc, int32_t n_obst_desc,
                          const double* gates, int32_t n_gates, const double* obstacles,
                          int32_t n_obstacles, epp_obb* out, int32_t capacity, int32_t* n_out);

/* Builds the AABB of every OBB (OBB::getAABB, src/OBB.cpp:93-123, inflated only for
 * "collision" OBBs by r_gate or r_obst) and a uniform cull grid over them, and
 * uploads both to the current device.  obbs is a HOST array. */
epp_status epp_world_create(const epp_obb* obbs, int32_t n_obbs, double r_gate, double r_obst,
                            epp_world** out);
/* Replaces the OBB set (gate-pose update = full rebuild, src/OnlineTrajGenerator.cpp:146).
 * Rebuilds the OBB records only, into the one of two pinned host slots that is not the
 * current version's (after the asynchronous small-query launches that read that slot
 * have finished; nothing else is waited for): small queries (<= 4096 states or 1024
 * edges on worlds of <= 256 OBBs) read those directly; the device index is rebuilt and
 * uploaded by the first call that needs it (or epp_world_build_index), after every kernel
 * that may read the old index, so an index error (e.g. too many distinct candidate
 * lists) is reported there.  Checks may run on other host threads meanwhile: each launch
 * uses the version of the index it finds (the one before or after the update, never a mix;
 * a rebuild waits until launches holding the old one are queued).  HIP graphs
 * that captured launches on this world must be re-captured afterwards, and only after
 * epp_world_build_index (launch shapes depend on the index; epp_world_generation
 * changes). */
epp_status epp_world_update(epp_world* w, const epp_obb* obbs, int32_t n_obbs);
/* Rebuilds and uploads the device index now if an update left it stale (synchronous;
 * not inside a stream capture). */
epp_status epp_world_build_index(const epp_world* w);
/* Number of versions of this world so far (create = 1, every update + 1). */
epp_status epp_world_generation(const epp_world* w, uint64_t* generation);
epp_status epp_world_destroy(epp_world* w);
epp_status epp_world_num_obbs(const epp_world* w, int32_t* n);
/* Host copy of the AABBs computed for the index (lo[3], hi[3] per OBB). */
epp_status epp_world_get_aabbs(const epp_world* w, double* lo_hi);

/* ---- collision checks (device pointers) ------------------------------------------- */
/* xyz: n x 3 f64 (AoS).  valid[i] = 1 if state i is collision free.  If compact_idx
 * is non-NULL, the indices of valid states are appended to it and *n_valid (device
 * int64, caller zeroes it) receives the count; the order of the compacted indices
 * is unspecified (wavefront order is preserved, inter-wavefront order is not). */
epp_status epp_check_states(const epp_world* w, const double* xyz, int64_t n, int32_t can_pass_gate,
                            uint8_t* valid, int32_t* compact_idx, int64_t* n_valid, void* stream);
epp_status epp_check_states_mindist(const epp_world* w, const double* xyz, int64_t n,
                                    double min_distance, uint8_t* valid, void* stream);
/* s1, s2: n x 3 f64.  mode 0 = analytic slab test (reference), 1 = discrete32:
 * points s1 + (s2 - s1) * (k/32), k = 1..32, each checked like epp_check_states. */
epp_status epp_check_motions(const epp_world* w, const double* s1, const double* s2, int64_t n,
                             int32_t can_pass_gate, int32_t mode, uint8_t* valid, void* stream);

/* ---- min-snap trajectory (device pointers) ---------------------------------------- */
/* Track k owns waypoints [wp_offsets[k], wp_offsets[k+1]) of wp (x,y,z f64) and
 * segments [wp_offsets[k]-k, wp_offsets[k+1]-k-1).  v0/a0: n_tracks x 3 (NULL = 0).
 * Outputs: seg_times (total segments), coeffs (total segments x 3 x 10, increasing
 * powers, the layout of mav_trajectory_generation::Polynomial).  status (n_tracks,
 * may be NULL): 0 ok, -1 fewer than 2 waypoints, -2 non-positive segment time,
 * -3 solver breakdown. */
epp_status epp_minsnap_batch(const double* wp, const int32_t* wp_offsets, int32_t n_tracks,
                             double v_max, double a_max, const double* v0, const double* a0,
                             double* seg_times, double* coeffs, int32_t* status, void* stream);
/* As epp_minsnap_batch with the caller's segment times instead of
 * estimateSegmentTimesNfabian: PolynomialOptimization<10>::setupFromVertices(vertices,
 * segment_times) (impl/polynomial_optimization_linear_impl.h:56-109), as the reference's
 * own tests call it (external/poly_traj/test/test_polynomial_optimization.cpp:765-769).
 * seg_times_in: total segments (device).  status -2 for a segment time <= 0. */
epp_status epp_minsnap_batch_times(const double* wp, const int32_t* wp_offsets, int32_t n_tracks, const double* v0,
                                   const double* a0, const double* seg_times_in, double* coeffs, int32_t* status,
                                   void* stream);
/* Number of rows Trajectory::evaluateRange produces for every track (device int64 out). */
epp_status epp_sample_count(const double* seg_times, const int32_t* wp_offsets, int32_t n_tracks,
                            double dt, int64_t* row_counts, void* stream);
/* rows: written at row_offsets[k] (device int64, exclusive scan of the counts), each
 * row [x,vx,ax,y,vy,ay,z,vz,az,t+t0[k]]; t0 may be NULL (= 0). */
epp_status epp_sample_batch(const double* seg_times, const double* coeffs,
                            const int32_t* wp_offsets, int32_t n_tracks, double dt, const double* t0,
                            const int64_t* row_offsets, double* rows, void* stream);

/* ---- batch planner building blocks (device pointers) ------------------------------- */
/* Replace OMPL's sampler / nearest-neighbour structure behind PathPlanner::planPath
 * (src/PathPlanner.cpp:80-158).  Counter-based uniform states in [lo, hi]:
 * u = (splitmix64(seed ^ (3 (start + i) + d)) >> 11) * 2^-53, x_d = lo_d + (hi_d - lo_d) u. */
epp_status epp_sample_uniform(uint64_t seed, const double lo[3], const double hi[3], int64_t n,
                              int64_t start, double* xyz, void* stream);
/* k nearest neighbours (k in {4, 8, 16, 32}) of every node within max_dist (<= 0: no
 * limit), sorted by distance, ties to the lower index; missing entries are -1. */
epp_status epp_knn(const double* nodes, int32_t n, int32_t k, double max_dist, int32_t* nbr, void* stream);
/* The two strategies behind epp_knn (same answers): all-pairs with LDS tiles, and a
 * uniform grid walked in shells. */
epp_status epp_knn_bruteforce(const double* nodes, int32_t n, int32_t k, double max_dist, int32_t* nbr,
                              void* stream);
epp_status epp_knn_grid(const double* nodes, int32_t n, int32_t k, double max_dist, int32_t* nbr, void* stream);
/* Caller-workspace variants (no allocation, no cross-stream ordering inside): `ws` is a
 * 256-byte aligned device buffer of at least epp_knn_workspace_size(n) bytes that no
 * other stream touches until this call's kernels completed.  Its prior contents do not
 * matter (the call clears what it reads before writing it).  epp_knn / epp_knn_grid
 * use a cached per-device workspace whose reuse is ordered by a completion event. */
uint64_t epp_knn_workspace_size(int32_t n);
epp_status epp_knn_ws(const double* nodes, int32_t n, int32_t k, double max_dist, int32_t* nbr, void* ws,
                      uint64_t ws_bytes, void* stream);
epp_status epp_knn_grid_ws(const double* nodes, int32_t n, int32_t k, double max_dist, int32_t* nbr, void* ws,
                           uint64_t ws_bytes, void* stream);
/* The same with the grid laid over the caller's box [lo, hi] (host arrays) instead of the
 * nodes' bounding box, which saves its device reduction (two kernels fewer): every node
 * must lie inside the closed box (the planner's samples lie in the world bounds; start and
 * goal widen them).  Same answers.  Precondition, not checked: a node outside the box is
 * clamped into a boundary cell, which breaks the search's distance bounds, and the table is
 * then unspecified (not necessarily exact). */
epp_status epp_knn_ws_box(const double* nodes, int32_t n, int32_t k, double max_dist, const double lo[3],
                          const double hi[3], int32_t* nbr, void* ws, uint64_t ws_bytes, void* stream);
epp_status epp_knn_grid_ws_box(const double* nodes, int32_t n, int32_t k, double max_dist, const double lo[3],
                               const double hi[3], int32_t* nbr, void* ws, uint64_t ws_bytes, void* stream);
/* Edge endpoints for every (node i, neighbour c): s1 = nodes[i], s2 = nodes[nbr[i k + c]]
 * (s2 = s1 for a missing neighbour).  s1, s2: n k x 3. */
epp_status epp_knn_edges(const double* nodes, const int32_t* nbr, int32_t n, int32_t k, double* s1,
                         double* s2, void* stream);
/* The motion checks of a k-NN table without materialising its edges: valid[e] for edge e
 * from node e / k to node nbr[e] (a missing neighbour, -1: the degenerate edge to itself),
 * as epp_check_motions on epp_knn_edges' output would give.  EPP_ERR_UNSUPPORTED when the
 * batch or world is not for the tile-filtered kernel (small batches, worlds without tile
 * tables): then use epp_knn_edges + epp_check_motions. */
epp_status epp_check_knn_motions(const epp_world* w, const double* nodes, const int32_t* nbr, int32_t n, int32_t k,
                                 int32_t can_pass_gate, int32_t mode, uint8_t* valid, void* stream);
/* Ordered stream compaction of the valid states (planner node list): out = xyz[i] for
 * valid[i] != 0, in index order; *n_out (device int64) = their count.  out holds n x 3. */
epp_status epp_compact_states(const double* xyz, const uint8_t* valid, int64_t n, double* out, int64_t* n_out,
                              void* stream);
/* Caller-workspace variant (ws: >= epp_compact_workspace_size(n) device bytes that no
 * other stream uses until this call's kernels completed; any prior contents: the call
 * zeroes its look-back status words first); epp_compact_states uses a
 * cached per-device workspace ordered by an event (serialising concurrent streams). */
uint64_t epp_compact_workspace_size(int64_t n);
epp_status epp_compact_states_ws(const double* xyz, const uint8_t* valid, int64_t n, double* out, int64_t* n_out,
                                 void* ws, uint64_t ws_bytes, void* stream);
/* nbr[e] = -1 where valid[e] == 0 (edges that failed the motion check), in place. */
epp_status epp_mask_edges(int32_t* nbr, const uint8_t* valid, int64_t m, void* stream);
/* The same, and count[0..1] (device memory, set by the call) = the entries of nbr that are
 * >= 0 afterwards and those equal to `target` (the planner's valid-edge statistic and the
 * goal's incoming edges, without a host pass over nbr). */
epp_status epp_mask_edges_count(int32_t* nbr, const uint8_t* valid, int64_t m, int32_t target, int64_t* count,
                                void* stream);

/* ---- multi-GPU: the multi-track plan's exchange step (RCCL over xGMI) --------------- */
/* BASELINE config 4 / SURVEY §8e: every rank (one GPU) plans its own track; the final
 * waypoint sets are then all-gathered.  No reference counterpart (the reference is
 * single-threaded CPU code).  RCCL is loaded at first use (librccl.so.1); without it these
 * return EPP_ERR_UNSUPPORTED.
 * One process per GPU: rank 0 calls epp_comm_unique_id and shares the 128 bytes out of
 * band (bench.py: a file rendezvous, eppamd/dist.py; or MPI, torch.distributed); every
 * rank calls epp_comm_init on its device.
 * One process, several GPUs: epp_comm_init_all (one communicator per device; use each
 * from its own host thread). */
typedef struct epp_comm epp_comm;
/* EPP_OK if RCCL can be loaded in this process (no communicator is created). */
epp_status epp_comm_available(void);
epp_status epp_comm_unique_id(uint8_t id[128]);
epp_status epp_comm_init(const uint8_t id[128], int32_t n_ranks, int32_t rank, epp_comm** out);
epp_status epp_comm_init_all(int32_t n_devices, const int32_t* devices, epp_comm** out /* n_devices */);
epp_status epp_comm_destroy(epp_comm* comm);
epp_status epp_comm_rank(const epp_comm* comm, int32_t* rank, int32_t* n_ranks);
/* Failure safety of every collective below: the call never blocks inside RCCL.  While its
 * collective runs it polls RCCL's asynchronous error state (a peer process died, a broken
 * connection), an abort requested with epp_comm_abort, and a deadline (default 120 s,
 * epp_comm_set_timeout).  On any of them it aborts the communicator (ncclCommAbort) and
 * returns EPP_ERR_PEER (error, abort) or EPP_ERR_TIMEOUT; every later call on that
 * communicator returns EPP_ERR_PEER at once (destroy it and create a new one).
 * epp_comm_abort may be called from any thread (e.g. by the owner of another rank's
 * communicator in the same process when that rank failed locally). */
epp_status epp_comm_set_timeout(epp_comm* comm, double seconds);
epp_status epp_comm_abort(epp_comm* comm);
/* All-gather of every rank's waypoint set (wp: n x 3 HOST doubles): counts[r] = rank r's
 * count (n_ranks entries), out + r * cap * 3 = its points (HOST, n_ranks x cap x 3).  Every
 * rank must call it, also a rank that has no set because its own work failed: it passes
 * n = -1 (wp may be NULL).  Every rank then returns EPP_ERR_PEER with counts filled (-1
 * marks the failed ranks) and the sets are not exchanged, so one rank's failure ends the
 * exchange on all ranks instead of leaving them in the collective.  EPP_ERR_CAPACITY
 * (counts filled, on every rank) if a rank has more than cap. */
epp_status epp_comm_allgather_waypoints(epp_comm* comm, const double* wp, int32_t n, int32_t cap, double* out,
                                        int32_t* counts);
/* x[0..n) (HOST doubles, in place) reduced over the ranks: op EPP_REDUCE_SUM / MAX / MIN.
 * The max-over-ranks timing and the collective error flags of a multi-rank caller. */
#define EPP_REDUCE_SUM 0
#define EPP_REDUCE_MAX 1
#define EPP_REDUCE_MIN 2
epp_status epp_comm_allreduce_f64(epp_comm* comm, double* x, int32_t n, int32_t op);
/* Returns once every rank has called it (an all-reduce of one double). */
epp_status epp_comm_barrier(epp_comm* comm);

/* ---- host-buffer convenience (synchronous; used by the C++ API shims) ------------- */
/* generateTrajectory for one track with host buffers (poly_traj::generateTrajectory,
 * external/poly_traj/src/trajectory_generator.cpp:12-100): one fused launch (min-snap
 * solve + evaluateRange sampling) reading and writing pinned host memory.  Returns the row
 * count in *n_rows; rows is allocated with malloc and must be released with
 * epp_host_free.  EPP_ERR_INVALID_ARGUMENT "At least two waypoints are required";
 * EPP_ERR_RUNTIME "Segment times need to be greater than zero" (the reference's glog
 * CHECK). */
epp_status epp_generate_trajectory_host(const double* wp, int32_t n_wp, double v_max, double a_max,
                                        double dt, double t0, const double v0[3], const double a0[3],
                                        double** rows, int64_t* n_rows);
/* The same with the caller's segment times (n_wp - 1 of them) instead of Nfabian's. */
epp_status epp_generate_trajectory_times_host(const double* wp, int32_t n_wp, const double* seg_times, double dt,
                                              double t0, const double v0[3], const double a0[3], double** rows,
                                              int64_t* n_rows);
/* The C5 online step's two GPU calls in ONE launch (an addition of this build; the
 * reference makes them one after the other: PathPlanner::checkTrajectoryValidity,
 * src/PathPlanner.cpp:267-280, then poly_traj::generateTrajectory, src/
 * OnlineTrajGenerator.cpp:374-379): check_valid[i] = World::checkPointValidity(check_xyz[i],
 * min_distance) (src/World.cpp:106-128) for the n_check points (HOST array, e.g. the
 * lookahead rows' positions) against `world`, and the trajectory of epp_generate_trajectory_host.
 * The check runs on extra workgroups of the refit's kernel: one pinned upload, one
 * completion poll.  Same answers as the two calls.  The check must be small (n_check <=
 * 4096, <= 256 OBBs), else EPP_ERR_UNSUPPORTED (make the two calls). */
epp_status epp_check_and_generate_trajectory_host(const epp_world* world, const double* check_xyz, int64_t n_check,
                                                  double min_distance, uint8_t* check_valid, const double* wp,
                                                  int32_t n_wp, double v_max, double a_max, double dt, double t0,
                                                  const double v0[3], const double a0[3], double** rows_out,
                                                  int64_t* n_rows);
/* The "optimal" trajectory type (OptimalTimeParametrizer::calculateTrajectory,
 * external/time_parametrization/src/OptimalTimeParametrizer.cpp:11-108; host code: one
 * sequential phase-plane integration).  wp: n_wp x 3, pre: n_pre x 3 lead-in points
 * (may be NULL when n_pre = 0).  rows: *n_rows x 11 [x vx ax y vy ay z vz az yaw t+t0],
 * malloc'd, release with epp_host_free.  EPP_ERR_RUNTIME "Trajectory is not valid" when
 * the integration fails. */
epp_status epp_optimal_trajectory_host(const double* wp, int32_t n_wp, const double* pre, int32_t n_pre,
                                       double v_max, double a_max, double dt, double t0, double max_deviation,
                                       double** rows, int64_t* n_rows);
/* The "spline" trajectory type (TrajInterpolation::interpolateTraj,
 * src/TrajInterpolation.cpp:44-68): cubic B-spline through wp (n_wp >= 4) at chord-length
 * parameters, int((max_t - t0) / dt) + 1 rows [x 0 0 y 0 0 z 0 0 t], t = i dt + t0;
 * malloc'd, release with epp_host_free. */
epp_status epp_spline_trajectory_host(const double* wp, int32_t n_wp, double max_t, double t0, double dt,
                                      double** rows, int64_t* n_rows);
void epp_host_free(void* p);

#ifdef __cplusplus
}
#endif

#endif /* EPP_H_ */
