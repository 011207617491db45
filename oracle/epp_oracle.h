/*
 * epp_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the Efficient-Path-Planner hot path, used as the parity
 * checker for the MI355X HIP path.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load this library.  The product path
 * (efficient-path-planner_amd/) never links or calls it.
 *
 * Pinning status:
 *   - min-snap half (A13–A19): pinned by the reference's own known-answer tests
 *     (TwoVerticesSetup golden coefficients, AMatrixInversion at 1e-10) and its
 *     property tests (checkPath continuity 1e-6, ConstraintPacking 1e-6) on the
 *     reference's own parameter sets, plus an independent numpy KKT restatement.
 *   - OBB / World half (A1–A9): "parity unpinned" against the reference binary —
 *     the reference needs Eigen/Boost/OMPL, absent here, and ships no World/OBB
 *     test.  It is a line-by-line restatement of src/OBB.cpp, src/World.cpp and
 *     src/Object.cpp with the operation order reasoned in DESIGN.md, checked
 *     against hand-derived boundary fixtures (tests/golden/obb_boundary.json).
 */
#pragma once
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* One OBB description inside a component (config.json component_geometry). */
typedef struct or_obb_desc {
    double pos[3];
    double size[3];
    int32_t filling; /* 0 = "collision", 1 = "filling" */
    int32_t pad;
} or_obb_desc;

/* One OBB after the world build (src/Object.cpp:52-85, src/OBB.cpp:93-123). */
typedef struct or_obb {
    double center[3];
    double half[3];
    double rot[9];     /* row-major R = Rz(yaw) (src/Object.cpp:72-83) */
    double aabb_lo[3]; /* rtree box, inflated only for "collision" */
    double aabb_hi[3];
    int32_t filling;   /* OBB::type == "filling" */
    int32_t is_gate;   /* key contains "gate" (src/World.cpp:89) */
} or_obb;

/* ---- world build (A9) ---------------------------------------------------- */
/* gates: G x 7 row-major (x,y,z,rx,ry,yaw,type); obstacles: O x 6.
 * gate_desc holds the OBB descriptions of every gate type, type t occupying
 * [gate_desc_off[t], gate_desc_off[t+1]).  Returns the number of OBBs written,
 * or a negative code: -1 out too small, -2 x/y rotation (Object.cpp:38-47),
 * -3 obstacle centre z > 1e-6 (Object.cpp:16-20), -4 unknown gate type. */
int or_world_build(const or_obb_desc* gate_desc, const int32_t* gate_desc_off, int n_gate_types,
                   const or_obb_desc* obst_desc, int n_obst_desc,
                   const double* gates, int n_gates, const double* obstacles, int n_obstacles,
                   double r_gate, double r_obst, or_obb* out, int max_out);

/* ---- collision queries (A1–A6) ------------------------------------------ */
int or_point_valid(const or_obb* w, int n, double r_gate, double r_obst, const double p[3],
                   int can_pass_gate);
int or_point_valid_mindist(const or_obb* w, int n, const double p[3], double min_distance);
int or_ray_valid(const or_obb* w, int n, double r_gate, double r_obst, const double s[3],
                 const double e[3], int can_pass_gate);

void or_check_states(const or_obb* w, int n, double r_gate, double r_obst, const double* xyz,
                     int64_t n_states, int can_pass_gate, uint8_t* valid);
void or_check_states_mindist(const or_obb* w, int n, const double* xyz, int64_t n_states,
                             double min_distance, uint8_t* valid);
/* mode 0 = analytic slab (World::checkRayValid), 1 = discrete32 */
void or_check_motions(const or_obb* w, int n, double r_gate, double r_obst, const double* s1,
                      const double* s2, int64_t n_edges, int can_pass_gate, int mode,
                      uint8_t* valid);
/* Same as or_check_states but split over n_threads std::threads (cpu baseline). */
void or_check_states_mt(const or_obb* w, int n, double r_gate, double r_obst, const double* xyz,
                        int64_t n_states, int can_pass_gate, uint8_t* valid, int n_threads);
void or_check_motions_mt(const or_obb* w, int n, double r_gate, double r_obst, const double* s1,
                         const double* s2, int64_t n_edges, int can_pass_gate, int mode,
                         uint8_t* valid, int n_threads);

/* ---- synthetic inputs ---------------------------------------------------- */
/* counter-based sampler: u = (splitmix64(seed ^ (3i+d)) >> 11) * 2^-53 */
void or_sample_states(uint64_t seed, const double lo[3], const double hi[3], int64_t n, double* xyz);

/* ---- min-snap (A13–A19) -------------------------------------------------- */
/* Nfabian segment times (src/vertex.cpp:272-289). */
void or_segment_times(const double* wp, int n_wp, int dim, double v_max, double a_max, double* times);
/* General PolynomialOptimization<10>::setupFromVertices + solveLinear.
 * fixed_mask[v*5+k] != 0 marks derivative k of vertex v as fixed with value
 * fixed_val[(v*5+k)*dim + d].  Coefficients out: seg x dim x 10 (increasing powers).
 * Returns n_free (>=0) or <0 on error (-1 bad time, -2 singular). */
int or_minsnap_solve(const uint8_t* fixed_mask, const double* fixed_val, int n_vertices, int dim,
                     const double* times, int derivative_to_optimize, double* coeffs);
/* poly_traj::generateTrajectory core: vertices from waypoints (start p,v0,a0,0,0; mids p;
 * end p,0,0,0,0), Nfabian times, solve.  coeffs: (W-1) x 3 x 10. */
int or_minsnap_track(const double* wp, int n_wp, double v_max, double a_max, const double v0[3],
                     const double a0[3], double* seg_times, double* coeffs);
/* A batch of independent tracks: track k = wp[off[k] .. off[k+1]) (v0 = a0 = 0) through
 * or_minsnap_track on nt threads; times at T + off[k] - k, coeffs at C + (off[k] - k) x 30,
 * status[k] its return value (the CPU baseline of BASELINE C5's batched refit). */
void or_minsnap_batch_mt(const double* wp, const int32_t* off, int n_tracks, double v_max, double a_max,
                         double* T, double* C, int32_t* status, int nt);
/* Trajectory::evaluateRange x3 -> rows x 10 [x,vx,ax,y,vy,ay,z,vz,az,t+t0].
 * Returns the number of rows (writes at most max_rows; call with rows=NULL to count). */
int64_t or_sample_traj(const double* seg_times, const double* coeffs, int n_seg, double dt,
                       double t0, double* rows, int64_t max_rows);
/* Full generateTrajectory (src/trajectory_generator.cpp:12-100). Returns rows or <0. */
int64_t or_generate_trajectory(const double* wp, int n_wp, double v_max, double a_max, double dt,
                               double t0, const double v0[3], const double a0[3], double* rows,
                               int64_t max_rows);

/* Mapping matrix (polynomial_optimization_linear_impl.h:111-121) and its Schur
 * inverse (:142-179); both 10x10 row-major. */
void or_mapping_matrix(double t, double* A);
void or_invert_mapping(const double* A, double* A_inv);
/* Evaluate derivative k of a 10-coefficient polynomial (polynomial.h:136-149). */
double or_poly_eval(const double* c, double t, int k);

/* createRandomVertices (src/vertex.cpp:27-82), std::mt19937 + uniform_real_distribution:
 * writes (n_segments+1) x dim positions. */
void or_random_vertices(int n_segments, int dim, double pos_min, double pos_max, uint64_t seed,
                        double* out);

/* ---- CPU restatement of this build's batch planner ------------------------- */
/* One attempt of PathPlanner::planOnce (efficient-path-planner_amd/csrc/host_planner.cpp)
 * on `threads` host threads: counter-RNG samples in [lo, hi], state checks, ordered
 * compaction (nodes = start, goal, valid samples), exact k-NN (ties to the lower index),
 * motion checks, A* (forward edges, then symmetrised), greedy shortcut.  Writes the path
 * (<= cap points) and returns its length, 0 if no path, -1 if cap is too small.
 * stats (may be NULL): samples, valid samples, edges, valid edges, 1 if the forward search
 * failed (the symmetrised search ran). */
int or_plan_once(const or_obb* w, int nw, double r_gate, double r_obst, const double lo[3], const double hi[3],
                 const double start[3], const double goal[3], int64_t samples, uint64_t seed, int k, int can_pass,
                 int threads, double* path, int cap, int64_t* stats);

#ifdef __cplusplus
}
#endif
