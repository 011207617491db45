// epp_internal.h — layouts shared by the host library and the HIP kernels.
//
// The world lives in HBM as one contiguous blob.  Its front part (what every state
// query touches) can be staged into LDS with straight 16-byte copies:
//
//   uint64  cell_mask[ncell]     occupancy of the 4x4x4 fine sub-cells of each coarse cell
//   uint32  cell_start[ncell+1]  CSR offsets of the coarse cells' OBB lists
//   -------------------------    (front: front_bytes)
//   uint16  cell_obb[...]        OBB ids per coarse cell
//   uint32  meta[n_pad]          bit0 filling, bit1 gate, bits 8-15/16-23/24-31 = first
//                                coarse cell (x, y, z) the OBB's AABB touches
//   double  soa[EPP_NF][n_pad]   field-major OBB table (see enum below)
//   double  aos[n_obb][17]       the OBB table again as 136-byte records (exact path)
//   uint32  hdr[n_lists]         candidate lists of the fine cells: start << 12 | count
//   uint16  ids[...]             the lists' OBB ids
//   uint8   cls8[ncells+1]       the fine-cell classes as bytes, when n_lists <= 256 (what
//                                k_states_v5 stages; else it stages the u16 cls[])
//   -------------------------    (everything above: staged into LDS by k_states_bm)
//   uint16  cls[ncells+1]        fine-cell class over the padded union box: 0 = outside
//                                every inflated AABB, else list index; the extra last
//                                entry is 0 (out-of-range lookups)
//   uint32  tiles[T*T][...]      motion filter (k_motions_v5): the xy extent split into
//                                T x T tiles, each with the OBBs whose slab-rounded AABB
//                                reaches it (<= 32 W, bit j = the tile's j-th OBB) and, per
//                                axis k and local slab s (S per tile and axis; z is not
//                                tiled), rows LE (bit set iff the OBB's AABB starts in a
//                                slab <= s) and GE (ends in a slab >= s), W words each, W+1
//                                words apart (an odd stride spreads a wave's row reads over
//                                the LDS banks); then rows FX / FY (the OBB's first tile
//                                along x / y is this one) and FILL (filling OBBs), and the
//                                tile's OBB ids (u16); tile_words words per tile
//
// n_pad rounds n_obbs up to a multiple of 4; every array starts 16-byte aligned.
#pragma once
#include <math.h>
#include <stdint.h>

#include <mutex>
#include <shared_mutex>
#include <string>
#include <vector>

#include <hip/hip_runtime_api.h>

#include "epp.h"

namespace epp {
// poly_traj::generateTrajectory of one track on the device (k_refit, minsnap.hip); the R
// sampled rows (R x 10 doubles) are copied into the buffer alloc(ctx, R) returns (NULL:
// out of memory).  times: the caller's segment times, or NULL for Nfabian's.
epp_status generate_trajectory_into(const double* wp, int32_t n_wp, const double* times, double v_max,
                                    double a_max, double dt, double t0, const double v0[3], const double a0[3],
                                    double* (*alloc)(void*, int64_t), void* ctx, int64_t* n_rows);
// The planner's pair of epp_sample_uniform + epp_compact_states_ws without the compaction's
// separate clearing launch: the sampler also zeroes the workspace's status words
// (clr_bytes: epp_compact_workspace_size), and the compaction that follows on the same
// stream trusts them to be zero.
epp_status sample_uniform_and_clear(uint64_t seed, const double lo[3], const double hi[3], int64_t n, double* xyz,
                                    void* clr, uint64_t clr_bytes, void* stream);
epp_status compact_states_cleared(const double* xyz, const uint8_t* valid, int64_t n, double* out, int64_t* n_out,
                                  void* ws, uint64_t ws_bytes, void* stream);
// The same with the C5 online step's A11 check fused into the launch (chk != NULL): the
// minDistance flags of chk->n points (host array) against chk->world, written to
// chk->valid, by extra workgroups of the refit's kernel (k_check_refit).  The check must be
// small (<= kSmallStates points, <= kSmallMaxObbs OBBs), else EPP_ERR_UNSUPPORTED.
struct FusedCheck {
    const epp_world* world;
    const double* xyz;
    int64_t n;
    double min_distance;
    uint8_t* valid;
};
epp_status check_and_generate_into(const FusedCheck* chk, const double* wp, int32_t n_wp, const double* times,
                                   double v_max, double a_max, double dt, double t0, const double v0[3],
                                   const double a0[3], double* (*alloc)(void*, int64_t), void* ctx, int64_t* n_rows);
// The planner's edge mask folded into the k-NN-table motion check (k_motions_v5, IDX):
// failed entries of nbr_w -> -1, out16 (optional) the masked table as u16, count[0] / [1]
// += kept edges / kept edges into node `target`.  count == nullptr: no mask.
struct MotionMask {
    int32_t* nbr_w = nullptr;
    uint16_t* out16 = nullptr;
    int32_t target = -1;
    unsigned long long* count = nullptr;
    // packed rows (the planner's row-restricted search): row r of the table is node
    // rowmap[r], and only rows r < *rows_n are checked
    const int32_t* rowmap = nullptr;
    const unsigned long long* rows_n = nullptr;
    // the planner batch (rows of several problems, node ids p << ns_log | node): mark[row's
    // node] and mark[each kept entry] = 1; per problem p the kept edges (pkept[p]) and those
    // into its node 1, the goal (pgoal[p]); nprob <= 64
    uint8_t* mark = nullptr;
    unsigned long long* pkept = nullptr;
    unsigned long long* pgoal = nullptr;
    int32_t ns_log = 0, nprob = 0;
};
// epp_check_knn_motions (mode 0) with the mask above; EPP_ERR_UNSUPPORTED as it (the
// caller then masks with mask_edges_count_acc).
epp_status check_knn_motions_masked(const epp_world* world, const double* nodes, int32_t* nbr, int32_t n, int32_t k,
                                    int32_t can_pass_gate, uint8_t* valid, uint16_t* out16, int32_t target,
                                    int64_t* count, void* stream);
// epp_mask_edges_count without clearing `count` first: the counts are added to what it
// holds (the planner clears them with its first upload).  out16 != NULL: also a copy of
// the masked table as u16, 0xFFFF for no edge (node counts <= 65535).
epp_status mask_edges_count_acc(int32_t* nbr, const uint8_t* valid, int64_t m, int32_t target, int64_t* count,
                                void* stream, uint16_t* out16 = nullptr);
// The planner's row-restricted search.  pack_ellipse_rows: the rows of the int32 k-NN table
// `tab` (n <= 65535 nodes x k) whose node x has |x - s| + |x - g| <= bound (widened by 1e-9
// relative + 1e-9 m), packed: ids32 / ids16[slot] = node, rows32[slot * k ..] = its row,
// *count += the rows found (slots >= cap are not written).
epp_status pack_ellipse_rows(const double* nodes, const int32_t* tab, int32_t n, int32_t k, const double s[3],
                             const double g[3], double bound, int32_t cap, int32_t* ids32, uint16_t* ids16,
                             int32_t* rows32, int64_t* count, void* stream);
// epp_knn_ws_box (max_dist 0) whose rows are exact for every node of that ellipsoid (the
// grid as usual, then those nodes' rows alone, one wave each; other rows: unspecified).
// The reverse edges of the masked k-NN table nbr (n x k, -1: none) as a CSR: roff (n + 1)
// and radj (the sources of every node's in-edges, ascending; radj16, if given, the same as
// u16); cnt / fill: n-int workspaces.  (PathPlanner's symmetrised search.)
epp_status reverse_csr(const int32_t* nbr, int32_t n, int32_t k, int32_t* cnt, int32_t* fill, int32_t* roff,
                       int32_t* radj, uint16_t* radj16, void* stream);
epp_status knn_ws_box_ellipse(const double* nodes, int32_t n, int32_t k, const double lo[3], const double hi[3],
                              const double s[3], const double g[3], double bound, int32_t* nbr, void* ws,
                              uint64_t ws_bytes, void* stream);
// check_knn_motions_masked over the packed rows: rows32 (cap rows x k, row r = node
// ids32[r]), rows r < min(*rows_n, cap) only; EPP_ERR_UNSUPPORTED for worlds without tile
// tables.  count == nullptr: the mask and out16 only (out16 = the entry's low 16 bits).
// marks (optional): its mark / pkept / pgoal / ns_log / nprob fields (the planner batch).
epp_status check_knn_motions_rows(const epp_world* world, const double* nodes, int32_t* rows32, const int32_t* ids32,
                                  const int64_t* rows_n, int32_t cap, int32_t k, int32_t can_pass_gate,
                                  uint8_t* valid, uint16_t* out16, int32_t target, int64_t* count, void* stream,
                                  const MotionMask* marks = nullptr);
// Whether check_knn_motions_rows can run on this world (its index current, rebuilt if
// stale): tile tables exist (slab_n > 0) and they, the records and the wave queues fit the
// LDS budget.  False for worlds without OBBs or past ~1000 OBBs: the planner then builds
// every problem's whole table instead of the restricted rows.
bool knn_motions_rows_supported(const epp_world* world);

// ---- the batched planner (PathPlanner::planPaths): a batch of gate-to-gate problems, one
// launch per device stage with blockIdx.y = the problem (planner.hip, plan_batch_launch).
// Stages: sample -> state check -> ordered compaction (start, goal, valid samples) -> the
// nodes inside each problem's grid ellipsoid |x - s| + |x - g| <= gbound into a small
// k-NN grid, those inside the row ellipsoid (<= bound) listed as queries -> their exact
// k-NN rows, one wave per query (exact because every node within the query's search
// radius lies in the grid ellipsoid: |x - s| + |x - g| is 2-Lipschitz; else the problem is
// flagged) -> the rows' motion checks (failed edges masked) -> the nodes the rows reference,
// numbered per problem in node order (0 = start, 1 = goal) -> one emit into pinned host
// memory.  Node counts stay on the device: no host round trip before the emit.
struct PlanSeg {                  // one problem (host -> device)
    uint64_t seed;                // the attempt's sampler seed
    double s[3], g[3];            // start, goal: nodes 0 and 1
    double bound;                 // rows: |x - s| + |x - g| <= bound
    double gbound;                // grid nodes: <= gbound (bound + a margin of cells)
    double glo[3], ghi[3];        // the grid's box (the gbound ellipsoid's box, clipped)
    double h;                     // the grid's cell edge
    int64_t row_off;              // first slot of its query list (rows: dense, see hdr)
    int64_t need_off;             // first slot of its referenced-node list
    int32_t cap;                  // query / row capacity (0: no restricted rows)
    int32_t need_cap;             // referenced-node list capacity
};
// Header words of the emitted results (u64): [1] rows (the problems' min(queries, cap),
// in problem order: problem p's rows follow those of problems < p), then per problem p:
// [3 + p] its queries (uncapped), [3 + S + p] kept edges of its rows, [3 + 2S + p] kept
// edges into its goal (node 1), [3 + 3S + p] its node count (valid samples + 2),
// [3 + 4S + p] its referenced nodes (compact indices 0 .. that - 1, in node order),
// [3 + 5S + p] nonzero: some query's exact rows needed nodes outside the grid ellipsoid.
enum : int { kPbRows = 1, kPbPerSeg = 3 };
struct PlanBatchLayout {
    int32_t S = 0, k = 0, ns_log = 0, nbc = 0, cap_total = 0, nctr = 0;
    int64_t ns = 0, NS = 0, need_cap = 0;  // samples per problem, node stride (2^ns_log >= 65536),
                                          // referenced-node slots of all problems
    // device workspace (bytes from its base, 256-B aligned parts)
    size_t o_seg = 0, o_ctr = 0, o_xyz = 0, o_valid = 0, o_nodes = 0, o_cstat = 0, o_kws = 0, kws_stride = 0,
           o_query = 0, o_ids32 = 0, o_rows32 = 0, o_rows16 = 0, o_ev = 0, o_mark = 0, o_map = 0, o_nstat = 0,
           o_need = 0, dev_bytes = 0;
    // pinned host block: the problems (uploaded), then the emitted header, per row its
    // problem and node (p << 16 | compact index), the masked rows (compact indices, 0xFFFF:
    // no edge) and each problem's referenced nodes (x, y, z at need_off + compact index)
    size_t h_seg = 0, h_hdr = 0, h_slot = 0, h_rows = 0, h_need = 0, h_done = 0, host_bytes = 0;
    int32_t done_n = 0;  // completion slots (u32 at h_done): the emit's workgroups publish the launch's seq
};
// segs: the problems with seed, ends, bound, gbound, the grid box and cell, cap filled;
// row_off / need_off / need_cap are filled in here
PlanBatchLayout plan_batch_layout(int32_t S, int64_t ns, int32_t k, PlanSeg* segs);
void plan_batch_trace_print();  // (EPP_PB_TRACE=1 diagnostics: the last batch's stage times)
epp_status plan_batch_launch(const epp_world* world, int32_t can_pass_gate, const double lo[3], const double hi[3],
                             const PlanBatchLayout& L, void* dev, void* host, uint32_t seq, void* stream);
}  // namespace epp

namespace epp {

// field index into the SoA table
enum Field : int {
    F_LOX = 0, F_LOY, F_LOZ, F_HIX, F_HIY, F_HIZ,  // AABB (rtree box, World.cpp:57-67)
    F_CX, F_CY, F_CZ,                              // OBB centre
    F_COS, F_SIN,                                  // R = [[c,-s,0],[s,c,0],[0,0,1]]
    F_HX, F_HY, F_HZ,                              // half sizes
    EPP_NF
};

// AoS OBB record of the fine-cell exact path: 17 doubles (136 B: consecutive records
// fall in different LDS banks), fields in the order of enum Field, meta bits in the last.
constexpr int kRecDoubles = 17;
constexpr int R_META = 16;

constexpr size_t kListMaxLen = 4095;  // OBBs per fine-cell list (12-bit count)
// LDS bytes k_states_v5 stages per workgroup (records, lists, class table): the class
// grid is coarsened until the world fits; the copy is register-staged, so this also
// bounds its per-lane registers (4 x 16 B at 1024 threads)
constexpr size_t kStageBudget = 64 * 1024;

constexpr uint32_t META_FILLING = 1u;
constexpr uint32_t META_GATE = 2u;
constexpr int kMaxGridAxis = 255;

// Passed to kernels by value.
struct WorldView {
    const unsigned char* blob;  // device pointer
    uint32_t blob_bytes;
    int32_t n_obb;
    int32_t n_pad;
    int32_t nx, ny, nz;
    uint32_t front_bytes;     // bytes of cell_mask + cell_start (16-byte multiple)
    uint32_t off_cell_mask;   // byte offsets inside the blob
    uint32_t off_cell_start;
    uint32_t off_cell_obb;
    uint32_t off_meta;
    uint32_t off_soa;
    double gx0, gy0, gz0;     // grid origin = min AABB lo
    double gx1, gy1, gz1;     // grid far corner = max AABB hi
    double icx, icy, icz;     // 1 / coarse cell size
    float ofx, ofy, ofz;      // grid origin rounded to float
    float i4x, i4y, i4z;      // 4 / coarse cell size, as float (fine-index scale)
    float limx, limy, limz;   // ~4n: fine coordinates beyond are outside every AABB
    float fmaxx, fmaxy, fmaxz; // 4 * n - 1: largest fine index
    double r_gate, r_obst;    // inflate radii (src/World.cpp:89-90)
    // fine cell classes (k_states fast path)
    uint32_t off_aos;         // OBB records (kRecDoubles each), then the lists
    uint32_t off_lists;       // list headers (u32: start << 12 | count)
    uint32_t off_ids;         // list OBB ids (u16)
    uint32_t n_lists;
    uint32_t off_bitmap;      // cls[] (u16 per fine cell)
    uint32_t bm_words;        // index of the zero sentinel class
    uint32_t off_cls8;        // the same classes as bytes (0: more than 255 lists, none) --
                              // sparse: u64 [occupancy | rank] per 32 cells, then the
                              // nonzero cells' bytes (world_index.cpp; dense with -DEPP_V5_DENSE_CLS)
    uint32_t cls8_bytes;      // bytes of that structure
    int32_t bnx, bny, bnz;    // cells per axis
    float bofx, bofy, bofz;   // offset: cell coordinate f = fmaf((float)p, bi, bof)
    float bix, biy, biz;      // 1 / cell size (float)
    // motion tile filter (slab_n = 0: none)
    uint32_t off_slab;
    int32_t slab_n;           // S = 1 << slab_log: local slabs per tile and axis
    int32_t slab_log;
    int32_t slab_w;           // W words of OBB bits per row (a power of two, <= 32)
    int32_t tile_n;           // T tiles per axis (x, y)
    uint32_t tile_words;      // words per tile (a multiple of 4)
    float sofx, sofy, sofz;   // global slab = (int)fmaf((float)p, si, sof), clamped to
    float six, siy, siz;      // [0, G-1], G = T S (x, y) or S (z); tile = slab >> slab_log
};

constexpr int kSlabMaxWords = 32;              // tiles of up to 1024 OBBs
constexpr size_t kSlabBudget = 40 * 1024;      // bytes of tile tables
constexpr size_t kSlabBudgetMax = 64 * 1024;   // ... when the records leave LDS room
constexpr size_t kMotionsLdsFree = 150 * 1024 - 16 * (256 * 4 + 64);  // k_motions_v5 LDS less its wave queues
// Words from one slab row of a tile to the next: the row width W rounded up to an odd
// number, so a wave's row gathers spread over all the LDS banks (an even stride would use
// half of them).
#if defined(__HIPCC__)
__host__ __device__
#endif
constexpr int slab_row_stride(int w) { return (w & 1) ? w : w + 1; }

// Global slab index along one axis: the same float operations on host and device, monotone in p
// (fmaf is correctly rounded), so an AABB overlap in doubles implies an overlap of the
// slab ranges (the filter is a superset of the rtree query).  NaN -> 0.
#if defined(__HIPCC__)
__host__ __device__
#endif
inline int slab_axis(double p, float off, float inv, int S) {
    float f = fmaf((float)p, inv, off);
    f = fminf(fmaxf(f, 0.0f), (float)(S - 1));
    return (int)f;
}

// Class-grid cell index along one axis: f = fmaf((float)p, inv, off), truncated.  The
// same float operations on host and device, so the host marks exactly the cells the
// kernels look up; monotone in p.  The grid keeps an empty margin cell at both ends of
// every axis (every AABB corner maps to [1, n-2]), so a kernel may clamp an
// out-of-range index to [0, n-1] (hardware cvt: NaN -> 0, saturating) instead of
// testing bounds: such states land in an empty cell, exactly like "outside".
#if defined(__HIPCC__)
__host__ __device__
#endif
inline int bm_axis(double p, float off, float inv) {
    float f = fmaf((float)p, inv, off);
    f = fminf(fmaxf(f, -1.0f), 16777216.0f);  // NaN -> -1 (outside); keeps (int) defined
    return (int)f;                             // truncation toward zero
}

// Host-side world: the upload plus host copies (for AABB introspection and rebuilds).
// epp_world_update only rebuilds the OBB records (into pinned host memory, which the
// small-query kernels read directly) and marks the device index stale; the index is
// rebuilt and uploaded by the first call that needs it (ensure_index).
struct HostWorld {
    WorldView view{};
    std::vector<epp_obb> obbs;          // the OBBs of the current version
    // Pinned records of the versions (n x kRecDoubles): two slots, the current version's
    // and the previous one's, so an update never rewrites records a kernel of the current
    // version may still read.  Kernels launched asynchronously on the host copy (the small
    // path while the index is stale) record an event per (slot, stream) after them; an
    // update waits for the slot's events before it reuses the slot.  (Polled host calls
    // have finished reading when they return.)
    struct RecReader {
        hipStream_t stream;
        hipEvent_t ev;
        bool pending;
    };
    double* h_recs = nullptr;           // = rec_buf[rec_slot]
    double* rec_buf[2] = {nullptr, nullptr};
    size_t rec_cap[2] = {0, 0};
    int rec_slot = 0;
    std::vector<RecReader> rec_readers[2];
    bool index_stale = false;           // the device blob is an older version
    std::mutex mu;                      // guards the lazy index rebuild
    // Held shared by a launcher from its snapshot of the device index or of the pinned
    // records until its kernel is queued (IndexLease, SmallWorld::lease), exclusively by a
    // rebuild and by epp_world_update: neither can free or rewrite the blob or a record slot
    // between another thread's snapshot and launch.
    // Lock order: index_mu, then mu.
    std::shared_mutex index_mu;
    WorldView dev_view{};               // `view` as uploaded (an update changes view.n_obb first)
    double r_gate = 0, r_obst = 0;
    int device = 0;
    void* d_blob = nullptr;
    const WorldView* d_view = nullptr;  // device copy of `view` (after the blob)
    size_t d_capacity = 0;
    void* h_stage = nullptr;            // pinned staging of the upload
    size_t h_capacity = 0;
    hipStream_t stream = nullptr;       // the upload's stream
    uint64_t generation = 0;            // uploads so far (epp_world_generation)
    std::string blob;            // host image of the device blob
    std::vector<double> aabbs;   // n x 6
};

// Fine (sub-cell) coordinate along one axis, computed in float with the same
// operations on host and device.  Every step is monotone in p, so the candidate lists
// and occupancy masks built from AABB corners are exact supersets of the rtree query
// results without any rounding slack.  A point strictly inside an AABB has
// 0 <= f <= 4n(1 + 3 * 2^-24) < lim; the fine index is F = min((int)f, 4n-1), coarse = F >> 2.
#if defined(__HIPCC__)
__host__ __device__
#endif
inline float fine_coord(double p, float o, float inv4) {
    return ((float)p - o) * inv4;
}
#if defined(__HIPCC__)
__host__ __device__
#endif
inline int fine_index(float f, int n) {
    const int nf = 4 * n;
    if (!(f >= 0.0f)) return 0;  // also catches NaN
    if (f >= (float)nf) return nf - 1;
    const int c = (int)f;        // f >= 0: truncation == floor
    return c < nf ? c : nf - 1;
}

void set_error(const std::string& msg);

// The OBB records of a world for the small-query kernels (brute force over every OBB):
// the device blob's when the index is current, else the pinned host copy (zero-copy).
struct SmallWorld {
    const double* recs;
    int32_t n_obb;
    double r_gate, r_obst;
    int host_slot;  // recs is the pinned host copy of this slot (index stale), else -1
    std::shared_lock<std::shared_mutex> lease;  // held until the launch reading recs is queued
};

// A launcher's snapshot of the device index (host view as uploaded + its device copy),
// valid while the lease is held: a rebuild on another thread waits for it.
struct IndexLease {
    std::shared_lock<std::shared_mutex> lk;
    WorldView view{};
    const WorldView* dview = nullptr;
};
// rebuild + upload a stale index (world_index.cpp); with a lease, the current index's
// snapshot, held until the lease is released (after the launch)
epp_status ensure_index(const epp_world* w, IndexLease* lease = nullptr);

}  // namespace epp
