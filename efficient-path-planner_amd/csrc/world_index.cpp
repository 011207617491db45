// world_index.cpp — host side of the collision index: per-OBB AABBs (the Boost
// rtree boxes of the reference) and a uniform cull grid, packed into one HBM blob.
//
// Reference: OBB::getAABB (src/OBB.cpp:93-123), World::addObject (src/World.cpp:57-67).
// The rtree (include/Types.h:16, quadratic<16>) is replaced by a uniform grid whose
// cell lists are a superset of the boxes that can contain / intersect a query; the
// kernels then apply the rtree's exact predicate (strict `within` for points, closed
// `intersects` for ray boxes) to every candidate, so the candidate set equals the
// rtree's query result.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <string>
#include <vector>

#include "epp_internal.h"

namespace epp {
namespace {

// OBB::getAABB — src/OBB.cpp:93-123.  Corner order (:100-102) and the
// `rotation * corners + centerStacked` evaluation (:110) are kept; min/max are
// order independent.
void compute_aabb(const epp_obb& o, double inflate, double lo[3], double hi[3]) {
    static const double sx[8] = {-1, 1, 1, -1, -1, 1, 1, -1};
    static const double sy[8] = {-1, -1, 1, 1, -1, -1, 1, 1};
    static const double sz[8] = {-1, -1, -1, -1, 1, 1, 1, 1};
    for (int j = 0; j < 8; ++j) {
        const double c0 = sx[j] * o.half[0], c1 = sy[j] * o.half[1], c2 = sz[j] * o.half[2];
        for (int i = 0; i < 3; ++i) {
            const double g =
                ((o.rot[3 * i] * c0 + o.rot[3 * i + 1] * c1) + o.rot[3 * i + 2] * c2) + o.center[i];
            if (j == 0 || g < lo[i]) lo[i] = g;
            if (j == 0 || g > hi[i]) hi[i] = g;
        }
    }
    if (!o.filling) {  // only "collision" boxes are inflated (:117-121)
        for (int i = 0; i < 3; ++i) {
            lo[i] = lo[i] - inflate;
            hi[i] = hi[i] + inflate;
        }
    }
}

bool is_rz(const epp_obb& o) {
    const double* r = o.rot;
    return r[2] == 0.0 && r[5] == 0.0 && r[6] == 0.0 && r[7] == 0.0 && r[8] == 1.0 &&
           r[0] == r[4] && r[1] == -r[3];
}

inline size_t align16(size_t x) { return (x + 15) & ~size_t(15); }

// The OBB records of a new version (AABBs, kRecDoubles-double records with the filling /
// gate bits) into hw.aabbs and the pinned record slot other than the current one (the
// cheap part of an update); that slot becomes current.
bool build_records(HostWorld& hw, const epp_obb* obbs, int n) {
    for (int i = 0; i < n; ++i)
        if (!is_rz(obbs[i])) {  // (checked first: a failed update leaves the world as it was)
            set_error("epp_world: OBB rotation must be a rotation about z (src/Object.cpp:38-47)");
            return false;
        }
    const int slot = hw.h_recs ? 1 - hw.rec_slot : 0;
    for (auto& r : hw.rec_readers[slot])  // asynchronous kernels may still read this slot's version
        if (r.pending) {
            const hipError_t e = hipEventSynchronize(r.ev);
            if (e != hipSuccess) {
                set_error(std::string("epp_world: waiting for the readers of the records: ") + hipGetErrorString(e));
                return false;
            }
            r.pending = false;
        }
    const size_t need = std::max<size_t>(1, (size_t)n * kRecDoubles) * sizeof(double);
    if (need > hw.rec_cap[slot]) {
        if (hw.rec_buf[slot]) (void)hipHostFree(hw.rec_buf[slot]);
        hw.rec_buf[slot] = nullptr;
        hw.rec_cap[slot] = 0;
        const hipError_t e = hipHostMalloc(reinterpret_cast<void**>(&hw.rec_buf[slot]), need * 2, hipHostMallocDefault);
        if (e != hipSuccess) {
            set_error(std::string("epp_world: allocation: ") + hipGetErrorString(e));
            return false;
        }
        hw.rec_cap[slot] = need * 2;
    }
    double* recs = hw.rec_buf[slot];
    hw.aabbs.assign((size_t)n * 6, 0.0);
    for (int i = 0; i < n; ++i) {
        const epp_obb& o = obbs[i];
        double lo[3], hi[3];
        compute_aabb(o, o.is_gate ? hw.r_gate : hw.r_obst, lo, hi);  // src/World.cpp:89-90
        double* r = recs + (size_t)i * kRecDoubles;
        for (int k = 0; k < 3; ++k) {
            hw.aabbs[(size_t)i * 6 + k] = r[F_LOX + k] = lo[k];
            hw.aabbs[(size_t)i * 6 + 3 + k] = r[F_HIX + k] = hi[k];
            r[F_CX + k] = o.center[k];
            r[F_HX + k] = o.half[k];
        }
        r[F_COS] = o.rot[0];
        r[F_SIN] = o.rot[3];
        r[14] = r[15] = 0.0;
        const uint64_t m = (o.filling ? META_FILLING : 0u) | (o.is_gate ? META_GATE : 0u);
        std::memcpy(&r[R_META], &m, 8);
    }
    hw.obbs.assign(obbs, obbs + n);
    hw.view.n_obb = n;
    hw.rec_slot = slot;
    hw.h_recs = recs;
    return true;
}

// Builds the blob (layout in epp_internal.h).  Returns false with an error set.
bool build_blob(HostWorld& hw, const epp_obb* obbs, int n) {
    WorldView& v = hw.view;
    const int n_pad = (n + 3) & ~3;
    v.n_obb = n;
    v.n_pad = n_pad;
    hw.aabbs.assign((size_t)n * 6, 0.0);
    std::vector<double> soa((size_t)EPP_NF * n_pad, 0.0);
    std::vector<uint32_t> meta(n_pad, 0);
    double g0[3] = {0, 0, 0}, g1[3] = {0, 0, 0};
    for (int i = 0; i < n; ++i) {
        const epp_obb& o = obbs[i];
        if (!is_rz(o)) {
            set_error("epp_world: OBB rotation must be a rotation about z (src/Object.cpp:38-47)");
            return false;
        }
        const double r = o.is_gate ? hw.r_gate : hw.r_obst;  // src/World.cpp:89-90
        double lo[3], hi[3];
        compute_aabb(o, r, lo, hi);
        for (int k = 0; k < 3; ++k) {
            hw.aabbs[(size_t)i * 6 + k] = lo[k];
            hw.aabbs[(size_t)i * 6 + 3 + k] = hi[k];
            if (i == 0 || lo[k] < g0[k]) g0[k] = lo[k];
            if (i == 0 || hi[k] > g1[k]) g1[k] = hi[k];
        }
        double* f = soa.data();
        f[F_LOX * n_pad + i] = lo[0]; f[F_LOY * n_pad + i] = lo[1]; f[F_LOZ * n_pad + i] = lo[2];
        f[F_HIX * n_pad + i] = hi[0]; f[F_HIY * n_pad + i] = hi[1]; f[F_HIZ * n_pad + i] = hi[2];
        f[F_CX * n_pad + i] = o.center[0]; f[F_CY * n_pad + i] = o.center[1]; f[F_CZ * n_pad + i] = o.center[2];
        f[F_COS * n_pad + i] = o.rot[0];  // R(0,0) = cos
        f[F_SIN * n_pad + i] = o.rot[3];  // R(1,0) = sin
        f[F_HX * n_pad + i] = o.half[0]; f[F_HY * n_pad + i] = o.half[1]; f[F_HZ * n_pad + i] = o.half[2];
        meta[i] = (o.filling ? META_FILLING : 0u) | (o.is_gate ? META_GATE : 0u);
    }
    // ---- cull grid -------------------------------------------------------------
    int nd[3] = {1, 1, 1};
    double inv[3] = {0, 0, 0};
    if (n > 0) {
        double ext[3], vol = 1.0;
        for (int k = 0; k < 3; ++k) {
            ext[k] = g1[k] - g0[k];
            vol *= std::max(ext[k], 1e-3);
        }
        // ~2 coarse cells per OBB (each split into 4x4x4 occupancy sub-cells), capped.
        const double target = std::min(4096.0, std::max(32.0, 2.0 * n));
        const double s = std::cbrt(vol / target);
        for (int k = 0; k < 3; ++k) {
            nd[k] = ext[k] > 0 ? (int)std::ceil(ext[k] / s) : 1;
            nd[k] = std::max(1, std::min(kMaxGridAxis, nd[k]));
            inv[k] = ext[k] > 0 ? (double)nd[k] / ext[k] : 0.0;
        }
    }
    v.nx = nd[0]; v.ny = nd[1]; v.nz = nd[2];
    v.gx0 = g0[0]; v.gy0 = g0[1]; v.gz0 = g0[2];
    v.gx1 = g1[0]; v.gy1 = g1[1]; v.gz1 = g1[2];
    v.icx = inv[0]; v.icy = inv[1]; v.icz = inv[2];
    v.r_gate = hw.r_gate;
    v.r_obst = hw.r_obst;
    const float of[3] = {(float)g0[0], (float)g0[1], (float)g0[2]};
    const float i4[3] = {(float)(4.0 * inv[0]), (float)(4.0 * inv[1]), (float)(4.0 * inv[2])};
    v.ofx = of[0]; v.ofy = of[1]; v.ofz = of[2];
    v.i4x = i4[0]; v.i4y = i4[1]; v.i4z = i4[2];
    // fine coordinate of any point strictly inside an AABB is <= 4n (1 + 3 * 2^-24)
    v.limx = (float)(4 * nd[0]) * (1.0f + 0x1.0p-20f);
    v.limy = (float)(4 * nd[1]) * (1.0f + 0x1.0p-20f);
    v.limz = (float)(4 * nd[2]) * (1.0f + 0x1.0p-20f);
    v.fmaxx = (float)(4 * nd[0] - 1); v.fmaxy = (float)(4 * nd[1] - 1); v.fmaxz = (float)(4 * nd[2] - 1);
    const int ncell = nd[0] * nd[1] * nd[2];
    std::vector<uint64_t> mask(ncell, 0);
    std::vector<int> cbox((size_t)n * 6);  // per OBB: first / last coarse cell per axis
    for (int i = 0; i < n; ++i) {
        const double* lo = &hw.aabbs[(size_t)i * 6];
        const double* hi = lo + 3;
        int f0[3], f1[3];
        for (int k = 0; k < 3; ++k) {
            f0[k] = fine_index(fine_coord(lo[k], of[k], i4[k]), nd[k]);
            f1[k] = fine_index(fine_coord(hi[k], of[k], i4[k]), nd[k]);
            cbox[(size_t)i * 6 + k] = f0[k] >> 2;
            cbox[(size_t)i * 6 + 3 + k] = f1[k] >> 2;
        }
        meta[i] |= ((uint32_t)(f0[0] >> 2) << 8) | ((uint32_t)(f0[1] >> 2) << 16) |
                   ((uint32_t)(f0[2] >> 2) << 24);
        for (int z = f0[2]; z <= f1[2]; ++z)
            for (int y = f0[1]; y <= f1[1]; ++y)
                for (int x = f0[0]; x <= f1[0]; ++x) {
                    const size_t c = ((size_t)(z >> 2) * nd[1] + (y >> 2)) * nd[0] + (x >> 2);
                    mask[c] |= 1ull << (((z & 3) * 4 + (y & 3)) * 4 + (x & 3));
                }
    }
    // coarse cell lists (CSR, ascending OBB id): count, scan, scatter
    std::vector<uint32_t> cell_start(ncell + 1, 0);
    auto for_coarse = [&](int i, auto&& fn) {
        const int* b = &cbox[(size_t)i * 6];
        for (int z = b[2]; z <= b[5]; ++z)
            for (int y = b[1]; y <= b[4]; ++y)
                for (int x = b[0]; x <= b[3]; ++x) fn(((size_t)z * nd[1] + y) * nd[0] + x);
    };
    for (int i = 0; i < n; ++i) for_coarse(i, [&](size_t c) { ++cell_start[c + 1]; });
    for (int c = 0; c < ncell; ++c) cell_start[c + 1] += cell_start[c];
    std::vector<uint16_t> cell_obb(cell_start[ncell]);
    {
        std::vector<uint32_t> fill(cell_start.begin(), cell_start.end() - 1);
        for (int i = 0; i < n; ++i) for_coarse(i, [&](size_t c) { cell_obb[fill[c]++] = (uint16_t)i; });
    }
    // ---- fine cell classes (k_states fast path) ------------------------------------
    // Per fine cell a u16 class: 0 = no inflated AABB reaches it (valid, no test), else
    // 1 + index of the cell's candidate list (the OBBs whose AABB covers the cell; equal
    // lists are shared).  A list of more than kListInline OBBs is stored as
    // count = kListOverflow: such states take the coarse-grid candidate walk.
    std::vector<uint16_t> cls;
    std::vector<uint32_t> hdr;    // per list: start << 12 | count
    std::vector<uint16_t> flat;   // the lists' OBB ids
    double cls_target = double(1 << 14);  // fine cells to start from (coarsened below if needed)
    for (;;) {
        const double target = cls_target;
        int bd[3] = {1, 1, 1};
        float bo[3] = {0, 0, 0}, bi[3] = {1, 1, 1};
        if (n > 0) {
            double ext[3], vol = 1.0;
            for (int k = 0; k < 3; ++k) {
                ext[k] = std::max(g1[k] - g0[k], 1e-3);
                vol *= ext[k];
            }
            double h = std::cbrt(vol / target);
            for (int pass = 0;; ++pass) {
                bool ok = true;
                for (int k = 0; k < 3; ++k) {
                    bd[k] = std::min(4096, (int)std::ceil(ext[k] / h) + 4 + pass);
                    bi[k] = (float)(1.0 / h);
                    bo[k] = (float)(-(g0[k] - 1.5 * h) * (double)bi[k]);  // origin 1.5 cells below g0
                }
                // every AABB corner must map to [1, n-2]: the first and last cell of each
                // axis stay empty (else widen and retry)
                for (int i = 0; i < n && ok; ++i)
                    for (int k = 0; k < 3; ++k) {
                        const int lo_i = bm_axis(hw.aabbs[(size_t)i * 6 + k], bo[k], bi[k]);
                        const int hi_i = bm_axis(hw.aabbs[(size_t)i * 6 + 3 + k], bo[k], bi[k]);
                        if (lo_i < 1 || hi_i > bd[k] - 2) ok = false;
                    }
                if (ok) break;
                if (pass > 8) h *= 1.1;
            }
        }
        const size_t cells = (size_t)bd[0] * bd[1] * bd[2];
        // the records and the class table alone already exceed the staging budget: coarsen
        // before building any list
        if (align16((size_t)n * kRecDoubles * 8) + align16((cells + 1) * 2) > kStageBudget && target > 4096.0) {
            cls_target = target / 2;
            continue;
        }
        // Per-cell candidate lists (ascending OBB id) as CSR: count, scan, scatter — the
        // OBBs are visited in id order, so every list comes out sorted.
        std::vector<uint32_t> cstart(cells + 1, 0);
        std::vector<int> box((size_t)n * 6);
        for (int i = 0; i < n; ++i)
            for (int k = 0; k < 3; ++k) {
                box[(size_t)i * 6 + k] = bm_axis(hw.aabbs[(size_t)i * 6 + k], bo[k], bi[k]);
                box[(size_t)i * 6 + 3 + k] = bm_axis(hw.aabbs[(size_t)i * 6 + 3 + k], bo[k], bi[k]);
            }
        auto for_cells = [&](int i, auto&& fn) {
            const int* b = &box[(size_t)i * 6];
            for (int z = b[2]; z <= b[5]; ++z)
                for (int y = b[1]; y <= b[4]; ++y) {
                    const size_t row = ((size_t)z * bd[1] + y) * bd[0];
                    for (int x = b[0]; x <= b[3]; ++x) fn(row + x);
                }
        };
        for (int i = 0; i < n; ++i) for_cells(i, [&](size_t c) { ++cstart[c + 1]; });
        for (size_t c = 0; c < cells; ++c) cstart[c + 1] += cstart[c];
        std::vector<uint16_t> cid(cstart[cells]);
        {
            std::vector<uint32_t> fill(cstart.begin(), cstart.end() - 1);
            for (int i = 0; i < n; ++i) for_cells(i, [&](size_t c) { cid[fill[c]++] = (uint16_t)i; });
        }
        // Equal lists share one id (first occurrence in cell order), found through an
        // open-addressing hash table over the lists.
        cls.assign(cells + 1, 0);  // + the zero sentinel (out-of-grid lookups)
        hdr.assign(1, 0u);         // list 0: unused (class 0 = free)
        flat.clear();
        std::vector<uint32_t> slot_cell;  // per table slot: 1 + the cell holding the list (0 = empty)
        std::vector<uint16_t> slot_id;
        size_t occupied = 0;
        for (size_t c = 0; c < cells; ++c) occupied += cstart[c + 1] != cstart[c];
        size_t tsize = 64;
        while (tsize < 2 * occupied) tsize <<= 1;
        slot_cell.assign(tsize, 0u);
        slot_id.assign(tsize, 0);
        bool full = false;
        for (size_t c = 0; c < cells && !full; ++c) {
            const uint32_t b0 = cstart[c], m = cstart[c + 1] - b0;
            if (m == 0) continue;
            uint64_t h = 1469598103934665603ull;  // FNV-1a over the ids
            for (uint32_t j = 0; j < m; ++j) h = (h ^ cid[b0 + j]) * 1099511628211ull;
            size_t t = (size_t)(h ^ (h >> 29)) & (tsize - 1);
            bool found = false;
            while (slot_cell[t]) {
                const size_t o = slot_cell[t] - 1;
                const uint32_t ob = cstart[o], om = cstart[o + 1] - ob;
                if (om == m && std::equal(&cid[b0], &cid[b0] + m, &cid[ob])) {
                    cls[c] = slot_id[t];
                    found = true;
                    break;
                }
                t = (t + 1) & (tsize - 1);
            }
            if (found) continue;
            if (hdr.size() >= 65535 || flat.size() + m >= (size_t(1) << 20) || m > kListMaxLen) {
                full = true;
                break;
            }
            const uint16_t id = (uint16_t)hdr.size();
            hdr.push_back((uint32_t)(flat.size() << 12) | m);  // start : 20, count : 12
            flat.insert(flat.end(), &cid[b0], &cid[b0] + m);
            slot_cell[t] = (uint32_t)c + 1;
            slot_id[t] = id;
            cls[c] = id;
        }
        if (full) {  // more distinct lists than a u16 class can name: a coarser grid
            if (target <= 8.0) {
                set_error("epp_world: candidate list table overflow");
                return false;
            }
            cls_target = target / 8;
            continue;
        }
        // k_states_v5 stages records + lists + class table into LDS: keep that part
        // within kStageBudget by coarsening the class grid (down to 4096 cells)
        const size_t staged = align16((size_t)n * kRecDoubles * 8) + align16(hdr.size() * 4 + flat.size() * 2) +
                              align16(cls.size() * 2);
        if (staged > kStageBudget && target > 4096.0) {
            cls_target = target / 2;
            continue;
        }
        v.bnx = bd[0]; v.bny = bd[1]; v.bnz = bd[2];
        v.bofx = bo[0]; v.bofy = bo[1]; v.bofz = bo[2];
        v.bix = bi[0]; v.biy = bi[1]; v.biz = bi[2];
        v.bm_words = (uint32_t)cells;  // index of the sentinel class
        v.n_lists = (uint32_t)hdr.size();
        break;
    }
    const size_t n_entries = cell_start[ncell];
    // ---- pack (layout in epp_internal.h) ---------------------------------------
    const size_t off_mask = 0;
    const size_t off_cs = align16(off_mask + mask.size() * 8);
    const size_t front = align16(off_cs + cell_start.size() * 4);
    const size_t off_co = front;
    const size_t off_meta = align16(off_co + n_entries * 2);
    const size_t off_soa = align16(off_meta + meta.size() * 4);
    // AoS OBB records for the fine-cell exact path (kRecDoubles doubles each)
    std::vector<double> aos((size_t)n * kRecDoubles, 0.0);
    for (int i = 0; i < n; ++i) {
        double* r = &aos[(size_t)i * kRecDoubles];
        const double* f = soa.data();
        const int fields[14] = {F_LOX, F_LOY, F_LOZ, F_HIX, F_HIY, F_HIZ, F_CX, F_CY, F_CZ, F_COS, F_SIN, F_HX, F_HY, F_HZ};
        for (int k = 0; k < 14; ++k) r[k] = f[(size_t)fields[k] * n_pad + i];
        uint64_t m = meta[i];
        std::memcpy(&r[R_META], &m, 8);
    }
    const size_t off_aos = align16(off_soa + soa.size() * sizeof(double));
    const size_t off_lists = align16(off_aos + aos.size() * sizeof(double));
    const size_t off_ids = off_lists + hdr.size() * 4;
    // byte classes (k_states_v5 stages them instead of the u16 table) when the lists fit.
    // Sparse form (the default; -DEPP_V5_DENSE_CLS: one byte per cell): per 32 cells one u64
    // [occupancy bits | nonzero cells before this word], then the class bytes of the nonzero
    // cells in cell order -- 0.25 B per cell plus ~1 B per occupied cell (C2: 7 KB instead of
    // 18.5 KB staged by every workgroup).
    const bool c8 = hdr.size() <= 256;
    const size_t off_c8 = align16(off_ids + flat.size() * 2);
    std::vector<uint64_t> cwords;
    std::vector<uint8_t> cnz;
#ifndef EPP_V5_DENSE_CLS
    if (c8) {
        cwords.assign((cls.size() + 31) / 32, 0ull);
        for (size_t w = 0; w < cwords.size(); ++w) {
            uint32_t m = 0;
            const uint64_t before = cnz.size();
            for (size_t j = 0; j < 32 && 32 * w + j < cls.size(); ++j)
                if (cls[32 * w + j]) {
                    m |= 1u << j;
                    cnz.push_back((uint8_t)cls[32 * w + j]);
                }
            cwords[w] = (uint64_t)m | (before << 32);
        }
    }
    const size_t c8_bytes = c8 ? cwords.size() * 8 + cnz.size() : 0;
#else
    const size_t c8_bytes = c8 ? cls.size() : 0;
#endif
    const size_t off_bm = c8 ? align16(off_c8 + c8_bytes) : off_c8;
    // ---- motion tile filter (k_motions_v5) ------------------------------------------
    // The smallest row width W (words of OBB bits), then the fewest tiles per axis T,
    // for which every tile holds <= 32 W OBBs; S local slabs per tile and axis as many as
    // fit kSlabBudget (4..64, a power of two).
    std::vector<uint32_t> slab;
    int S = 0, SL = 0, W = 0, T = 0;
    uint32_t tw = 0;
    float so[3] = {0, 0, 0}, si[3] = {0, 0, 0};
    std::vector<int> gsl((size_t)n * 6);  // per OBB: global slab lo / hi per axis
    // tile bytes: kSlabBudget, or up to kSlabBudgetMax while the records, the tiles and the
    // wave queues of k_motions_v5 still fit its LDS budget (finer slabs, fewer candidates)
    const size_t slab_budget = std::max<size_t>(
        kSlabBudget, std::min<size_t>(kSlabBudgetMax, kMotionsLdsFree > (size_t)n * kRecDoubles * 8
                                                          ? kMotionsLdsFree - (size_t)n * kRecDoubles * 8
                                                          : 0));
    auto tile_words = [](int s_, int w_) {
        return (uint32_t)((6 * s_ * slab_row_stride(w_) + 3 * w_ + 16 * w_ + 3) & ~3);
    };
    auto place = [&](int t_, int sl_) {  // slab ranges for (T, S); returns the largest tile population
        const int s_ = 1 << sl_;
        for (int k = 0; k < 3; ++k) {
            const int G = k < 2 ? t_ * s_ : s_;
            const double ext = std::max(g1[k] - g0[k], 1e-6);
            si[k] = (float)(G / ext);
            so[k] = (float)(-g0[k] * (G / ext));
            for (int i = 0; i < n; ++i) {
                const double* lo = &hw.aabbs[(size_t)i * 6];
                gsl[(size_t)i * 6 + k] = slab_axis(lo[k], so[k], si[k], G);
                gsl[(size_t)i * 6 + 3 + k] = slab_axis(lo[3 + k], so[k], si[k], G);
            }
        }
        std::vector<int> pop((size_t)t_ * t_, 0);
        for (int i = 0; i < n; ++i) {
            const int* g = &gsl[(size_t)i * 6];
            for (int ty = g[1] >> sl_; ty <= g[4] >> sl_; ++ty)
                for (int tx = g[0] >> sl_; tx <= g[3] >> sl_; ++tx) ++pop[(size_t)ty * t_ + tx];
        }
        return *std::max_element(pop.begin(), pop.end());
    };
    // first with >= 16 local slabs (the filter's resolution sets how many pairs reach the
    // exact test), then with >= 4
    for (int min_sl = 4; n > 0 && !W && min_sl >= 2; min_sl -= 2)
        for (int w_ = 1; w_ <= kSlabMaxWords && !W; w_ *= 2)
            for (int t_ = 1; t_ <= 16 && !W; ++t_) {
                int sl_ = 6;
                while (sl_ >= min_sl && (size_t)t_ * t_ * tile_words(1 << sl_, w_) * 4 > slab_budget) --sl_;
                if (sl_ < min_sl) break;
                if (place(t_, sl_) <= 32 * w_) {
                    W = w_;
                    T = t_;
                    SL = sl_;
                }
            }
    if (W) {
        S = 1 << SL;
        place(T, SL);
        tw = tile_words(S, W);
        const int stride = slab_row_stride(W);
        slab.assign((size_t)T * T * tw, 0u);
        std::vector<int> fill_n((size_t)T * T, 0);
        for (int i = 0; i < n; ++i) {
            const int* g = &gsl[(size_t)i * 6];
            const int tx0 = g[0] >> SL, ty0 = g[1] >> SL;
            for (int ty = ty0; ty <= g[4] >> SL; ++ty)
                for (int tx = tx0; tx <= g[3] >> SL; ++tx) {
                    const size_t t = (size_t)ty * T + tx;
                    uint32_t* tile = &slab[t * tw];
                    const int j = fill_n[t]++;
                    const uint32_t bit = 1u << (j & 31);
                    const int wd = j >> 5;
                    // local slab of the OBB's ends (clamped into the tile; z is not tiled)
                    const int l[3] = {std::min(std::max(g[0] - (tx << SL), 0), S - 1),
                                      std::min(std::max(g[1] - (ty << SL), 0), S - 1), g[2]};
                    const int h[3] = {std::min(std::max(g[3] - (tx << SL), 0), S - 1),
                                      std::min(std::max(g[4] - (ty << SL), 0), S - 1), g[5]};
                    for (int k = 0; k < 3; ++k) {
                        tile[((size_t)(2 * k) * S + l[k]) * stride + wd] |= bit;
                        tile[((size_t)(2 * k + 1) * S + h[k]) * stride + wd] |= bit;
                    }
                    uint32_t* tail = tile + (size_t)6 * S * stride;
                    if (tx == tx0) tail[wd] |= bit;                        // FX
                    if (ty == ty0) tail[W + wd] |= bit;                    // FY
                    if (meta[i] & META_FILLING) tail[2 * W + wd] |= bit;   // FILL
                    reinterpret_cast<uint16_t*>(tail + 3 * W)[j] = (uint16_t)i;
                }
        }
        for (size_t t = 0; t < (size_t)T * T; ++t)
            for (int k = 0; k < 3; ++k) {  // marks -> prefix ORs: LE up, GE down
                uint32_t* le = &slab[t * tw + (size_t)(2 * k) * S * stride];
                uint32_t* ge = &slab[t * tw + (size_t)(2 * k + 1) * S * stride];
                for (int s_ = 1; s_ < S; ++s_)
                    for (int w_ = 0; w_ < W; ++w_) le[(size_t)s_ * stride + w_] |= le[(size_t)(s_ - 1) * stride + w_];
                for (int s_ = S - 2; s_ >= 0; --s_)
                    for (int w_ = 0; w_ < W; ++w_) ge[(size_t)s_ * stride + w_] |= ge[(size_t)(s_ + 1) * stride + w_];
            }
    }
    v.slab_n = S;
    v.slab_log = SL;
    v.slab_w = W;
    v.tile_n = T;
    v.tile_words = tw;
    v.sofx = so[0]; v.sofy = so[1]; v.sofz = so[2];
    v.six = si[0]; v.siy = si[1]; v.siz = si[2];
    const size_t off_slab = align16(off_bm + cls.size() * 2);
    const size_t total = align16(off_slab + slab.size() * 4);
    if (total > 0xFFFFFFFFull) {
        set_error("epp_world: index too large");
        return false;
    }
    hw.blob.assign(total, '\0');
    char* b = &hw.blob[0];
    std::memcpy(b + off_mask, mask.data(), mask.size() * 8);
    std::memcpy(b + off_cs, cell_start.data(), cell_start.size() * 4);
    if (n_entries) std::memcpy(b + off_co, cell_obb.data(), n_entries * 2);
    std::memcpy(b + off_meta, meta.data(), meta.size() * 4);
    std::memcpy(b + off_soa, soa.data(), soa.size() * sizeof(double));
    if (!aos.empty()) std::memcpy(b + off_aos, aos.data(), aos.size() * sizeof(double));
    std::memcpy(b + off_lists, hdr.data(), hdr.size() * 4);
    if (!flat.empty()) std::memcpy(b + off_ids, flat.data(), flat.size() * 2);
    v.off_ids = (uint32_t)off_ids;
    v.off_aos = (uint32_t)off_aos;
    std::memcpy(b + off_bm, cls.data(), cls.size() * 2);
    if (!slab.empty()) std::memcpy(b + off_slab, slab.data(), slab.size() * 4);
    v.off_slab = (uint32_t)off_slab;
#ifndef EPP_V5_DENSE_CLS
    if (c8) {
        std::memcpy(b + off_c8, cwords.data(), cwords.size() * 8);
        if (!cnz.empty()) std::memcpy(b + off_c8 + cwords.size() * 8, cnz.data(), cnz.size());
    }
#else
    if (c8)
        for (size_t c = 0; c < cls.size(); ++c) b[off_c8 + c] = (char)(uint8_t)cls[c];
#endif
    v.off_cls8 = c8 ? (uint32_t)off_c8 : 0u;
    v.cls8_bytes = (uint32_t)c8_bytes;
    v.off_lists = (uint32_t)off_lists;
    v.off_bitmap = (uint32_t)off_bm;
    v.blob_bytes = (uint32_t)total;
    v.front_bytes = (uint32_t)front;
    v.off_cell_mask = (uint32_t)off_mask;
    v.off_cell_start = (uint32_t)off_cs;
    v.off_cell_obb = (uint32_t)off_co;
    v.off_meta = (uint32_t)off_meta;
    v.off_soa = (uint32_t)off_soa;
    return true;
}

// The device allocation holds the blob followed by a copy of the WorldView (kernels
// that keep only a pointer to it read the fields they need through the scalar cache).
// The upload goes through a pinned staging buffer on the world's own stream (one DMA,
// no pageable bounce); the caller has made sure no kernel still reads the old blob.
bool upload(HostWorld& hw) {
    const size_t bytes = hw.blob.size();
    const size_t view_off = (bytes + 255) & ~size_t(255);
    const size_t need = view_off + sizeof(WorldView);
    hipError_t e = hipSuccess;
    if (!hw.stream) e = hipStreamCreateWithFlags(&hw.stream, hipStreamNonBlocking);
    if (e == hipSuccess && need > hw.d_capacity) {
        if (hw.d_blob) (void)hipFree(hw.d_blob);
        hw.d_blob = nullptr;
        hw.d_capacity = 0;
        e = hipMalloc(&hw.d_blob, need);
        if (e == hipSuccess) hw.d_capacity = need;
    }
    if (e == hipSuccess && need > hw.h_capacity) {
        if (hw.h_stage) (void)hipHostFree(hw.h_stage);
        hw.h_stage = nullptr;
        hw.h_capacity = 0;
        e = hipHostMalloc(&hw.h_stage, need, hipHostMallocDefault);
        if (e == hipSuccess) hw.h_capacity = need;
    }
    if (e != hipSuccess) {
        set_error(std::string("epp_world: allocation: ") + hipGetErrorString(e));
        return false;
    }
    hw.view.blob = (const unsigned char*)hw.d_blob;
    hw.d_view = reinterpret_cast<const WorldView*>(static_cast<char*>(hw.d_blob) + view_off);
    hw.dev_view = hw.view;
    std::memcpy(hw.h_stage, hw.blob.data(), bytes);
    std::memcpy(static_cast<char*>(hw.h_stage) + view_off, &hw.view, sizeof(WorldView));
    e = hipMemcpyAsync(hw.d_blob, hw.h_stage, need, hipMemcpyHostToDevice, hw.stream);
    if (e == hipSuccess) e = hipStreamSynchronize(hw.stream);
    if (e != hipSuccess) {
        set_error(std::string("epp_world: upload: ") + hipGetErrorString(e));
        return false;
    }
    return true;
}

// Buffers of destroyed worlds, kept for the next epp_world_create on the same device: a
// fresh PathPlanner / OnlineTrajGenerator per request then reuses the pinned record slots,
// the pinned upload staging, the device blob and the upload stream instead of allocating
// them again (pinned allocations are the cold cost of a world; the buffers grow as needed).
// Never freed (the pool lives until the process exits, as the HIP runtime's own caches).
struct WorldBufs {
    int device = 0;
    double* rec_buf[2] = {nullptr, nullptr};
    size_t rec_cap[2] = {0, 0};
    std::vector<HostWorld::RecReader> readers[2];
    void* h_stage = nullptr;
    size_t h_capacity = 0;
    void* d_blob = nullptr;
    size_t d_capacity = 0;
    hipStream_t stream = nullptr;
};
constexpr size_t kWorldPoolMax = 8;
std::mutex g_world_pool_mu;
std::vector<WorldBufs>& world_pool() {
    static auto* pool = new std::vector<WorldBufs>();  // (intentionally leaked, see above)
    return *pool;
}

void pool_take(HostWorld& hw) {
    std::lock_guard<std::mutex> lk(g_world_pool_mu);
    auto& pool = world_pool();
    for (size_t i = 0; i < pool.size(); ++i)
        if (pool[i].device == hw.device) {
            WorldBufs& b = pool[i];
            for (int k = 0; k < 2; ++k) {
                hw.rec_buf[k] = b.rec_buf[k];
                hw.rec_cap[k] = b.rec_cap[k];
                hw.rec_readers[k] = std::move(b.readers[k]);
            }
            hw.h_stage = b.h_stage;
            hw.h_capacity = b.h_capacity;
            hw.d_blob = b.d_blob;
            hw.d_capacity = b.d_capacity;
            hw.stream = b.stream;
            pool.erase(pool.begin() + (std::ptrdiff_t)i);
            return;
        }
}

// The world's buffers into the pool (the device is idle: epp_world_destroy synchronised);
// false when the pool is full (the caller frees them).
bool pool_give(HostWorld& hw) {
    std::lock_guard<std::mutex> lk(g_world_pool_mu);
    auto& pool = world_pool();
    if (pool.size() >= kWorldPoolMax) return false;
    WorldBufs b;
    b.device = hw.device;
    for (int k = 0; k < 2; ++k) {
        b.rec_buf[k] = hw.rec_buf[k];
        b.rec_cap[k] = hw.rec_cap[k];
        b.readers[k] = std::move(hw.rec_readers[k]);
        for (auto& r : b.readers[k]) r.pending = false;
    }
    b.h_stage = hw.h_stage;
    b.h_capacity = hw.h_capacity;
    b.d_blob = hw.d_blob;
    b.d_capacity = hw.d_capacity;
    b.stream = hw.stream;
    pool.push_back(std::move(b));
    return true;
}

}  // namespace

}  // namespace epp

struct epp_world : epp::HostWorld {};


extern "C" {

epp_status epp_world_create(const epp_obb* obbs, int32_t n, double r_gate, double r_obst,
                            epp_world** out) {
    if (!out || n < 0 || (n > 0 && !obbs)) {
        epp::set_error("epp_world_create: invalid argument");
        return EPP_ERR_INVALID_ARGUMENT;
    }
    if (n > 65535) {
        epp::set_error("epp_world_create: at most 65535 OBBs");
        return EPP_ERR_INVALID_ARGUMENT;
    }
    epp_world* w = new (std::nothrow) epp_world();
    if (!w) return EPP_ERR_RUNTIME;
    w->r_gate = r_gate;
    w->r_obst = r_obst;
    (void)hipGetDevice(&w->device);
    epp::pool_take(*w);  // (buffers of a destroyed world on this device, if any)
    // (on failure the buffers go back to the pool or are freed; the error message stays)
    if (!epp::build_records(*w, obbs, n) || !epp::build_blob(*w, obbs, n)) {
        (void)epp_world_destroy(w);
        return EPP_ERR_UNSUPPORTED;
    }
    if (!epp::upload(*w)) {
        (void)epp_world_destroy(w);
        return EPP_ERR_HIP;
    }
    w->generation = 1;
    *out = w;
    return EPP_OK;
}

epp_status epp_world_update(epp_world* w, const epp_obb* obbs, int32_t n) {
    if (!w || n < 0 || n > 65535 || (n > 0 && !obbs)) {
        epp::set_error("epp_world_update: invalid argument");
        return EPP_ERR_INVALID_ARGUMENT;
    }
    // (the device blob is not touched: ensure_index rebuilds it after in-flight kernels;
    // the records go to the other pinned slot, see HostWorld).  Exclusive on index_mu: a
    // launcher holding a SmallWorld snapshot of the pinned records has queued its kernel and
    // recorded its reader event (or, polled, finished) before the slot can be rewritten.
    std::unique_lock<std::shared_mutex> ix(w->index_mu);
    std::lock_guard<std::mutex> lk(w->mu);
    if (!epp::build_records(*w, obbs, n)) return EPP_ERR_UNSUPPORTED;
    w->index_stale = true;
    ++w->generation;
    return EPP_OK;
}

epp_status epp_world_destroy(epp_world* w) {
    if (!w) return EPP_OK;
    // the world's own device, whichever device the calling thread has current: its buffers
    // go to the pool (or are freed) only once no kernel on that device can still read them
    int prev = 0;
    const bool restore = hipGetDevice(&prev) == hipSuccess && prev != w->device;
    if (restore) (void)hipSetDevice(w->device);
    (void)hipDeviceSynchronize();
    if (restore) (void)hipSetDevice(prev);
    if (epp::pool_give(*w)) {  // kept for the next world (no kernel reads them any more)
        delete w;
        return EPP_OK;
    }
    if (w->d_blob) (void)hipFree(w->d_blob);
    if (w->h_stage) (void)hipHostFree(w->h_stage);
    for (int k = 0; k < 2; ++k) {
        if (w->rec_buf[k]) (void)hipHostFree(w->rec_buf[k]);
        for (auto& r : w->rec_readers[k]) (void)hipEventDestroy(r.ev);
    }
    if (w->stream) (void)hipStreamDestroy(w->stream);
    delete w;
    return EPP_OK;
}

epp_status epp_world_build_index(const epp_world* w) {
    if (!w) {
        epp::set_error("epp_world_build_index: invalid argument");
        return EPP_ERR_INVALID_ARGUMENT;
    }
    return epp::ensure_index(w, nullptr);
}

epp_status epp_world_generation(const epp_world* w, uint64_t* generation) {
    if (!w || !generation) {
        epp::set_error("epp_world_generation: invalid argument");
        return EPP_ERR_INVALID_ARGUMENT;
    }
    *generation = w->generation;
    return EPP_OK;
}

epp_status epp_world_num_obbs(const epp_world* w, int32_t* n) {
    if (!w || !n) return EPP_ERR_INVALID_ARGUMENT;
    *n = w->view.n_obb;
    return EPP_OK;
}

epp_status epp_world_get_aabbs(const epp_world* w, double* lo_hi) {
    if (!w || !lo_hi) return EPP_ERR_INVALID_ARGUMENT;
    std::memcpy(lo_hi, w->aabbs.data(), w->aabbs.size() * sizeof(double));
    return EPP_OK;
}

}  // extern "C"

namespace epp {

// The device index of the current version: rebuilt and uploaded here when an update made
// it stale (exclusively: after every launcher holding a lease has queued its kernel, and
// after every kernel that may still read the old blob has finished).  With a lease, a
// snapshot of the uploaded index that stays valid until the lease is released.
epp_status ensure_index(const epp_world* cw, IndexLease* lease) {
    HostWorld& hw = const_cast<epp_world&>(*cw);
    bool stale;
    {
        std::lock_guard<std::mutex> lk(hw.mu);
        stale = hw.index_stale;
    }
    if (stale) {
        std::unique_lock<std::shared_mutex> ix(hw.index_mu);
        std::lock_guard<std::mutex> lk(hw.mu);
        if (hw.index_stale) {
            (void)hipDeviceSynchronize();
            if (!build_blob(hw, hw.obbs.data(), (int)hw.obbs.size())) return EPP_ERR_UNSUPPORTED;
            if (!upload(hw)) return EPP_ERR_HIP;
            hw.index_stale = false;
        }
    }
    if (lease) {
        // (an update after the rebuild above leaves the uploaded index consistent: the
        // launch checks the version it snapshots, as if it had run before the update)
        lease->lk = std::shared_lock<std::shared_mutex>(hw.index_mu);
        std::lock_guard<std::mutex> lk(hw.mu);
        lease->view = hw.dev_view;
        lease->dview = hw.d_view;
    }
    return EPP_OK;
}

SmallWorld small_world(const epp_world* cw) {
    HostWorld& hw = const_cast<epp_world&>(*cw);
    std::shared_lock<std::shared_mutex> ix(hw.index_mu);
    std::lock_guard<std::mutex> lk(hw.mu);
    SmallWorld s;
    s.recs = hw.index_stale ? hw.h_recs : reinterpret_cast<const double*>(hw.dev_view.blob + hw.dev_view.off_aos);
    s.host_slot = hw.index_stale ? hw.rec_slot : -1;
    s.n_obb = (int32_t)hw.obbs.size();
    s.r_gate = hw.r_gate;
    s.r_obst = hw.r_obst;
    // held until the caller's kernel is queued (and its reader event recorded) or, polled,
    // has finished: no rebuild frees the device records and no update rewrites or
    // reallocates the pinned slot under a launch
    s.lease = std::move(ix);
    return s;
}

// An asynchronous launch reading the pinned records of `sw`'s slot was queued on `st`:
// the next update that would rewrite that slot waits for it.
epp_status note_record_reader(const epp_world* cw, const SmallWorld& sw, hipStream_t st) {
    if (sw.host_slot < 0) return EPP_OK;
    HostWorld& hw = const_cast<epp_world&>(*cw);
    std::lock_guard<std::mutex> lk(hw.mu);
    auto& rd = hw.rec_readers[sw.host_slot];
    HostWorld::RecReader* r = nullptr;  // one event per stream: a later launch on it ends later
    for (auto& x : rd)
        if (x.stream == st) r = &x;
    hipError_t e = hipSuccess;
    if (!r) {
        hipEvent_t ev = nullptr;
        e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
        if (e == hipSuccess) {
            rd.push_back({st, ev, false});
            r = &rd.back();
        }
    }
    if (e == hipSuccess) e = hipEventRecord(r->ev, st);
    if (e != hipSuccess) {
        set_error(std::string("epp_world: recording a reader of the records: ") + hipGetErrorString(e));
        return EPP_ERR_HIP;
    }
    r->pending = true;
    return EPP_OK;
}

}  // namespace epp

// Debug entry (not part of include/epp.h): sizes of the device index, for tests and
// kernel tuning.  out: blob_bytes, staged prefix bytes, n_lists, fine cells, coarse
// cells, n_obb.
extern "C" epp_status epp_dbg_world_info(const epp_world* w, int64_t out[6]) {
    if (!w || !out) return EPP_ERR_INVALID_ARGUMENT;
    const epp::WorldView& v = w->view;
    out[0] = v.blob_bytes;
    out[1] = v.off_bitmap;
    out[2] = v.n_lists;
    out[3] = (int64_t)v.bnx * v.bny * v.bnz;
    out[4] = (int64_t)v.nx * v.ny * v.nz;
    out[5] = v.n_obb;
    return EPP_OK;
}

// Debug entry (not part of include/epp.h): host-side index build only (no device), for
// timing the world rebuild on the CPU.  out: [microseconds per build, blob bytes, tile
// count per axis, tile words, slab words W, slabs S].
extern "C" epp_status epp_dbg_build_blob(const epp_obb* obbs, int32_t n, double r_gate, double r_obst, int32_t reps,
                                         double out[6]) {
    if (!out || n < 0 || (n > 0 && !obbs) || reps < 1) return EPP_ERR_INVALID_ARGUMENT;
    epp::HostWorld hw;
    hw.r_gate = r_gate;
    hw.r_obst = r_obst;
    const auto t0 = std::chrono::steady_clock::now();
    for (int r = 0; r < reps; ++r)
        if (!epp::build_blob(hw, obbs, n)) return EPP_ERR_UNSUPPORTED;
    const auto t1 = std::chrono::steady_clock::now();
    out[0] = std::chrono::duration<double, std::micro>(t1 - t0).count() / reps;
    out[1] = hw.view.blob_bytes;
    out[2] = hw.view.tile_n;
    out[3] = hw.view.tile_words;
    out[4] = hw.view.slab_w;
    out[5] = hw.view.slab_n;
    return EPP_OK;
}

// Debug entry (not part of include/epp.h): the class-grid layout of a world's index, host
// build only.  out: off_aos, off_lists, off_ids, off_cls8, off_bitmap, blob_bytes, n_lists,
// class cells (bm_words), bnx, bny, bnz, staged bytes of k_states_v5.
extern "C" epp_status epp_dbg_class_layout(const epp_obb* obbs, int32_t n, double r_gate, double r_obst,
                                           int64_t out[12]) {
    if (!out || n < 0 || (n > 0 && !obbs)) return EPP_ERR_INVALID_ARGUMENT;
    epp::HostWorld hw;
    hw.r_gate = r_gate;
    hw.r_obst = r_obst;
    if (!epp::build_blob(hw, obbs, n)) return EPP_ERR_UNSUPPORTED;
    const epp::WorldView& v = hw.view;
    const int64_t vals[12] = {v.off_aos, v.off_lists, v.off_ids, v.off_cls8, v.off_bitmap, v.blob_bytes, v.n_lists,
                              v.bm_words, v.bnx, v.bny, v.bnz,
                              (int64_t)((v.off_cls8 ? ((v.off_cls8 + v.cls8_bytes + 15u) & ~15u) : v.blob_bytes) -
                                        v.off_aos)};
    for (int k = 0; k < 12; ++k) out[k] = vals[k];
    return EPP_OK;
}

// Debug entry (not part of include/epp.h): host check of k_states_v5's sparse byte-class
// encoding -- for every class-grid cell (the zero sentinel included) the lookup the kernel
// does (occupancy word, rank, class byte; states.hip cls_of) must give the cell's class of
// the u16 table.  Returns the number of mismatching cells (0), or -1 when the world has no
// byte classes.
extern "C" int64_t epp_dbg_check_sparse_classes(const epp_obb* obbs, int32_t n, double r_gate, double r_obst) {
    if (n < 0 || (n > 0 && !obbs)) return -2;
    epp::HostWorld hw;
    hw.r_gate = r_gate;
    hw.r_obst = r_obst;
    if (!epp::build_blob(hw, obbs, n)) return -2;
    const epp::WorldView& v = hw.view;
    if (!v.off_cls8) return -1;
    const unsigned char* b = reinterpret_cast<const unsigned char*>(hw.blob.data());
    const uint16_t* cls = reinterpret_cast<const uint16_t*>(b + v.off_bitmap);
    const unsigned char* base = b + v.off_cls8;
    const unsigned char* nz = base + ((v.bm_words + 1u + 31u) >> 5) * 8u;
    int64_t bad = 0;
    for (uint32_t idx = 0; idx <= v.bm_words; ++idx) {
#ifndef EPP_V5_DENSE_CLS
        uint64_t wd;
        std::memcpy(&wd, base + (size_t)(idx >> 5) * 8, 8);
        const uint32_t m = (uint32_t)wd, sh = idx & 31u;
        const uint32_t rank = (uint32_t)(wd >> 32) + (uint32_t)__builtin_popcount(m & ((1u << sh) - 1u));
        const uint32_t c = ((m >> sh) & 1u) ? (uint32_t)nz[rank] : 0u;
#else
        const uint32_t c = base[idx];
#endif
        bad += c != (uint32_t)cls[idx];
    }
    return bad;
}
