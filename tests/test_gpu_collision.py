"""GPU parity: OBB validity kernels (through the C ABI) vs the CPU oracle, bit-exact.

Reference semantics: src/World.cpp:80-162, src/OBB.cpp:10-123.
"""
import json
import os

import numpy as np
import pytest

import oracle as O
from eppamd import capi, config, synth

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


def _worlds(cfg, geom):
    rg, ro = config.inflate_radii(cfg)
    out = {}
    g, o, _, _ = synth.c1_world()
    out["c1"] = (g, o, synth.C1_BOUNDS)
    out["c2"] = synth.track_world(42) + (synth.C2_BOUNDS,)
    g3, o3 = synth.track_world(42, n_obstacles=472)
    out["c3"] = (g3, o3, synth.C2_BOUNDS)
    return rg, ro, out


def _adversarial_points(ref_w):
    """Points exactly on / one ulp around every AABB face and corner."""
    pts = []
    for o in ref_w:
        mid = (o["aabb_lo"] + o["aabb_hi"]) / 2
        for k in range(3):
            for v in (o["aabb_lo"][k], o["aabb_hi"][k]):
                for w in (v, np.nextafter(v, np.inf), np.nextafter(v, -np.inf)):
                    p = mid.copy()
                    p[k] = w
                    pts.append(p)
        pts += [o["aabb_lo"].copy(), o["aabb_hi"].copy(), np.nextafter(o["aabb_hi"], -np.inf),
                np.nextafter(o["aabb_lo"], np.inf), o["center"].copy()]
        # points on the inflated OBB faces in local coordinates
        c, s = o["rot"][0], o["rot"][3]
        for sx in (-1, 1):
            l = np.array([sx * (o["half"][0] + 0.2), 0.3 * o["half"][1], 0.0])
            pts.append(o["center"] + np.array([c * l[0] - s * l[1], s * l[0] + c * l[1], l[2]]))
    return np.array(pts)


@pytest.fixture(scope="module")
def worlds(cfg, geom):
    return _worlds(cfg, geom)


@pytest.mark.parametrize("name", ["c1", "c2", "c3"])
def test_aabbs_match_oracle(geom, worlds, name):
    rg, ro, ws = worlds
    gates, obstacles, _ = ws[name]
    obbs = capi.build_obbs(geom, gates, obstacles)
    ref = O.world_build(geom, gates, obstacles, rg, ro)
    w = capi.World(obbs, rg, ro)
    a = w.aabbs()
    assert np.array_equal(a[:, :3], ref["aabb_lo"]) and np.array_equal(a[:, 3:], ref["aabb_hi"])


@pytest.mark.parametrize("name", ["c1", "c2", "c3"])
@pytest.mark.parametrize("can_pass", [0, 1])
def test_states_bit_exact(geom, worlds, name, can_pass):
    rg, ro, ws = worlds
    gates, obstacles, (lo, hi) = ws[name]
    ref = O.world_build(geom, gates, obstacles, rg, ro)
    w = capi.World(capi.build_obbs(geom, gates, obstacles), rg, ro)
    pts = np.vstack([synth.sample_states(7, lo, hi, 200_003), _adversarial_points(ref)])
    got = w.check_states(pts, can_pass)
    exp = O.check_states(ref, rg, ro, pts, can_pass, threads=8)
    assert exp.min() == 0 and exp.max() == 1  # both outcomes exercised
    assert np.array_equal(got, exp), np.flatnonzero(got != exp)[:10]


@pytest.mark.parametrize("name", ["c1", "c2"])
def test_states_mindist(geom, worlds, name):
    rg, ro, ws = worlds
    gates, obstacles, (lo, hi) = ws[name]
    ref = O.world_build(geom, gates, obstacles, rg, ro)
    w = capi.World(capi.build_obbs(geom, gates, obstacles), rg, ro)
    pts = np.vstack([synth.sample_states(9, lo, hi, 100_001), _adversarial_points(ref)])
    for md in (0.0, 0.1, 0.2, 0.35):
        got = w.check_states_mindist(pts, md)
        exp = O.check_states_mindist(ref, pts, md)
        assert np.array_equal(got, exp), md


@pytest.mark.parametrize("impl", ["v5", "v5b256", "v5b512", "v5b1024", "v4", "generic"])
@pytest.mark.parametrize("name", ["c2", "c3"])
def test_states_every_kernel_variant(geom, worlds, name, impl, monkeypatch):
    """Each state kernel (k_states_v5 = default, k_states_v4 = fallback for worlds whose
    staged part exceeds LDS, e.g. C3; k_states = generic) on plain, compacting and
    minDistance launches, ragged n.  "v5" runs the default launch shape (two 512-thread
    workgroups per CU for a single pass), "v5b512"/"v5b1024" force one workgroup shape
    (test hooks EPP_STATES_KERNEL / EPP_V5_BLOCK)."""
    monkeypatch.setenv("EPP_STATES_KERNEL", impl[:2] if impl.startswith("v") else impl)
    monkeypatch.setenv("EPP_V5_BLOCK", impl[3:] if impl.startswith("v5b") else "")
    seed = 31 + len(impl)
    rg, ro, ws = worlds
    gates, obstacles, (lo, hi) = ws[name]
    ref = O.world_build(geom, gates, obstacles, rg, ro)
    w = capi.World(capi.build_obbs(geom, gates, obstacles), rg, ro)
    pts = np.vstack([synth.sample_states(seed, lo, hi, 150_001), _adversarial_points(ref)])
    exp = O.check_states(ref, rg, ro, pts, False, threads=8)
    assert np.array_equal(w.check_states(pts, False), exp)
    valid, idx = w.check_states(pts, False, compact=True)
    assert np.array_equal(valid, exp) and np.array_equal(np.sort(idx), np.flatnonzero(exp))
    for n in (1, 2, 3, 5, 4097):
        assert np.array_equal(w.check_states(pts[:n], False), exp[:n]), n
    assert np.array_equal(w.check_states_mindist(pts, 0.15), O.check_states_mindist(ref, pts, 0.15))


@pytest.mark.parametrize("n", [1 << 20, (1 << 20) + 4 * 256 * 512 + 7, 5 << 20])
def test_states_full_size(geom, worlds, n):
    """BASELINE C2 size (1,048,576 states: the single-pass two-workgroups-per-CU shape),
    just past it, and 5M states (prefetching multi-pass shape), bit-exact vs the oracle."""
    rg, ro, ws = worlds
    gates, obstacles, (lo, hi) = ws["c2"]
    ref = O.world_build(geom, gates, obstacles, rg, ro)
    w = capi.World(capi.build_obbs(geom, gates, obstacles), rg, ro)
    pts = synth.sample_states(7, lo, hi, n)
    assert np.array_equal(w.check_states(pts, False), O.check_states(ref, rg, ro, pts, False, threads=8))


def test_compaction(geom, worlds):
    rg, ro, ws = worlds
    gates, obstacles, (lo, hi) = ws["c2"]
    ref = O.world_build(geom, gates, obstacles, rg, ro)
    w = capi.World(capi.build_obbs(geom, gates, obstacles), rg, ro)
    pts = synth.sample_states(21, lo, hi, 65_537)
    valid, idx = w.check_states(pts, False, compact=True)
    exp = O.check_states(ref, rg, ro, pts, False, threads=8)
    assert np.array_equal(valid, exp)
    assert np.array_equal(np.sort(idx), np.flatnonzero(exp))


@pytest.mark.parametrize("impl", ["lds", "v4", "v4/512", "v4/1024", "generic"])
@pytest.mark.parametrize("name", ["c1", "c2", "c3"])
@pytest.mark.parametrize("mode", [0, 1])
def test_motions_bit_exact(geom, worlds, name, mode, impl, monkeypatch):
    """The default slab-filter kernel (k_motions_v5, both modes), the cell-list kernels
    (k_motions_v4 analytic, k_motions_d32b discrete32) at the default block size and forced
    512/1024-thread blocks, and the generic k_motions, vs the oracle; includes edges
    parallel to an axis within the 1e-6 threshold."""
    impl, _, block = impl.partition("/")
    monkeypatch.setenv("EPP_MOTIONS_KERNEL", impl)
    monkeypatch.setenv("EPP_MOTIONS_BLOCK", block)  # "" = by LDS fit (the default)
    rg, ro, ws = worlds
    gates, obstacles, (lo, hi) = ws[name]
    ref = O.world_build(geom, gates, obstacles, rg, ro)
    w = capi.World(capi.build_obbs(geom, gates, obstacles), rg, ro)
    n = 100_000 if mode == 0 else 20_000
    s1, s2 = synth.edges(43, 8, lo, hi, n, max_len=0.5 if name != "c1" else 1.5)
    # near-parallel edges (|d_i| around the 1e-6 threshold of src/OBB.cpp:34)
    k = 2000
    t1 = synth.sample_states(5, lo, hi, k)
    t2 = t1.copy()
    t2[:, 0] += 0.8
    t2[:, 1] += np.where(np.arange(k) % 2, 9.9e-7, 1.01e-6)
    s1, s2 = np.vstack([s1, t1]), np.vstack([s2, t2])
    for cp in (0, 1):
        got = w.check_motions(s1, s2, cp, mode)
        exp = O.check_motions(ref, rg, ro, s1, s2, cp, mode, threads=8)
        assert exp.min() == 0 and exp.max() == 1
        assert np.array_equal(got, exp), (cp, np.flatnonzero(got != exp)[:10])


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("impl", ["lds", "v4", "generic"])
def test_motions_queue_overflow(geom, worlds, impl, mode, monkeypatch):
    """Long edges through the 512-OBB world: the LDS kernels flush their wave queues many
    times per wave (k_motions_v5: several queue windows per wave).  Answers still match
    the oracle."""
    monkeypatch.setenv("EPP_MOTIONS_KERNEL", impl)
    rg, ro, ws = worlds
    gates, obstacles, (lo, hi) = ws["c3"]
    ref = O.world_build(geom, gates, obstacles, rg, ro)
    w = capi.World(capi.build_obbs(geom, gates, obstacles), rg, ro)
    s1, s2 = synth.edges(61, 62, lo, hi, 20_000, max_len=6.0)
    for cp in (0, 1):
        got = w.check_motions(s1, s2, cp, mode)
        exp = O.check_motions(ref, rg, ro, s1, s2, cp, mode, threads=8)
        assert np.array_equal(got, exp), (cp, np.flatnonzero(got != exp)[:10])


@pytest.mark.parametrize("mode", [0, 1])
def test_motions_outside_and_across(geom, worlds, mode):
    """Edges beyond the world's box on every side (slab indices clamp to the end slabs),
    edges across the whole world, zero-length edges and edges touching AABB faces, through
    the default kernel vs the oracle."""
    rg, ro, ws = worlds
    gates, obstacles, (lo, hi) = ws["c3"]
    ref = O.world_build(geom, gates, obstacles, rg, ro)
    w = capi.World(capi.build_obbs(geom, gates, obstacles), rg, ro)
    rs = np.random.RandomState(17)
    lo, hi = np.asarray(lo, float), np.asarray(hi, float)
    far = rs.uniform(lo - 20, hi + 20, size=(20_000, 3))
    across = np.stack([rs.uniform(lo, hi, size=(5000, 3)), rs.uniform(lo, hi, size=(5000, 3))])
    bl, bh = ref["aabb_lo"], ref["aabb_hi"]
    face = np.where(rs.rand(5000, 1) < 0.5, bl[rs.randint(0, len(ref), 5000)], bh[rs.randint(0, len(ref), 5000)])
    s1 = np.vstack([far[:10_000], across[0], face, face])
    s2 = np.vstack([far[10_000:], across[1], face + rs.normal(size=(5000, 3)) * 0.2, face])
    for cp in (0, 1):
        got = w.check_motions(s1, s2, cp, mode)
        exp = O.check_motions(ref, rg, ro, s1, s2, cp, mode, threads=8)
        assert exp.min() == 0 and exp.max() == 1
        assert np.array_equal(got, exp), (cp, np.flatnonzero(got != exp)[:10])


def test_boundary_known_answers():
    f = json.load(open(os.path.join(GOLDEN, "obb_boundary.json")))

    def descs(lst):
        a = np.zeros(len(lst), config.OBB_DESC_DTYPE)
        for i, d in enumerate(lst):
            a[i]["pos"], a[i]["size"], a[i]["filling"] = d["pos"], d["size"], d["filling"]
        return a
    g = config.Geometry(descs(f["gate_desc"]), np.array([0, len(f["gate_desc"])], np.int32),
                        descs(f["obst_desc"]), np.array([1.0]))
    w = capi.World(capi.build_obbs(g, f["gates"], f["obstacles"]), f["r_gate"], f["r_obst"])
    for c in f["points"]:
        assert w.check_states(np.array([c["p"]]), c["can_pass"])[0] == c["valid"], c
    for c in f["mindist"]:
        assert w.check_states_mindist(np.array([c["p"]]), c["md"])[0] == c["valid"], c
    for c in f["rays"]:
        got = w.check_motions(np.array([c["s"]]), np.array([c["e"]]), c["can_pass"], c["mode"])[0]
        assert got == c["valid"], c


def test_golden_c1_states(geom):
    f = json.load(open(os.path.join(GOLDEN, "c1_states.json")))
    w = capi.World(capi.build_obbs(geom, f["gates"], f["obstacles"]), f["r_gate"], f["r_obst"])
    for cp in ("0", "1"):
        assert w.check_states(np.array(f["states"]), int(cp)).tolist() == f["valid"][cp]


def test_edge_sizes_and_alignment(geom, worlds):
    rg, ro, ws = worlds
    gates, obstacles, (lo, hi) = ws["c2"]
    ref = O.world_build(geom, gates, obstacles, rg, ro)
    w = capi.World(capi.build_obbs(geom, gates, obstacles), rg, ro)
    pts = synth.sample_states(3, lo, hi, 4099)
    exp = O.check_states(ref, rg, ro, pts, False)
    for n in (0, 1, 2, 3, 4, 5, 63, 64, 65, 255, 257, 1023, 4099):
        assert np.array_equal(w.check_states(pts[:n]), exp[:n]), n
    # unaligned input/output pointers (8-byte aligned xyz, odd flag offset)
    d = capi.DeviceBuffer(8 * 3 * 4099 + 64)
    d.upload(np.concatenate([[0.0], pts.ravel()]))
    v = capi.DeviceBuffer(4099 + 8)
    w.check_states_dev(d.ptr + 8, 4099, 0, v.ptr + 1)
    capi.sync()
    got = v.download(np.uint8, 4100)[1:]
    assert np.array_equal(got, exp)


def test_empty_world_and_update(geom, worlds):
    rg, ro, ws = worlds
    w = capi.World(np.zeros(0, capi.OBB_DTYPE), rg, ro)
    pts = synth.sample_states(3, *synth.C2_BOUNDS, 1000)
    assert w.check_states(pts).all()
    assert w.check_motions(pts, pts[::-1].copy()).all()
    gates, obstacles, _ = ws["c2"]
    w.update(capi.build_obbs(geom, gates, obstacles))
    ref = O.world_build(geom, gates, obstacles, rg, ro)
    assert np.array_equal(w.check_states(pts), O.check_states(ref, rg, ro, pts))


def test_global_memory_path_large_world(cfg, geom):
    """A world whose index exceeds the LDS budget runs the global-memory kernel variant."""
    rg, ro = config.inflate_radii(cfg)
    gates, obstacles = synth.track_world(5, n_gates=8, n_obstacles=3000)
    ref = O.world_build(geom, gates, obstacles, rg, ro)
    w = capi.World(capi.build_obbs(geom, gates, obstacles), rg, ro)
    pts = synth.sample_states(4, *synth.C2_BOUNDS, 50_000)
    assert np.array_equal(w.check_states(pts), O.check_states(ref, rg, ro, pts, threads=8))
    s1, s2 = synth.edges(1, 2, *synth.C2_BOUNDS, 20_000)
    assert np.array_equal(w.check_motions(s1, s2), O.check_motions(ref, rg, ro, s1, s2, threads=8))


# ---- worlds with "filling" OBBs (configs/config_filling.json: one per gate, the portal
# opening).  Reference semantics: a filling OBB is skipped by the state and ray checks when
# canPassGate (src/World.cpp:92-95, :150-153), always by the minDistance check (:116-119);
# its AABB is not inflated (src/OBB.cpp:117-121) and its point test is not inflated
# (src/OBB.h:54-57), but the ray slab test always inflates (src/OBB.cpp:28).
FILLING_CONFIG = os.path.join(os.path.dirname(GOLDEN), "..", "configs", "config_filling.json")


@pytest.fixture(scope="module")
def fworlds():
    cfg = config.load(FILLING_CONFIG)
    fgeom = config.geometry(cfg)
    assert fgeom.gate_desc["filling"].sum() == 2
    rg, ro, ws = _worlds(cfg, fgeom)
    return fgeom, rg, ro, ws


def _gate_openings(gates, geom, n_per_gate=400, seed=3):
    """States in and around every gate opening (the filling boxes), in world coordinates."""
    rs = np.random.RandomState(seed)
    out = []
    for g in gates:
        h = geom.gate_height[int(g[6])]
        loc = rs.uniform([-0.3, -0.05, -0.3], [0.3, 0.05, 0.3], size=(n_per_gate, 3))
        c, s = np.cos(g[5]), np.sin(g[5])
        out.append(np.stack([g[0] + c * loc[:, 0] - s * loc[:, 1], g[1] + s * loc[:, 0] + c * loc[:, 1],
                             h + loc[:, 2]], 1))
    return np.vstack(out)


@pytest.mark.parametrize("kernel", ["v5", "v4", "generic"])
@pytest.mark.parametrize("name", ["c1", "c2", "c3"])
def test_filling_states_bit_exact(fworlds, name, kernel, monkeypatch):
    monkeypatch.setenv("EPP_STATES_KERNEL", kernel)
    fgeom, rg, ro, ws = fworlds
    gates, obstacles, (lo, hi) = ws[name]
    ref = O.world_build(fgeom, gates, obstacles, rg, ro)
    assert sum(int(o["filling"]) for o in ref) == len(gates)
    w = capi.World(capi.build_obbs(fgeom, gates, obstacles), rg, ro)
    pts = np.vstack([synth.sample_states(17, lo, hi, 100_003), _gate_openings(gates, fgeom),
                     _adversarial_points(ref)])
    res = {}
    for cp in (0, 1):
        got = w.check_states(pts, cp)
        exp = O.check_states(ref, rg, ro, pts, cp, threads=8)
        assert exp.min() == 0 and exp.max() == 1
        assert np.array_equal(got, exp), (cp, np.flatnonzero(got != exp)[:10])
        res[cp] = exp
    # the filling boxes decide: states in an opening are invalid unless the gate may be passed
    assert (res[1] >= res[0]).all() and (res[1] > res[0]).sum() >= 20
    for md in (0.0, 0.1, 0.3):  # minDistance skips every filling OBB
        assert np.array_equal(w.check_states_mindist(pts, md), O.check_states_mindist(ref, pts, md)), md


@pytest.mark.parametrize("kernel", ["lds", "v4", "generic"])
@pytest.mark.parametrize("name", ["c1", "c2", "c3"])
@pytest.mark.parametrize("mode", [0, 1])
def test_filling_motions_bit_exact(fworlds, name, mode, kernel, monkeypatch):
    monkeypatch.setenv("EPP_MOTIONS_KERNEL", kernel)
    fgeom, rg, ro, ws = fworlds
    gates, obstacles, (lo, hi) = ws[name]
    ref = O.world_build(fgeom, gates, obstacles, rg, ro)
    w = capi.World(capi.build_obbs(fgeom, gates, obstacles), rg, ro)
    n = 60_000 if mode == 0 else 15_000
    s1, s2 = synth.edges(45, 9, lo, hi, n, max_len=0.5 if name != "c1" else 1.5)
    # edges through the openings, along the gate normal (the way a drone passes a gate)
    a = _gate_openings(gates, fgeom, 300, seed=5)
    yaw = np.repeat(gates[:, 5], 300)
    nrm = np.stack([-np.sin(yaw), np.cos(yaw), np.zeros_like(yaw)], 1)
    s1, s2 = np.vstack([s1, a - 0.4 * nrm]), np.vstack([s2, a + 0.4 * nrm])
    res = {}
    for cp in (0, 1):
        got = w.check_motions(s1, s2, cp, mode)
        exp = O.check_motions(ref, rg, ro, s1, s2, cp, mode, threads=8)
        assert exp.min() == 0 and exp.max() == 1
        assert np.array_equal(got, exp), (cp, np.flatnonzero(got != exp)[:10])
        res[cp] = exp
    assert (res[1] >= res[0]).all() and (res[1] > res[0]).sum() >= 20


@pytest.mark.parametrize("n", [1 << 20, 5 << 20])
def test_filling_states_full_size(fworlds, n):
    """BASELINE C2 size with filling OBBs, both can_pass_gate outcomes, bit-exact."""
    fgeom, rg, ro, ws = fworlds
    gates, obstacles, (lo, hi) = ws["c2"]
    ref = O.world_build(fgeom, gates, obstacles, rg, ro)
    w = capi.World(capi.build_obbs(fgeom, gates, obstacles), rg, ro)
    pts = synth.sample_states(7, lo, hi, n)
    e0 = O.check_states(ref, rg, ro, pts, False, threads=8)
    e1 = O.check_states(ref, rg, ro, pts, True, threads=8)
    assert (e1 > e0).sum() > 0
    assert np.array_equal(w.check_states(pts, False), e0)
    assert np.array_equal(w.check_states(pts, True), e1)


def test_graph_replay_matches_direct_launch(geom, worlds):
    """bench.py times replayed HIP graphs of epp_check_states: K captured launches over
    rotating batches give the same flags as direct launches and as the oracle."""
    import ctypes as C
    L = capi.lib()
    rg, ro, ws = worlds
    gates, obstacles, (lo, hi) = ws["c2"]
    ref = O.world_build(geom, gates, obstacles, rg, ro)
    w = capi.World(capi.build_obbs(geom, gates, obstacles), rg, ro)
    n, nb = 200_000, 3
    pts = [synth.sample_states(77 + b, lo, hi, n) for b in range(nb)]
    d_in = [capi.DeviceBuffer.from_array(p) for p in pts]
    d_out = [capi.DeviceBuffer(n) for _ in range(nb)]
    s = C.c_void_p()
    capi.check(L.epp_stream_create(C.byref(s)))
    g = C.c_void_p()
    gen0 = w.generation()
    capi.check(L.epp_graph_begin(s.value))
    for k in range(2 * nb):
        w.check_states_dev(d_in[k % nb].ptr, n, 0, d_out[k % nb].ptr, stream=s.value)
    capi.check(L.epp_graph_end(s.value, C.byref(g)))
    for b in range(nb):
        d_out[b].zero()
    capi.sync()
    capi.check(L.epp_graph_launch(g.value, s.value))
    capi.check(L.epp_stream_sync(s.value))
    for b in range(nb):
        got = d_out[b].download(np.uint8, n)
        assert np.array_equal(got, w.check_states(pts[b]))
        assert np.array_equal(got, O.check_states(ref, rg, ro, pts[b], False, threads=8))
    capi.check(L.epp_graph_destroy(g.value))
    # an update is a new version: captured graphs must be re-captured, after the index
    # is rebuilt (epp.h); a capture over a rebuilt index replays the new world
    g2 = np.array(gates, float)
    g2[:, 0] += 0.15
    w.update(capi.build_obbs(geom, g2, obstacles))
    assert w.generation() == gen0 + 1
    w.build_index()
    ref2 = O.world_build(geom, g2, obstacles, rg, ro)
    capi.check(L.epp_graph_begin(s.value))
    w.check_states_dev(d_in[0].ptr, n, 0, d_out[0].ptr, stream=s.value)
    capi.check(L.epp_graph_end(s.value, C.byref(g)))
    d_out[0].zero()
    capi.sync()
    capi.check(L.epp_graph_launch(g.value, s.value))
    capi.check(L.epp_stream_sync(s.value))
    assert np.array_equal(d_out[0].download(np.uint8, n), O.check_states(ref2, rg, ro, pts[0], False, threads=8))
    capi.check(L.epp_graph_destroy(g.value))
    L.epp_stream_destroy(s.value)


def test_world_update_small_queries_zero_copy(cfg, geom, worlds):
    """The C++ World's host-array queries (zero-copy below 16384 queries, DMA above) after
    gate-pose updates agree with the oracle rebuilt from the same poses."""
    import online_traj_planner as otp
    rg, ro, ws = worlds
    gates, obstacles, (lo, hi) = ws["c2"]
    from conftest import CONFIG
    pp = otp.PathPlanner(gates, obstacles, CONFIG)
    rs = np.random.RandomState(0)
    g = np.array(gates, float)
    for step in range(6):
        k = step % len(g)
        g[k, 0] += rs.uniform(-0.1, 0.1)
        g[k, 5] += rs.uniform(-0.1, 0.1)
        pp.update_gate_pos(k, list(g[k, :6]))
        ref = O.world_build(geom, g, obstacles, rg, ro)
        for n in (1, 100, 20_000):
            pts = synth.sample_states(300 + step, lo, hi, n)
            rows = np.zeros((n, 10))
            rows[:, [0, 3, 6]] = pts
            exp = O.check_states_mindist(ref, pts, 0.1)
            assert pp.check_trajectory_validity(rows, 0.1) == bool(exp.all())
            for p, e in zip(pts[:50], O.check_states(ref, rg, ro, pts[:50], False)):
                assert pp.check_point_validity(p, False) == bool(e)


@pytest.mark.parametrize("name", ["c1", "c2"])
def test_small_query_path(fworlds, name, monkeypatch):
    """Small batches (<= 4096 states / 1024 edges on worlds of <= 256 OBBs) take the
    brute-force kernels of small.hip: with a current index (records from the device blob),
    after epp_world_update (stale index: records read from the pinned host copy), and a
    large query afterwards rebuilds the index.  Every answer vs the oracle, both can_pass
    values, both motion modes, minDistance; and equal to the index kernels' answers."""
    fgeom, rg, ro, ws = fworlds
    gates, obstacles, (lo, hi) = ws[name]
    w = capi.World(capi.build_obbs(fgeom, gates, obstacles), rg, ro)
    rs = np.random.RandomState(11)
    g = np.array(gates, float)
    for version in range(3):
        if version:
            g[:, 0] += rs.uniform(-0.2, 0.2, len(g))
            g[:, 5] += rs.uniform(-0.2, 0.2, len(g))
            w.update(capi.build_obbs(fgeom, g, obstacles))  # index stale until a large query
        ref = O.world_build(fgeom, g, obstacles, rg, ro)
        a = _gate_openings(g, fgeom, 200, seed=version)
        pts = np.vstack([synth.sample_states(40 + version, lo, hi, 4096 - len(a)), a])  # 4096: still "small"
        yaw = np.repeat(g[:, 5], 200)[:1024 - 500]
        nrm = np.stack([-np.sin(yaw), np.cos(yaw), np.zeros_like(yaw)], 1)
        e1, e2 = synth.edges(50 + version, 51, lo, hi, 500, max_len=1.0)
        s1 = np.vstack([e1, a[:len(yaw)] - 0.4 * nrm])
        s2 = np.vstack([e2, a[:len(yaw)] + 0.4 * nrm])
        for cp in (0, 1):
            exp = O.check_states(ref, rg, ro, pts, cp)
            for n in (1, 37, len(pts)):
                assert np.array_equal(w.check_states(pts[:n], cp), exp[:n]), (version, cp, n)
            for mode in (0, 1):
                exp_m = O.check_motions(ref, rg, ro, s1, s2, cp, mode, threads=8)
                assert exp_m.min() == 0 and exp_m.max() == 1
                assert np.array_equal(w.check_motions(s1, s2, cp, mode), exp_m), (version, cp, mode)
        for md in (0.0, 0.2):
            assert np.array_equal(w.check_states_mindist(pts, md), O.check_states_mindist(ref, pts, md))
        # the index kernels agree (forced; the first call after an update rebuilds the index)
        monkeypatch.setenv("EPP_STATES_KERNEL", "v5")
        monkeypatch.setenv("EPP_MOTIONS_KERNEL", "v5")
        assert np.array_equal(w.check_states(pts, 1), O.check_states(ref, rg, ro, pts, 1))
        assert np.array_equal(w.check_motions(s1, s2, 1, 1), O.check_motions(ref, rg, ro, s1, s2, 1, 1))
        monkeypatch.delenv("EPP_STATES_KERNEL")
        monkeypatch.delenv("EPP_MOTIONS_KERNEL")
    # a large query after an update rebuilds the index on its own
    g[0, 1] += 0.3
    w.update(capi.build_obbs(fgeom, g, obstacles))
    ref = O.world_build(fgeom, g, obstacles, rg, ro)
    big = synth.sample_states(99, lo, hi, 50_000)
    assert np.array_equal(w.check_states(big), O.check_states(ref, rg, ro, big, threads=8))


def test_async_small_queries_across_updates(fworlds):
    """Asynchronous small queries on a stale index read the pinned records of their
    version; the updates in between go to the other record slot, and an update that
    reuses a slot waits for the queued kernels reading it (no device-wide wait).  Four
    versions queued back to back on one stream without host synchronisation, each
    answer vs the oracle of its version."""
    import ctypes as C
    fgeom, rg, ro, ws = fworlds
    gates, obstacles, (lo, hi) = ws["c2"]
    w = capi.World(capi.build_obbs(fgeom, gates, obstacles), rg, ro)
    L = capi.lib()
    st = C.c_void_p()
    capi.check(L.epp_stream_create(C.byref(st)))
    rs = np.random.RandomState(21)
    g = np.array(gates, float)
    pts = np.vstack([synth.sample_states(70, lo, hi, 4000), _gate_openings(g, fgeom, 12, seed=3)])
    s1, s2 = synth.edges(71, 72, lo, hi, 1000, max_len=1.0)
    d_pts, d1, d2 = (capi.DeviceBuffer.from_array(a) for a in (pts, s1, s2))
    outs, refs = [], []
    for version in range(4):
        if version:
            g[:, 0] += rs.uniform(-0.2, 0.2, len(g))
            g[:, 5] += rs.uniform(-0.2, 0.2, len(g))
            w.update(capi.build_obbs(fgeom, g, obstacles))
        refs.append(O.world_build(fgeom, g, obstacles, rg, ro))
        o_s, o_m = capi.DeviceBuffer(len(pts)), capi.DeviceBuffer(len(s1))
        w.check_states_dev(d_pts.ptr, len(pts), 1, o_s.ptr, stream=st.value)
        w.check_motions_dev(d1.ptr, d2.ptr, len(s1), 0, 1, o_m.ptr, stream=st.value)
        outs.append((o_s, o_m))
    capi.check(L.epp_stream_sync(st.value))
    for (o_s, o_m), ref in zip(outs, refs):
        assert np.array_equal(o_s.download(np.uint8, len(pts)), O.check_states(ref, rg, ro, pts, 1))
        assert np.array_equal(o_m.download(np.uint8, len(s1)), O.check_motions(ref, rg, ro, s1, s2, 0, 1, threads=8))
    L.epp_stream_destroy(st.value)


@pytest.mark.parametrize("name", ["c2", "c3"])
@pytest.mark.parametrize("filling", [False, True])
def test_knn_motions_equal_materialised(cfg, geom, fworlds, name, filling):
    """epp_check_knn_motions (edges read off a k-NN table, no endpoint arrays) gives the
    CPU oracle's flags for the same edges (World::checkRayValid / the 32-step check, src/
    World.cpp:130-162) and those of epp_knn_edges + epp_check_motions, both modes and
    can_pass_gate values, missing neighbours (-1) and edges far longer than a tile
    included."""
    if filling:
        g_, rg, ro, ws = fworlds
    else:
        g_ = geom
        rg, ro, ws = _worlds(cfg, geom)
    gates, obstacles, (lo, hi) = ws[name]
    w = capi.World(capi.build_obbs(g_, gates, obstacles), rg, ro)
    rs = np.random.RandomState(11)
    n, k = 6000, 16
    nodes = rs.uniform(lo, hi, size=(n, 3))
    near = np.clip(np.arange(n)[:, None] + rs.randint(-40, 41, size=(n, k)), 0, n - 1)
    far = rs.randint(0, n, size=(n, k))  # long edges across many tiles
    nbr = np.where(rs.rand(n, k) < 0.9, near, far).astype(np.int32)
    nbr[rs.rand(n, k) < 0.03] = -1
    s1, s2 = capi.knn_edges(nodes, nbr)
    # the edges the table denotes, built on the host (a missing neighbour: the node to itself)
    src = np.repeat(np.arange(n), k)
    dst = np.where(nbr.reshape(-1) < 0, src, nbr.reshape(-1))
    assert np.array_equal(s1, nodes[src]) and np.array_equal(s2, nodes[dst])
    ref = O.world_build(g_, gates, obstacles, rg, ro)
    d_n, d_k, d_v = capi.DeviceBuffer.from_array(nodes), capi.DeviceBuffer.from_array(nbr), capi.DeviceBuffer(n * k)
    for mode in (0, 1):
        for cp in (0, 1):
            exp = O.check_motions(ref, rg, ro, nodes[src], nodes[dst], bool(cp), mode, threads=8)
            want = w.check_motions(s1, s2, bool(cp), mode)
            assert np.array_equal(want, exp), (mode, cp)
            capi.check(capi.lib().epp_check_knn_motions(w.handle, d_n.ptr, d_k.ptr, n, k, cp, mode, d_v.ptr, None))
            capi.sync()
            got = d_v.download(np.uint8, n * k)
            assert np.array_equal(got, exp), (mode, cp, int((got != exp).sum()))


def test_knn_motions_unsupported_small_batch(cfg, geom):
    rg, ro, ws = _worlds(cfg, geom)
    gates, obstacles, (lo, hi) = ws["c2"]
    w = capi.World(capi.build_obbs(geom, gates, obstacles), rg, ro)
    nodes = np.random.RandomState(1).uniform(lo, hi, size=(8, 3))
    nbr = np.zeros((8, 4), np.int32)
    d_n, d_k, d_v = capi.DeviceBuffer.from_array(nodes), capi.DeviceBuffer.from_array(nbr), capi.DeviceBuffer(32)
    rc = capi.lib().epp_check_knn_motions(w.handle, d_n.ptr, d_k.ptr, 8, 4, 0, 0, d_v.ptr, None)
    assert rc == capi.EPP_ERR_UNSUPPORTED


def test_updates_racing_large_checks(geom, worlds):
    """One thread updates the world back and forth between C2 (64 OBBs) and C3 (512 OBBs:
    the index grows, the device blob is reallocated) while another launches large state and
    motion checks.  A launch holds its snapshot of the device index until it is queued
    (IndexLease), so every answer is the oracle's for one of the two versions, never a mix
    or a read of a freed blob."""
    import threading
    rg, ro, ws = worlds
    (g2, o2, (lo, hi)), (g3, o3, _) = ws["c2"], ws["c3"]
    obbs = [capi.build_obbs(geom, g2, o2), capi.build_obbs(geom, g3, o3)]
    refs = [O.world_build(geom, g2, o2, rg, ro), O.world_build(geom, g3, o3, rg, ro)]
    pts = synth.sample_states(11, lo, hi, 1 << 17)
    s1, s2 = synth.edges(12, 8, lo, hi, 1 << 14)
    exp_s = [O.check_states(r, rg, ro, pts) for r in refs]
    exp_m = [O.check_motions(r, rg, ro, s1, s2) for r in refs]
    world = capi.World(obbs[0], rg, ro)
    stop, err = threading.Event(), []

    def updater():
        k = 1
        try:
            while not stop.is_set():
                world.update(obbs[k % 2])
                k += 1
        except Exception as e:  # pragma: no cover - reported below
            err.append(e)

    t = threading.Thread(target=updater)
    t.start()
    try:
        for i in range(24):
            got = world.check_states(pts)
            assert any(np.array_equal(got, e) for e in exp_s), f"states call {i}: no version matches"
            got = world.check_motions(s1, s2)
            assert any(np.array_equal(got, e) for e in exp_m), f"motions call {i}: no version matches"
    finally:
        stop.set()
        t.join()
    assert not err, err
    world.close()


def test_updates_racing_small_checks(geom, worlds):
    """small-path checks (<= 4096 states / 1024 edges, <= 256 OBBs) read the
    pinned host records of the newest version while the index is stale.  One thread runs
    back-to-back updates over three versions (64 OBBs, 190 OBBs: the pinned slot is
    reallocated, 64 OBBs with every gate moved) while another launches small checks: a
    launcher holds its snapshot of the records until its kernel is queued and its reader
    recorded, so every answer is the oracle's for one version."""
    import threading
    rg, ro, ws = worlds
    g2, o2, (lo, hi) = ws["c2"]
    gb, ob = synth.track_world(42, n_obstacles=150)
    gm = g2.copy()
    gm[:, :2] += 0.3
    gm[:, 5] += 0.2
    versions = [(g2, o2), (gb, ob), (gm, o2)]
    obbs = [capi.build_obbs(geom, g, o) for g, o in versions]
    assert all(len(b) <= 256 for b in obbs) and len(obbs[1]) > 2 * len(obbs[0])
    refs = [O.world_build(geom, g, o, rg, ro) for g, o in versions]
    pts = synth.sample_states(13, lo, hi, 4096)
    s1, s2 = synth.edges(14, 9, lo, hi, 1024)
    exp_s = [O.check_states(r, rg, ro, pts) for r in refs]
    exp_m = [O.check_motions(r, rg, ro, s1, s2) for r in refs]
    assert not np.array_equal(exp_s[0], exp_s[2]) and not np.array_equal(exp_s[0], exp_s[1])
    world = capi.World(obbs[0], rg, ro)
    world.update(obbs[1])  # index stale from here on: every check below reads pinned records
    stop, err = threading.Event(), []

    def updater():
        k = 2
        try:
            while not stop.is_set():
                world.update(obbs[k % 3])
                world.update(obbs[(k + 1) % 3])  # two updates back to back
                k += 1
        except Exception as e:  # pragma: no cover - reported below
            err.append(e)

    t = threading.Thread(target=updater)
    t.start()
    try:
        for i in range(200):
            got = world.check_states(pts)
            assert any(np.array_equal(got, e) for e in exp_s), f"states call {i}: no version matches"
            got = world.check_motions(s1, s2)
            assert any(np.array_equal(got, e) for e in exp_m), f"motions call {i}: no version matches"
    finally:
        stop.set()
        t.join()
    assert not err, err
    world.close()


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("can_pass", [0, 1])
def test_c3_motions_full_bench_size(geom, worlds, mode, can_pass):
    """BASELINE C3 at the bench's own size and inputs (bench.py side_measurements: 512 OBBs,
    1,048,576 edges from seeds 43 / 8): analytic and 32-step discretised flags bit-exact
    against the oracle (World::checkRayValid, src/World.cpp:130-162), both can_pass_gate
    values -- the grid and window-count shape of the bench launch itself."""
    rg, ro, ws = worlds
    g3, o3, (lo, hi) = ws["c3"]
    ref = O.world_build(geom, g3, o3, rg, ro)
    w = capi.World(capi.build_obbs(geom, g3, o3), rg, ro)
    s1, s2 = synth.edges(43, 8, lo, hi, 1 << 20)
    got = w.check_motions(s1, s2, bool(can_pass), mode)
    exp = O.check_motions(ref, rg, ro, s1, s2, bool(can_pass), mode, threads=16)
    assert 0 < int(exp.sum()) < len(exp)
    assert np.array_equal(got, exp), int((got != exp).sum())
    w.close()


def test_world_buffers_reused_across_worlds(geom, worlds):
    """Destroyed worlds leave their pinned and device buffers to the next world on the
    device (a fresh PathPlanner per request allocates nothing): worlds of growing and
    shrinking size created one after the other keep the oracle's answers (the device blob
    and the record slots grow when a reused buffer is too small)."""
    rg, ro, ws = worlds
    lo, hi = synth.C2_BOUNDS
    pts = synth.sample_states(31, lo, hi, 50_000)
    small = synth.sample_states(32, lo, hi, 1000)
    for name in ("c2", "c3", "c1", "c3", "c2"):
        g, o, _ = ws[name]
        ref = O.world_build(geom, g, o, rg, ro)
        w = capi.World(capi.build_obbs(geom, g, o), rg, ro)
        assert np.array_equal(w.check_states(pts), O.check_states(ref, rg, ro, pts, threads=8)), name
        assert np.array_equal(w.check_states(small), O.check_states(ref, rg, ro, small)), name
        w.close()
