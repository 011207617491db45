"""CPU tests of the product boundary: libepp.so loads, exports every symbol of
include/epp.h, and its host-side world build (no GPU involved) matches the oracle
bit for bit."""
import ctypes
import os
import re

import numpy as np
import pytest

import oracle as O
from eppamd import capi, config, synth

from conftest import ROOT


def _header_functions():
    src = open(os.path.join(ROOT, "include", "epp.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(epp_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_header_symbol():
    lib = ctypes.CDLL(capi.LIB_PATH)
    declared = _header_functions()
    assert len(declared) >= 25
    for name in declared:
        assert hasattr(lib, name), name
    assert sorted(capi.EXPORTED) == declared


def test_pybind_modules_present():
    pkg = os.path.join(ROOT, "efficient-path-planner_amd")
    names = os.listdir(pkg)
    for mod in ("polynomial_trajectory", "online_traj_planner"):
        assert any(n.startswith(mod) and n.endswith(".so") for n in names), mod


@pytest.mark.parametrize("seed", [42, 100, 107])
def test_build_obbs_matches_oracle(cfg, geom, seed):
    rg, ro = config.inflate_radii(cfg)
    gates, obstacles = synth.track_world(seed)
    mine = capi.build_obbs(geom, gates, obstacles)
    ref = O.world_build(geom, gates, obstacles, rg, ro)
    assert len(mine) == len(ref) == 8 * 5 + 24
    for f in ("center", "half", "rot"):
        assert np.array_equal(mine[f], ref[f]), f
    assert np.array_equal(mine["filling"], ref["filling"])
    assert np.array_equal(mine["is_gate"], ref["is_gate"])


def test_build_obbs_errors(geom):
    with pytest.raises(capi.EppError) as e:
        capi.build_obbs(geom, [[0, 0, 0, 0.0, 0.2, 0, 0]], np.zeros((0, 6)))
    assert e.value.code == capi.EPP_ERR_UNSUPPORTED and "y axis" in str(e.value)
    with pytest.raises(capi.EppError) as e:
        capi.build_obbs(geom, np.zeros((0, 7)), [[0, 0, 0.01, 0, 0, 0]])
    assert e.value.code == capi.EPP_ERR_RUNTIME and "z position" in str(e.value)
    with pytest.raises(capi.EppError):
        capi.build_obbs(geom, [[0, 0, 0, 0, 0, 0, 7]], np.zeros((0, 6)))
    # gate z is forced to 0 (src/PathPlanner.cpp:68); negative obstacle z is accepted
    a = capi.build_obbs(geom, [[1, 2, 3.0, 0, 0, 0.3, 1]], [[0, 0, -0.5, 0, 0, 0]])
    b = capi.build_obbs(geom, [[1, 2, 0.0, 0, 0, 0.3, 1]], [[0, 0, -0.5, 0, 0, 0]])
    assert np.array_equal(a, b)


def test_knn_workspace_size_host_only():
    """epp_knn_workspace_size is host arithmetic (no GPU): 0 for n <= 0, grows with n,
    256-byte granular."""
    L = capi.lib()
    assert L.epp_knn_workspace_size(0) == 0
    a, b = L.epp_knn_workspace_size(3000), L.epp_knn_workspace_size(65538)
    assert 0 < a < b and a % 256 == 0 and b % 256 == 0
    assert b >= 65538 * (4 + 4 + 24 + 3 * 4)


def test_sparse_byte_classes_match_the_class_table():
    """k_states_v5's staged byte classes (sparse: an occupancy word with the rank of its
    first occupied cell per 32 cells, then the class bytes of the occupied cells) decode,
    cell by cell with the kernel's lookup, to the class table of the index (host build, no
    GPU): C1, C2, C2 with filling boxes, and a 190-OBB world."""
    import ctypes as C
    from eppamd import config, synth
    from conftest import ROOT
    L = capi.lib()
    f = L.epp_dbg_check_sparse_classes
    f.restype = C.c_int64
    f.argtypes = [C.c_void_p, C.c_int32, C.c_double, C.c_double]
    checked = 0
    for cfg_name in ("config.json", "config_filling.json"):
        cfg = config.load(os.path.join(ROOT, "configs", cfg_name))
        geom = config.geometry(cfg)
        rg, ro = config.inflate_radii(cfg)
        g1, o1, _, _ = synth.c1_world()
        for g, o in ((g1, o1), synth.track_world(42), synth.track_world(42, n_obstacles=150)):
            obbs = capi.build_obbs(geom, g, o)
            r = f(obbs.ctypes.data, len(obbs), rg, ro)
            assert r in (0, -1), r
            checked += r == 0
    assert checked >= 4


def test_planner_abi_guard_rejects_stale_caller(tmp_path):
    """epp/PathPlanner.h hands the caller's compiled sizes of PathPlanner / PlannerStats and
    the layout version to the library's constructor (a stale tools/c5_native
    segfaulted after PlannerStats grew).  A caller with another layout gets
    std::runtime_error before anything else runs (no GPU needed).  The current header's own
    tag passes: every GPU test constructs PathPlanner through it."""
    import subprocess
    src = tmp_path / "abi.cpp"
    src.write_text(r'''
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include "epp/PathPlanner.h"
int main() {
    epp::Matrix g(0, 7), o(0, 6);
    using Tag = epp::PathPlanner::AbiTag;
    const Tag stale{(uint32_t)sizeof(epp::PathPlanner), (uint32_t)sizeof(epp::PlannerStats) - 8, epp::kPlannerAbiVersion};
    const Tag old{(uint32_t)sizeof(epp::PathPlanner), (uint32_t)sizeof(epp::PlannerStats), epp::kPlannerAbiVersion - 1};
    int rejected = 0;
    for (const Tag& t : {stale, old}) {
        try { epp::PathPlanner p(g, o, nullptr, t); } catch (const std::runtime_error& e) {
            rejected += std::strstr(e.what(), "rebuild the caller") != nullptr; }
    }
    epp::PlannerStats s;
    std::printf("%d %d\n", rejected, (int)(s.size == sizeof(epp::PlannerStats) && s.version == epp::kPlannerAbiVersion));
    return 0;
}
''')
    exe = tmp_path / "abi"
    pkg = os.path.join(ROOT, "efficient-path-planner_amd")
    subprocess.run(["g++", "-std=c++17", "-O0", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe),
                    "-L", pkg, "-lepp", f"-Wl,-rpath,{pkg}"], check=True, capture_output=True, timeout=120)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60)
    assert out.returncode == 0, out.stderr[-2000:]
    assert out.stdout.split() == ["2", "1"], out.stdout
