"""TEST INFRASTRUCTURE ONLY — ctypes binding of the CPU oracle (oracle/liboracle.so).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this.
See epp_oracle.h for what it restates and how it is pinned.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "liboracle.so")

OR_OBB_DTYPE = np.dtype([("center", "<f8", 3), ("half", "<f8", 3), ("rot", "<f8", 9),
                         ("aabb_lo", "<f8", 3), ("aabb_hi", "<f8", 3),
                         ("filling", "<i4"), ("is_gate", "<i4")])

_lib = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        l = C.CDLL(LIB_PATH)
        vp, i32, i64, dp, u64 = C.c_void_p, C.c_int, C.c_int64, C.c_double, C.c_uint64
        sig = {
            "or_world_build": (i32, [vp, vp, i32, vp, i32, vp, i32, vp, i32, dp, dp, vp, i32]),
            "or_point_valid": (i32, [vp, i32, dp, dp, vp, i32]),
            "or_point_valid_mindist": (i32, [vp, i32, vp, dp]),
            "or_ray_valid": (i32, [vp, i32, dp, dp, vp, vp, i32]),
            "or_check_states": (None, [vp, i32, dp, dp, vp, i64, i32, vp]),
            "or_check_states_mindist": (None, [vp, i32, vp, i64, dp, vp]),
            "or_check_motions": (None, [vp, i32, dp, dp, vp, vp, i64, i32, i32, vp]),
            "or_check_states_mt": (None, [vp, i32, dp, dp, vp, i64, i32, vp, i32]),
            "or_check_motions_mt": (None, [vp, i32, dp, dp, vp, vp, i64, i32, i32, vp, i32]),
            "or_sample_states": (None, [u64, vp, vp, i64, vp]),
            "or_segment_times": (None, [vp, i32, i32, dp, dp, vp]),
            "or_minsnap_solve": (i32, [vp, vp, i32, i32, vp, i32, vp]),
            "or_minsnap_track": (i32, [vp, i32, dp, dp, vp, vp, vp, vp]),
            "or_minsnap_batch_mt": (None, [vp, vp, i32, dp, dp, vp, vp, vp, i32]),
            "or_sample_traj": (i64, [vp, vp, i32, dp, dp, vp, i64]),
            "or_generate_trajectory": (i64, [vp, i32, dp, dp, dp, dp, vp, vp, vp, i64]),
            "or_mapping_matrix": (None, [dp, vp]),
            "or_invert_mapping": (None, [vp, vp]),
            "or_poly_eval": (dp, [vp, dp, i32]),
            "or_random_vertices": (None, [i32, i32, dp, dp, u64, vp]),
            "or_plan_once": (i32, [vp, i32, dp, dp, vp, vp, vp, vp, i64, u64, i32, i32, i32, vp, i32, vp]),
        }
        for name, (res, args) in sig.items():
            f = getattr(l, name)
            f.restype = res
            f.argtypes = args
        _lib = l
    return _lib


def _p(a):
    return a.ctypes.data if a is not None and a.size else None


def world_build(geom, gates, obstacles, r_gate, r_obst) -> np.ndarray:
    gates = np.ascontiguousarray(np.asarray(gates, np.float64).reshape(-1, 7))
    obstacles = np.ascontiguousarray(np.asarray(obstacles, np.float64).reshape(-1, 6))
    cap = len(gates) * max(1, len(geom.gate_desc)) + len(obstacles) * max(1, len(geom.obst_desc)) + 1
    out = np.zeros(cap, OR_OBB_DTYPE)
    n = lib().or_world_build(_p(geom.gate_desc), _p(geom.gate_desc_off), len(geom.gate_desc_off) - 1,
                             _p(geom.obst_desc), len(geom.obst_desc), _p(gates), len(gates), _p(obstacles),
                             len(obstacles), r_gate, r_obst, _p(out), cap)
    if n < 0:
        raise ValueError(f"or_world_build failed: {n}")
    return out[:n].copy()


def check_states(w, r_gate, r_obst, xyz, can_pass_gate=False, threads=1):
    xyz = np.ascontiguousarray(xyz, np.float64).reshape(-1, 3)
    out = np.zeros(len(xyz), np.uint8)
    if threads > 1:
        lib().or_check_states_mt(_p(w), len(w), r_gate, r_obst, _p(xyz), len(xyz), int(can_pass_gate),
                                 _p(out), threads)
    else:
        lib().or_check_states(_p(w), len(w), r_gate, r_obst, _p(xyz), len(xyz), int(can_pass_gate), _p(out))
    return out


def check_states_mindist(w, xyz, min_distance):
    xyz = np.ascontiguousarray(xyz, np.float64).reshape(-1, 3)
    out = np.zeros(len(xyz), np.uint8)
    lib().or_check_states_mindist(_p(w), len(w), _p(xyz), len(xyz), float(min_distance), _p(out))
    return out


def check_motions(w, r_gate, r_obst, s1, s2, can_pass_gate=False, mode=0, threads=1):
    s1 = np.ascontiguousarray(s1, np.float64).reshape(-1, 3)
    s2 = np.ascontiguousarray(s2, np.float64).reshape(-1, 3)
    out = np.zeros(len(s1), np.uint8)
    if threads > 1:
        lib().or_check_motions_mt(_p(w), len(w), r_gate, r_obst, _p(s1), _p(s2), len(s1), int(can_pass_gate),
                                  int(mode), _p(out), threads)
    else:
        lib().or_check_motions(_p(w), len(w), r_gate, r_obst, _p(s1), _p(s2), len(s1), int(can_pass_gate),
                               int(mode), _p(out))
    return out


def sample_states(seed, lo, hi, n):
    lo = np.ascontiguousarray(lo, np.float64)
    hi = np.ascontiguousarray(hi, np.float64)
    out = np.zeros((n, 3))
    lib().or_sample_states(seed, _p(lo), _p(hi), n, _p(out))
    return out


def segment_times(wp, v_max, a_max):
    wp = np.ascontiguousarray(wp, np.float64)
    dim = wp.shape[1]
    out = np.zeros(len(wp) - 1)
    lib().or_segment_times(_p(wp), len(wp), dim, v_max, a_max, _p(out))
    return out


def minsnap_solve(fixed_mask, fixed_val, times, dim, derivative=4):
    fixed_mask = np.ascontiguousarray(fixed_mask, np.uint8)
    fixed_val = np.ascontiguousarray(fixed_val, np.float64)
    times = np.ascontiguousarray(times, np.float64)
    nv = len(times) + 1
    coeffs = np.zeros((len(times), dim, 10))
    rc = lib().or_minsnap_solve(_p(fixed_mask), _p(fixed_val), nv, dim, _p(times), derivative, _p(coeffs))
    if rc < 0:
        raise RuntimeError(f"or_minsnap_solve failed {rc}")
    return coeffs


def minsnap_track(wp, v_max, a_max, v0=(0, 0, 0), a0=(0, 0, 0)):
    wp = np.ascontiguousarray(wp, np.float64).reshape(-1, 3)
    v0 = np.ascontiguousarray(v0, np.float64)
    a0 = np.ascontiguousarray(a0, np.float64)
    T = np.zeros(len(wp) - 1)
    Cf = np.zeros((len(wp) - 1, 3, 10))
    rc = lib().or_minsnap_track(_p(wp), len(wp), v_max, a_max, _p(v0), _p(a0), _p(T), _p(Cf))
    if rc < 0:
        raise RuntimeError(f"or_minsnap_track failed {rc}")
    return T, Cf


def minsnap_batch(tracks, v_max, a_max, threads=1):
    """or_minsnap_batch_mt: every track (v0 = a0 = 0) solved by or_minsnap_track on
    `threads` threads.  Returns (times list, coeff list, status array) like
    eppamd.capi.minsnap_batch."""
    wp = np.ascontiguousarray(np.concatenate([np.asarray(t, np.float64).reshape(-1, 3) for t in tracks]))
    off = np.zeros(len(tracks) + 1, np.int32)
    off[1:] = np.cumsum([len(t) for t in tracks])
    nseg = int(off[-1]) - len(tracks)
    T = np.zeros(max(nseg, 1))
    Cf = np.zeros((max(nseg, 1), 3, 10))
    st = np.zeros(len(tracks), np.int32)
    lib().or_minsnap_batch_mt(_p(wp), _p(off), len(tracks), v_max, a_max, _p(T), _p(Cf), _p(st), int(threads))
    Ts, Cs = [], []
    for k in range(len(tracks)):
        a, b = off[k] - k, off[k + 1] - k - 1
        Ts.append(T[a:b])
        Cs.append(Cf[a:b])
    return Ts, Cs, st


def sample_traj(T, coeffs, dt, t0=0.0):
    T = np.ascontiguousarray(T, np.float64)
    coeffs = np.ascontiguousarray(coeffs, np.float64)
    n = lib().or_sample_traj(_p(T), _p(coeffs), len(T), dt, t0, None, 0)
    rows = np.zeros((max(n, 1), 10))
    lib().or_sample_traj(_p(T), _p(coeffs), len(T), dt, t0, _p(rows), n)
    return rows[:n]


def generate_trajectory(wp, v_max, a_max, dt, t0=0.0, v0=(0, 0, 0), a0=(0, 0, 0)):
    T, Cf = minsnap_track(wp, v_max, a_max, v0, a0)
    return sample_traj(T, Cf, dt, t0)


def mapping_matrix(t):
    A = np.zeros((10, 10))
    lib().or_mapping_matrix(t, _p(A))
    return A


def invert_mapping(A):
    A = np.ascontiguousarray(A, np.float64)
    Ai = np.zeros((10, 10))
    lib().or_invert_mapping(_p(A), _p(Ai))
    return Ai


def poly_eval(c, t, k):
    c = np.ascontiguousarray(c, np.float64)
    return lib().or_poly_eval(_p(c), t, k)


def random_vertices(n_segments, dim, pos_min, pos_max, seed):
    out = np.zeros((n_segments + 1, dim))
    lib().or_random_vertices(n_segments, dim, pos_min, pos_max, seed, _p(out))
    return out


def plan_once(w, r_gate, r_obst, lo, hi, start, goal, samples, seed, k=16, can_pass_gate=False, threads=1):
    """CPU restatement of PathPlanner::planOnce (this build's batch planner): the path as an
    (L, 3) array, or None; plus (samples, valid samples, edges, valid edges, 1 if the
    symmetrised search ran)."""
    lo, hi = np.ascontiguousarray(lo, np.float64), np.ascontiguousarray(hi, np.float64)
    start, goal = np.ascontiguousarray(start, np.float64), np.ascontiguousarray(goal, np.float64)
    cap = 4096
    path = np.zeros((cap, 3))
    stats = np.zeros(5, np.int64)
    n = lib().or_plan_once(_p(w), len(w), r_gate, r_obst, _p(lo), _p(hi), _p(start), _p(goal), int(samples),
                           int(seed) & 0xFFFFFFFFFFFFFFFF, int(k), int(bool(can_pass_gate)), int(threads), _p(path),
                           cap, _p(stats))
    if n < 0:
        raise ValueError("or_plan_once: path buffer too small")
    return (path[:n].copy() if n > 0 else None), stats
