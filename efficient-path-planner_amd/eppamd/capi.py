"""ctypes binding of the C ABI in include/epp.h (libepp.so, built in-tree).

This is the product path: every call goes to the HIP kernels in libepp.so.  There is
no CPU fallback — if the library or a GPU is missing the calls raise.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# EPP_LIB: another build of the same ABI (diagnostics A/B builds under scripts/dbg/)
LIB_PATH = os.environ.get("EPP_LIB") or os.path.join(os.path.dirname(_HERE), "libepp.so")

OBB_DTYPE = np.dtype([("center", "<f8", 3), ("half", "<f8", 3), ("rot", "<f8", 9),
                      ("filling", "<i4"), ("is_gate", "<i4")])

EPP_OK = 0
EPP_ERR_INVALID_ARGUMENT = -1
EPP_ERR_RUNTIME = -2
EPP_ERR_HIP = -3
EPP_ERR_UNSUPPORTED = -4
EPP_ERR_CAPACITY = -5
EPP_ERR_PEER = -6
EPP_ERR_TIMEOUT = -7
EPP_REDUCE_SUM, EPP_REDUCE_MAX, EPP_REDUCE_MIN = 0, 1, 2

_lib = None


class EppError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"epp error {code}: {msg}")
        self.code = code


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} not built: run __graft_entry__.build()")
        l = C.CDLL(LIB_PATH)
        vp, i32, i64, u64, dp = C.c_void_p, C.c_int32, C.c_int64, C.c_uint64, C.c_double
        sig = {
            "epp_last_error": (C.c_char_p, []),
            "epp_version": (C.c_char_p, []),
            "epp_device_count": (i32, [C.POINTER(C.c_int)]),
            "epp_set_device": (i32, [C.c_int]),
            "epp_malloc": (i32, [C.POINTER(vp), u64]),
            "epp_free": (i32, [vp]),
            "epp_memcpy_h2d": (i32, [vp, vp, u64, vp]),
            "epp_memcpy_d2h": (i32, [vp, vp, u64, vp]),
            "epp_memcpy_h2d_async": (i32, [vp, vp, u64, vp]),
            "epp_memcpy_d2h_async": (i32, [vp, vp, u64, vp]),
            "epp_memset": (i32, [vp, C.c_int, u64, vp]),
            "epp_stream_create": (i32, [C.POINTER(vp)]),
            "epp_stream_destroy": (i32, [vp]),
            "epp_stream_sync": (i32, [vp]),
            "epp_device_sync": (i32, []),
            "epp_event_create": (i32, [C.POINTER(vp)]),
            "epp_event_destroy": (i32, [vp]),
            "epp_event_record": (i32, [vp, vp]),
            "epp_event_elapsed_ms": (i32, [vp, vp, C.POINTER(C.c_float)]),
            "epp_graph_begin": (i32, [vp]),
            "epp_graph_end": (i32, [vp, C.POINTER(vp)]),
            "epp_graph_launch": (i32, [vp, vp]),
            "epp_graph_destroy": (i32, [vp]),
            "epp_build_obbs": (i32, [vp, vp, i32, vp, i32, vp, i32, vp, i32, vp, i32, C.POINTER(i32)]),
            "epp_world_create": (i32, [vp, i32, dp, dp, C.POINTER(vp)]),
            "epp_world_update": (i32, [vp, vp, i32]),
            "epp_world_destroy": (i32, [vp]),
            "epp_world_num_obbs": (i32, [vp, C.POINTER(i32)]),
            "epp_world_get_aabbs": (i32, [vp, vp]),
            "epp_world_generation": (i32, [vp, C.POINTER(C.c_uint64)]),
            "epp_world_build_index": (i32, [vp]),
            "epp_comm_unique_id": (i32, [vp]),
            "epp_comm_init": (i32, [vp, i32, i32, C.POINTER(vp)]),
            "epp_comm_init_all": (i32, [i32, vp, vp]),
            "epp_comm_destroy": (i32, [vp]),
            "epp_comm_rank": (i32, [vp, C.POINTER(i32), C.POINTER(i32)]),
            "epp_comm_allgather_waypoints": (i32, [vp, vp, i32, i32, vp, vp]),
            "epp_comm_allreduce_f64": (i32, [vp, vp, i32, i32]),
            "epp_comm_barrier": (i32, [vp]),
            "epp_comm_set_timeout": (i32, [vp, dp]),
            "epp_comm_abort": (i32, [vp]),
            "epp_comm_available": (i32, []),
            "epp_check_states": (i32, [vp, vp, i64, i32, vp, vp, vp, vp]),
            "epp_check_states_mindist": (i32, [vp, vp, i64, dp, vp, vp]),
            "epp_check_motions": (i32, [vp, vp, vp, i64, i32, i32, vp, vp]),
            "epp_minsnap_batch": (i32, [vp, vp, i32, dp, dp, vp, vp, vp, vp, vp, vp]),
            "epp_minsnap_batch_times": (i32, [vp, vp, i32, vp, vp, vp, vp, vp, vp]),
            "epp_sample_count": (i32, [vp, vp, i32, dp, vp, vp]),
            "epp_sample_batch": (i32, [vp, vp, vp, i32, dp, vp, vp, vp, vp]),
            "epp_check_and_generate_trajectory_host": (i32, [vp, vp, i64, dp, vp, vp, i32, dp, dp, dp, dp, vp, vp,
                                                               C.POINTER(C.POINTER(C.c_double)), C.POINTER(i64)]),
            "epp_generate_trajectory_host": (i32, [vp, i32, dp, dp, dp, dp, vp, vp,
                                                   C.POINTER(C.POINTER(C.c_double)), C.POINTER(i64)]),
            "epp_generate_trajectory_times_host": (i32, [vp, i32, vp, dp, dp, vp, vp,
                                                         C.POINTER(C.POINTER(C.c_double)), C.POINTER(i64)]),
            "epp_optimal_trajectory_host": (i32, [vp, i32, vp, i32, dp, dp, dp, dp, dp,
                                                  C.POINTER(C.POINTER(C.c_double)), C.POINTER(i64)]),
            "epp_spline_trajectory_host": (i32, [vp, i32, dp, dp, dp, C.POINTER(C.POINTER(C.c_double)),
                                                 C.POINTER(i64)]),
            "epp_host_free": (None, [vp]),
            "epp_sample_uniform": (i32, [C.c_uint64, vp, vp, i64, i64, vp, vp]),
            "epp_knn": (i32, [vp, i32, i32, dp, vp, vp]),
            "epp_knn_bruteforce": (i32, [vp, i32, i32, dp, vp, vp]),
            "epp_knn_grid": (i32, [vp, i32, i32, dp, vp, vp]),
            "epp_knn_workspace_size": (C.c_uint64, [i32]),
            "epp_knn_ws": (i32, [vp, i32, i32, dp, vp, vp, C.c_uint64, vp]),
            "epp_knn_grid_ws": (i32, [vp, i32, i32, dp, vp, vp, C.c_uint64, vp]),
            "epp_knn_ws_box": (i32, [vp, i32, i32, dp, vp, vp, vp, vp, C.c_uint64, vp]),
            "epp_knn_grid_ws_box": (i32, [vp, i32, i32, dp, vp, vp, vp, vp, C.c_uint64, vp]),
            "epp_knn_edges": (i32, [vp, vp, i32, i32, vp, vp, vp]),
            "epp_compact_states": (i32, [vp, vp, i64, vp, vp, vp]),
            "epp_compact_workspace_size": (C.c_uint64, [i64]),
            "epp_compact_states_ws": (i32, [vp, vp, i64, vp, vp, vp, C.c_uint64, vp]),
            "epp_mask_edges": (i32, [vp, vp, i64, vp]),
            "epp_mask_edges_count": (i32, [vp, vp, i64, i32, vp, vp]),
            "epp_check_knn_motions": (i32, [vp, vp, vp, i32, i32, i32, i32, vp, vp]),
        }
        for name, (res, args) in sig.items():
            if os.environ.get("EPP_LIB") and not hasattr(l, name):
                continue  # (an A/B build from before the symbol existed)
            f = getattr(l, name)
            f.restype = res
            f.argtypes = args
        _lib = l
    return _lib


# every symbol include/epp.h declares (the CPU test checks the library exports them)
EXPORTED = [
    "epp_last_error", "epp_version", "epp_device_count", "epp_set_device", "epp_malloc", "epp_free",
    "epp_memcpy_h2d", "epp_memcpy_d2h", "epp_memcpy_h2d_async", "epp_memcpy_d2h_async", "epp_memset", "epp_stream_create", "epp_stream_destroy",
    "epp_stream_sync", "epp_device_sync", "epp_event_create", "epp_event_destroy", "epp_event_record",
    "epp_event_elapsed_ms", "epp_build_obbs", "epp_world_create", "epp_world_update",
    "epp_world_destroy", "epp_world_num_obbs", "epp_world_get_aabbs", "epp_check_states",
    "epp_check_states_mindist", "epp_check_motions", "epp_minsnap_batch", "epp_sample_count",
    "epp_sample_batch", "epp_generate_trajectory_host", "epp_host_free", "epp_sample_uniform", "epp_knn",
    "epp_knn_bruteforce", "epp_knn_grid", "epp_knn_workspace_size", "epp_knn_ws", "epp_knn_grid_ws",
    "epp_knn_edges", "epp_compact_states", "epp_mask_edges", "epp_mask_edges_count", "epp_check_knn_motions", "epp_optimal_trajectory_host",
    "epp_spline_trajectory_host", "epp_compact_workspace_size", "epp_compact_states_ws",
    "epp_graph_begin", "epp_graph_end", "epp_graph_launch", "epp_graph_destroy", "epp_minsnap_batch_times",
    "epp_generate_trajectory_times_host", "epp_world_generation", "epp_world_build_index", "epp_comm_unique_id", "epp_comm_init",
    "epp_comm_init_all", "epp_comm_destroy", "epp_comm_rank", "epp_comm_allgather_waypoints",
    "epp_comm_allreduce_f64", "epp_comm_barrier", "epp_comm_available", "epp_knn_ws_box", "epp_knn_grid_ws_box",
    "epp_comm_set_timeout", "epp_comm_abort", "epp_check_and_generate_trajectory_host",
]


def check(rc: int) -> None:
    if rc != EPP_OK:
        raise EppError(rc, lib().epp_last_error().decode())


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


class DeviceBuffer:
    """A raw HBM allocation (epp_malloc)."""

    def __init__(self, nbytes: int):
        p = C.c_void_p()
        check(lib().epp_malloc(C.byref(p), max(int(nbytes), 16)))
        self.ptr = p.value
        self.nbytes = int(nbytes)

    @classmethod
    def from_array(cls, a: np.ndarray, stream=None) -> "DeviceBuffer":
        a = np.ascontiguousarray(a)
        b = cls(a.nbytes)
        b.upload(a, stream)
        return b

    def upload(self, a: np.ndarray, stream=None) -> None:
        a = np.ascontiguousarray(a)
        assert a.nbytes <= self.nbytes
        check(lib().epp_memcpy_h2d(self.ptr, _ptr(a), a.nbytes, stream))

    def download(self, dtype, count: int, stream=None) -> np.ndarray:
        out = np.empty(count, dtype=dtype)
        assert out.nbytes <= self.nbytes
        check(lib().epp_memcpy_d2h(_ptr(out), self.ptr, out.nbytes, stream))
        return out

    def zero(self, stream=None) -> None:
        check(lib().epp_memset(self.ptr, 0, self.nbytes, stream))

    def free(self) -> None:
        if self.ptr:
            lib().epp_free(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def device_count() -> int:
    n = C.c_int(0)
    check(lib().epp_device_count(C.byref(n)))
    return n.value


def sync() -> None:
    check(lib().epp_device_sync())


def build_obbs(geom, gates: np.ndarray, obstacles: np.ndarray) -> np.ndarray:
    """World::addGate / addObstacle (src/World.cpp:13-55) on the host."""
    gates = np.ascontiguousarray(np.asarray(gates, np.float64).reshape(-1, 7))
    obstacles = np.ascontiguousarray(np.asarray(obstacles, np.float64).reshape(-1, 6))
    cap = len(gates) * max(1, len(geom.gate_desc)) + len(obstacles) * max(1, len(geom.obst_desc))
    out = np.zeros(max(cap, 1), OBB_DTYPE)
    n = C.c_int32(0)
    check(lib().epp_build_obbs(_ptr(geom.gate_desc), _ptr(geom.gate_desc_off), len(geom.gate_desc_off) - 1,
                               _ptr(geom.obst_desc), len(geom.obst_desc), _ptr(gates), len(gates),
                               _ptr(obstacles), len(obstacles), _ptr(out), len(out), C.byref(n)))
    return out[: n.value].copy()


class World:
    """Device-resident OBB table + cull grid (epp_world)."""

    def __init__(self, obbs: np.ndarray, r_gate: float, r_obst: float):
        obbs = np.ascontiguousarray(obbs, dtype=OBB_DTYPE)
        h = C.c_void_p()
        check(lib().epp_world_create(_ptr(obbs) if len(obbs) else None, len(obbs), r_gate, r_obst, C.byref(h)))
        self.handle = h.value
        self.n = len(obbs)

    def update(self, obbs: np.ndarray) -> None:
        obbs = np.ascontiguousarray(obbs, dtype=OBB_DTYPE)
        check(lib().epp_world_update(self.handle, _ptr(obbs) if len(obbs) else None, len(obbs)))
        self.n = len(obbs)

    def build_index(self) -> None:
        """Rebuild + upload a stale device index now (epp_world_build_index)."""
        check(lib().epp_world_build_index(self.handle))

    def generation(self) -> int:
        g = C.c_uint64(0)
        check(lib().epp_world_generation(self.handle, C.byref(g)))
        return g.value

    def aabbs(self) -> np.ndarray:
        out = np.zeros((max(self.n, 1), 6))
        check(lib().epp_world_get_aabbs(self.handle, _ptr(out)))
        return out[: self.n]

    def close(self) -> None:
        if self.handle:
            lib().epp_world_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- device-pointer calls ----------------------------------------------------
    def check_states_dev(self, xyz_ptr, n, can_pass_gate, valid_ptr, compact_ptr=None, nvalid_ptr=None,
                         stream=None):
        check(lib().epp_check_states(self.handle, xyz_ptr, n, int(can_pass_gate), valid_ptr, compact_ptr,
                                     nvalid_ptr, stream))

    def check_motions_dev(self, s1_ptr, s2_ptr, n, can_pass_gate, mode, valid_ptr, stream=None):
        check(lib().epp_check_motions(self.handle, s1_ptr, s2_ptr, n, int(can_pass_gate), int(mode),
                                      valid_ptr, stream))

    # ---- host-array convenience (copies in/out) ----------------------------------
    def check_states(self, xyz: np.ndarray, can_pass_gate: bool = False, compact: bool = False):
        xyz = np.ascontiguousarray(xyz, np.float64).reshape(-1, 3)
        n = len(xyz)
        d_xyz = DeviceBuffer.from_array(xyz)
        d_valid = DeviceBuffer(n)
        if compact:
            d_idx = DeviceBuffer(4 * max(n, 1))
            d_cnt = DeviceBuffer(8)
            d_cnt.zero()
            self.check_states_dev(d_xyz.ptr, n, can_pass_gate, d_valid.ptr, d_idx.ptr, d_cnt.ptr)
            sync()
            cnt = int(d_cnt.download(np.int64, 1)[0])
            return d_valid.download(np.uint8, n), d_idx.download(np.int32, cnt)
        self.check_states_dev(d_xyz.ptr, n, can_pass_gate, d_valid.ptr)
        sync()
        return d_valid.download(np.uint8, n)

    def check_states_mindist(self, xyz: np.ndarray, min_distance: float) -> np.ndarray:
        xyz = np.ascontiguousarray(xyz, np.float64).reshape(-1, 3)
        n = len(xyz)
        d_xyz = DeviceBuffer.from_array(xyz)
        d_valid = DeviceBuffer(n)
        check(lib().epp_check_states_mindist(self.handle, d_xyz.ptr, n, float(min_distance), d_valid.ptr, None))
        sync()
        return d_valid.download(np.uint8, n)

    def check_motions(self, s1: np.ndarray, s2: np.ndarray, can_pass_gate: bool = False, mode: int = 0):
        s1 = np.ascontiguousarray(s1, np.float64).reshape(-1, 3)
        s2 = np.ascontiguousarray(s2, np.float64).reshape(-1, 3)
        n = len(s1)
        d1, d2 = DeviceBuffer.from_array(s1), DeviceBuffer.from_array(s2)
        d_valid = DeviceBuffer(n)
        self.check_motions_dev(d1.ptr, d2.ptr, n, can_pass_gate, mode, d_valid.ptr)
        sync()
        return d_valid.download(np.uint8, n)


def minsnap_batch(tracks, v_max, a_max, v0=None, a0=None):
    """epp_minsnap_batch on a list of (W_k x 3) waypoint arrays.

    Returns (seg_times list, coeffs list [M_k x 3 x 10], status array)."""
    wp = np.ascontiguousarray(np.concatenate([np.asarray(t, np.float64).reshape(-1, 3) for t in tracks]))
    off = np.zeros(len(tracks) + 1, np.int32)
    off[1:] = np.cumsum([len(t) for t in tracks])
    nt = len(tracks)
    nseg = int(off[-1]) - nt
    d_wp, d_off = DeviceBuffer.from_array(wp), DeviceBuffer.from_array(off)
    d_v0 = DeviceBuffer.from_array(np.ascontiguousarray(v0, np.float64)) if v0 is not None else None
    d_a0 = DeviceBuffer.from_array(np.ascontiguousarray(a0, np.float64)) if a0 is not None else None
    d_T, d_C, d_st = DeviceBuffer(8 * max(nseg, 1)), DeviceBuffer(240 * max(nseg, 1)), DeviceBuffer(4 * nt)
    check(lib().epp_minsnap_batch(d_wp.ptr, d_off.ptr, nt, float(v_max), float(a_max),
                                  d_v0.ptr if d_v0 else None, d_a0.ptr if d_a0 else None,
                                  d_T.ptr, d_C.ptr, d_st.ptr, None))
    sync()
    T = d_T.download(np.float64, nseg)
    Cf = d_C.download(np.float64, nseg * 30).reshape(nseg, 3, 10)
    st = d_st.download(np.int32, nt)
    Ts, Cs = [], []
    for k in range(nt):
        a, b = int(off[k]) - k, int(off[k + 1]) - k - 1
        Ts.append(T[a:max(a, b)])
        Cs.append(Cf[a:max(a, b)])
    return Ts, Cs, st


def minsnap_batch_times(tracks, times, v0=None, a0=None):
    """epp_minsnap_batch_times: as minsnap_batch with the caller's segment times (a list
    of (W_k - 1) arrays; setupFromVertices(vertices, segment_times)).  Returns (coeffs
    list, status array)."""
    wp = np.ascontiguousarray(np.concatenate([np.asarray(t, np.float64).reshape(-1, 3) for t in tracks]))
    off = np.zeros(len(tracks) + 1, np.int32)
    off[1:] = np.cumsum([len(t) for t in tracks])
    nt = len(tracks)
    nseg = int(off[-1]) - nt
    T = np.ascontiguousarray(np.concatenate([np.asarray(t, np.float64).ravel() for t in times]))
    assert len(T) == nseg
    d_wp, d_off, d_T = DeviceBuffer.from_array(wp), DeviceBuffer.from_array(off), DeviceBuffer.from_array(T)
    d_v0 = DeviceBuffer.from_array(np.ascontiguousarray(v0, np.float64)) if v0 is not None else None
    d_a0 = DeviceBuffer.from_array(np.ascontiguousarray(a0, np.float64)) if a0 is not None else None
    d_C, d_st = DeviceBuffer(240 * max(nseg, 1)), DeviceBuffer(4 * nt)
    check(lib().epp_minsnap_batch_times(d_wp.ptr, d_off.ptr, nt, d_v0.ptr if d_v0 else None,
                                        d_a0.ptr if d_a0 else None, d_T.ptr, d_C.ptr, d_st.ptr, None))
    sync()
    Cf = d_C.download(np.float64, nseg * 30).reshape(nseg, 3, 10)
    st = d_st.download(np.int32, nt)
    return [Cf[int(off[k]) - k:int(off[k + 1]) - k - 1] for k in range(nt)], st


def generate_trajectory_times(waypoints, seg_times, dt, t0=0.0, v0=(0, 0, 0), a0=(0, 0, 0)) -> np.ndarray:
    """generateTrajectory with the caller's segment times (epp_generate_trajectory_times_host)."""
    wp = np.ascontiguousarray(np.asarray(waypoints, np.float64).reshape(-1, 3))
    T = np.ascontiguousarray(seg_times, np.float64)
    v0 = np.ascontiguousarray(v0, np.float64)
    a0 = np.ascontiguousarray(a0, np.float64)
    rows = C.POINTER(C.c_double)()
    n = C.c_int64(0)
    check(lib().epp_generate_trajectory_times_host(_ptr(wp), len(wp), _ptr(T), float(dt), float(t0), _ptr(v0),
                                                   _ptr(a0), C.byref(rows), C.byref(n)))
    if n.value == 0:
        lib().epp_host_free(C.cast(rows, C.c_void_p))
        return np.zeros((0, 10))
    out = np.ctypeslib.as_array(rows, shape=(n.value * 10,)).copy().reshape(-1, 10)
    lib().epp_host_free(C.cast(rows, C.c_void_p))
    return out


def generate_trajectory(waypoints, v_max, a_max, dt, t0=0.0, v0=(0, 0, 0), a0=(0, 0, 0)) -> np.ndarray:
    """poly_traj::generateTrajectory (src/trajectory_generator.cpp:12-100) on the GPU."""
    wp = np.ascontiguousarray(np.asarray(waypoints, np.float64).reshape(-1, 3))
    v0 = np.ascontiguousarray(v0, np.float64)
    a0 = np.ascontiguousarray(a0, np.float64)
    rows = C.POINTER(C.c_double)()
    n = C.c_int64(0)
    check(lib().epp_generate_trajectory_host(_ptr(wp), len(wp), float(v_max), float(a_max), float(dt), float(t0),
                                             _ptr(v0), _ptr(a0), C.byref(rows), C.byref(n)))
    if n.value == 0:
        lib().epp_host_free(C.cast(rows, C.c_void_p))
        return np.zeros((0, 10))
    out = np.ctypeslib.as_array(rows, shape=(n.value * 10,)).copy().reshape(-1, 10)
    lib().epp_host_free(C.cast(rows, C.c_void_p))
    return out


def check_and_generate_trajectory(world: "World", check_xyz, min_distance, waypoints, v_max, a_max, dt, t0=0.0,
                                  v0=(0, 0, 0), a0=(0, 0, 0)):
    """epp_check_and_generate_trajectory_host: (minDistance flags of check_xyz against the
    world, the trajectory rows of generate_trajectory) from one launch."""
    pts = np.ascontiguousarray(np.asarray(check_xyz, np.float64).reshape(-1, 3))
    wp = np.ascontiguousarray(np.asarray(waypoints, np.float64).reshape(-1, 3))
    v0 = np.ascontiguousarray(v0, np.float64)
    a0 = np.ascontiguousarray(a0, np.float64)
    flags = np.zeros(max(len(pts), 1), np.uint8)
    rows = C.POINTER(C.c_double)()
    n = C.c_int64(0)
    check(lib().epp_check_and_generate_trajectory_host(world.handle, _ptr(pts), len(pts), float(min_distance),
                                                       _ptr(flags), _ptr(wp), len(wp), float(v_max), float(a_max),
                                                       float(dt), float(t0), _ptr(v0), _ptr(a0), C.byref(rows),
                                                       C.byref(n)))
    out = np.ctypeslib.as_array(rows, shape=(n.value * 10,)).copy().reshape(-1, 10) if n.value else np.zeros((0, 10))
    lib().epp_host_free(C.cast(rows, C.c_void_p))
    return flags[:len(pts)], out


def optimal_trajectory(waypoints, v_max, a_max, dt, t0=0.0, max_deviation=0.1, pre_waypoints=()) -> np.ndarray:
    """OptimalTimeParametrizer::calculateTrajectory (the "optimal" type; host code,
    external/time_parametrization/src/OptimalTimeParametrizer.cpp:11-108): rows x 11."""
    wp = np.ascontiguousarray(np.asarray(waypoints, np.float64).reshape(-1, 3))
    pre = np.ascontiguousarray(np.asarray(pre_waypoints, np.float64).reshape(-1, 3))
    rows = C.POINTER(C.c_double)()
    n = C.c_int64(0)
    check(lib().epp_optimal_trajectory_host(_ptr(wp), len(wp), _ptr(pre) if len(pre) else None, len(pre),
                                            float(v_max), float(a_max), float(dt), float(t0), float(max_deviation),
                                            C.byref(rows), C.byref(n)))
    if n.value == 0:
        lib().epp_host_free(C.cast(rows, C.c_void_p))
        return np.zeros((0, 11))
    out = np.ctypeslib.as_array(rows, shape=(n.value * 11,)).copy().reshape(-1, 11)
    lib().epp_host_free(C.cast(rows, C.c_void_p))
    return out


def spline_trajectory(waypoints, max_t, dt, t0=0.0) -> np.ndarray:
    """TrajInterpolation::interpolateTraj (the "spline" type; host code,
    src/TrajInterpolation.cpp:44-68): rows x 10."""
    wp = np.ascontiguousarray(np.asarray(waypoints, np.float64).reshape(-1, 3))
    rows = C.POINTER(C.c_double)()
    n = C.c_int64(0)
    check(lib().epp_spline_trajectory_host(_ptr(wp), len(wp), float(max_t), float(t0), float(dt),
                                           C.byref(rows), C.byref(n)))
    out = np.ctypeslib.as_array(rows, shape=(n.value * 10,)).copy().reshape(-1, 10) if n.value else np.zeros((0, 10))
    lib().epp_host_free(C.cast(rows, C.c_void_p))
    return out


def sample_uniform(seed: int, lo, hi, n: int, start: int = 0) -> np.ndarray:
    """epp_sample_uniform: n counter-based uniform states (rows start..start+n-1)."""
    lo = np.ascontiguousarray(lo, np.float64)
    hi = np.ascontiguousarray(hi, np.float64)
    d = DeviceBuffer(24 * max(n, 1))
    check(lib().epp_sample_uniform(int(seed) & 0xFFFFFFFFFFFFFFFF, _ptr(lo), _ptr(hi), int(n), int(start), d.ptr, None))
    sync()
    return d.download(np.float64, 3 * n).reshape(n, 3)


def _filled(nbytes: int, word) -> DeviceBuffer:
    """A device buffer of nbytes (multiple of 8) holding `word` (u64) in every slot, or
    zeros when word is None -- a caller workspace that held other data."""
    b = DeviceBuffer(nbytes)
    if word is None:
        b.zero()
    else:
        b.upload(np.full(nbytes // 8, int(word) & 0xFFFFFFFFFFFFFFFF, np.uint64))
    return b


def knn(nodes: np.ndarray, k: int, max_dist: float = 0.0, method: str = "auto", box=None,
        ws_fill=None) -> np.ndarray:
    """epp_knn (method "auto"), epp_knn_bruteforce ("brute") or epp_knn_grid ("grid"):
    (n, k) neighbour indices, nearest first, ties to the lower index, -1 where fewer
    than k exist.  box=(lo, hi) with method "ws" / "grid_ws": the caller-box variants
    (epp_knn_ws_box / epp_knn_grid_ws_box; every node inside the box).  ws_fill: the u64
    word the caller workspace holds before the call (tests: stale data)."""
    nodes = np.ascontiguousarray(np.asarray(nodes, np.float64).reshape(-1, 3))
    n = len(nodes)
    d_n = DeviceBuffer.from_array(nodes)
    d_k = DeviceBuffer(4 * max(n * k, 1))
    if method in ("ws", "grid_ws"):  # caller workspace variants
        d_w = _filled(max(int(lib().epp_knn_workspace_size(n)), 256), ws_fill)
        if box is not None:
            lo, hi = (np.ascontiguousarray(np.asarray(b, np.float64).reshape(3)) for b in box)
            fn = lib().epp_knn_ws_box if method == "ws" else lib().epp_knn_grid_ws_box
            check(fn(d_n.ptr, n, int(k), float(max_dist), _ptr(lo), _ptr(hi), d_k.ptr, d_w.ptr, d_w.nbytes, None))
        else:
            fn = lib().epp_knn_ws if method == "ws" else lib().epp_knn_grid_ws
            check(fn(d_n.ptr, n, int(k), float(max_dist), d_k.ptr, d_w.ptr, d_w.nbytes, None))
    else:
        fn = {"auto": lib().epp_knn, "brute": lib().epp_knn_bruteforce, "grid": lib().epp_knn_grid}[method]
        check(fn(d_n.ptr, n, int(k), float(max_dist), d_k.ptr, None))
    sync()
    return d_k.download(np.int32, n * k).reshape(n, k)


def compact_states(xyz: np.ndarray, valid: np.ndarray, ws: bool = False, ws_fill=None) -> np.ndarray:
    """epp_compact_states (ws: epp_compact_states_ws, caller workspace): the valid rows of
    xyz, in index order.  ws_fill: the u64 word the caller workspace holds before the call."""
    xyz = np.ascontiguousarray(np.asarray(xyz, np.float64).reshape(-1, 3))
    valid = np.ascontiguousarray(np.asarray(valid, np.uint8))
    n = len(xyz)
    d_x, d_v = DeviceBuffer.from_array(xyz), DeviceBuffer.from_array(valid)
    d_o, d_c = DeviceBuffer(24 * max(n, 1)), DeviceBuffer(8)
    if ws:
        d_w = _filled(int(lib().epp_compact_workspace_size(n)), ws_fill)
        check(lib().epp_compact_states_ws(d_x.ptr, d_v.ptr, n, d_o.ptr, d_c.ptr, d_w.ptr, d_w.nbytes, None))
    else:
        check(lib().epp_compact_states(d_x.ptr, d_v.ptr, n, d_o.ptr, d_c.ptr, None))
    sync()
    cnt = int(d_c.download(np.int64, 1)[0])
    return d_o.download(np.float64, 3 * cnt).reshape(cnt, 3) if cnt else np.zeros((0, 3))


def mask_edges(nbr: np.ndarray, valid: np.ndarray) -> np.ndarray:
    """epp_mask_edges: nbr with -1 where valid == 0."""
    nbr = np.ascontiguousarray(np.asarray(nbr, np.int32))
    valid = np.ascontiguousarray(np.asarray(valid, np.uint8).reshape(nbr.shape))
    d_n, d_v = DeviceBuffer.from_array(nbr), DeviceBuffer.from_array(valid)
    check(lib().epp_mask_edges(d_n.ptr, d_v.ptr, nbr.size, None))
    sync()
    return d_n.download(np.int32, nbr.size).reshape(nbr.shape)


def mask_edges_count(nbr: np.ndarray, valid: np.ndarray, target: int = 1):
    """epp_mask_edges_count: (nbr with -1 where valid == 0, entries >= 0 afterwards,
    entries == target afterwards)."""
    nbr = np.ascontiguousarray(np.asarray(nbr, np.int32))
    valid = np.ascontiguousarray(np.asarray(valid, np.uint8).reshape(nbr.shape))
    d_n, d_v, d_c = DeviceBuffer.from_array(nbr), DeviceBuffer.from_array(valid), DeviceBuffer(16)
    check(lib().epp_mask_edges_count(d_n.ptr, d_v.ptr, nbr.size, target, d_c.ptr, None))
    sync()
    c = d_c.download(np.int64, 2)
    return d_n.download(np.int32, nbr.size).reshape(nbr.shape), int(c[0]), int(c[1])


def knn_edges(nodes: np.ndarray, nbr: np.ndarray):
    """epp_knn_edges: the (node, neighbour) endpoint arrays of every k-NN edge."""
    nodes = np.ascontiguousarray(np.asarray(nodes, np.float64).reshape(-1, 3))
    nbr = np.ascontiguousarray(nbr, np.int32)
    n, k = nbr.shape
    d_n, d_k = DeviceBuffer.from_array(nodes), DeviceBuffer.from_array(nbr)
    d_1, d_2 = DeviceBuffer(24 * max(n * k, 1)), DeviceBuffer(24 * max(n * k, 1))
    check(lib().epp_knn_edges(d_n.ptr, d_k.ptr, n, k, d_1.ptr, d_2.ptr, None))
    sync()
    return d_1.download(np.float64, 3 * n * k).reshape(-1, 3), d_2.download(np.float64, 3 * n * k).reshape(-1, 3)


class Comm:
    """RCCL communicator of the multi-track plan's exchange step (epp_comm_*).

    One process per GPU: Comm(unique_id, n_ranks, rank) on the rank's device, with the
    id from Comm.unique_id() on rank 0 shared out of band."""

    def __init__(self, uid: bytes, n_ranks: int, rank: int, handle=None):
        if handle is not None:
            self.handle = handle
        else:
            assert len(uid) == 128
            buf = (C.c_uint8 * 128).from_buffer_copy(uid)
            h = C.c_void_p()
            check(lib().epp_comm_init(C.cast(buf, C.c_void_p), n_ranks, rank, C.byref(h)))
            self.handle = h.value
        r, n = C.c_int32(), C.c_int32()
        check(lib().epp_comm_rank(self.handle, C.byref(r), C.byref(n)))
        self.rank, self.n_ranks = r.value, n.value

    @staticmethod
    def unique_id() -> bytes:
        buf = (C.c_uint8 * 128)()
        check(lib().epp_comm_unique_id(C.cast(buf, C.c_void_p)))
        return bytes(buf)

    @classmethod
    def init_all(cls, devices) -> list["Comm"]:
        devs = np.ascontiguousarray(devices, np.int32)
        hs = (C.c_void_p * len(devs))()
        check(lib().epp_comm_init_all(len(devs), _ptr(devs), C.cast(hs, C.c_void_p)))
        return [cls(b"", 0, 0, handle=h) for h in hs]

    def allgather_waypoints(self, wp: np.ndarray | None, cap: int = 4096) -> list[np.ndarray]:
        """Every rank's (W_r, 3) set.  wp=None: this rank failed (count -1); every rank then
        raises EppError(EPP_ERR_PEER) with `.counts` naming the failed ranks (-1)."""
        out = np.zeros((self.n_ranks, cap, 3))
        counts = np.zeros(self.n_ranks, np.int32)
        if wp is None:
            rc = lib().epp_comm_allgather_waypoints(self.handle, None, -1, cap, _ptr(out), _ptr(counts))
        else:
            wp = np.ascontiguousarray(np.asarray(wp, np.float64).reshape(-1, 3))
            rc = lib().epp_comm_allgather_waypoints(self.handle, _ptr(wp) if len(wp) else None, len(wp), cap,
                                                    _ptr(out), _ptr(counts))
        if rc != EPP_OK:
            err = EppError(rc, lib().epp_last_error().decode())
            err.counts = counts.copy()
            raise err
        return [out[r, :counts[r]].copy() for r in range(self.n_ranks)]

    def allreduce(self, x, op: int = EPP_REDUCE_SUM) -> np.ndarray:
        """x (doubles) reduced over the ranks (epp_comm_allreduce_f64)."""
        a = np.ascontiguousarray(np.array(x, np.float64).reshape(-1))
        check(lib().epp_comm_allreduce_f64(self.handle, _ptr(a), len(a), op))
        return a

    def barrier(self) -> None:
        check(lib().epp_comm_barrier(self.handle))

    def set_timeout(self, seconds: float) -> None:
        """Deadline of every later collective (epp_comm_set_timeout)."""
        check(lib().epp_comm_set_timeout(self.handle, float(seconds)))

    def abort(self) -> None:
        """Request an abort (epp_comm_abort; any thread): the collective in flight, or the
        next one, aborts the communicator and fails."""
        check(lib().epp_comm_abort(self.handle))

    def close(self) -> None:
        if self.handle:
            lib().epp_comm_destroy(self.handle)
            self.handle = None
