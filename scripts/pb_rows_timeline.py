"""Per-query timeline of k_pb_rows (diagnostics, round 6).  Needs the package built with
-DEPP_PB_ROWS_TL (EXTRA=-DEPP_PB_ROWS_TL bash scripts/ab_pkg.sh WORKTREE pbtl -> ab/pkg_pbtl,
built on the CPU side).  Plans the C4 track (world seed 100) through
OnlineTrajGenerator.pre_compute_traj a few times, then prints, for the last call's
k_pb_rows launch (s_memrealtime, 100 MHz, relative to the first wave's start): when the
waves start, how long one query takes and in which phase (its cells' run starts loaded,
its candidates listed, its row ranked and written), the radius iterations and candidate
counts, and the queries per wave."""
import ctypes as C
import json
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.environ.get("EPP_PKG") or os.path.join(ROOT, "ab", "pkg_pbtl")
sys.path[:0] = [ROOT, PKG]
import online_traj_planner as otp  # noqa: E402
from eppamd import config, synth  # noqa: E402

cfg = config.load(os.path.join(ROOT, "configs", "config.json"))
cfg["world_properties"]["lower_bound"] = [-6, -6, 0]
cfg["world_properties"]["upper_bound"] = [6, 6, 2]
cfg["path_planner_properties"]["samples_fmt"] = 65536
geom = config.geometry(cfg)
fd, path = tempfile.mkstemp(suffix=".json")
with os.fdopen(fd, "w") as f:
    json.dump(cfg, f)
gates, obstacles = synth.track_world(100)
cps = synth.gate_checkpoints(gates, geom.gate_height, 0.55)
otg = otp.OnlineTrajGenerator(cps[0], cps[-1], gates, obstacles, path)
L = C.CDLL(os.path.join(PKG, "libepp.so"))
for r in range(4):
    otg.pre_compute_traj(0.0)
st = otg.planner_stats()
os.unlink(path)
n = int(st["restricted_rows"])
tl = np.zeros((1 << 15) * 6, np.uint64)
assert L.epp_dbg_pb_rows_tl(C.c_void_p(tl.ctypes.data), C.c_int64(1 << 15)) == 0
tl = tl.reshape(-1, 6).astype(np.int64)[:min(n, 1 << 15)]
t0 = tl[:, 5].min()
q0, q1, q2, q3 = tl[:, 0] - t0, tl[:, 1] - t0, tl[:, 2] - t0, tl[:, 3] - t0
it, cnt, wave = tl[:, 4] & 0xFF, (tl[:, 4] >> 8) & 0xFFFFFF, tl[:, 4] >> 32
ws = tl[:, 5] - t0
us = lambda x: x / 100.0  # noqa: E731 (100 MHz ticks -> us)
pct = lambda a: f"p50 {us(np.median(a)):.2f} p90 {us(np.quantile(a, .9)):.2f} max {us(a.max()):.2f} us"  # noqa: E731
print(f"queries (restricted rows) {n}, waves used {len(np.unique(wave))}, queries per wave max "
      f"{np.bincount(wave).max()}")
print("wave start:           ", pct(ws))
print("query start:          ", pct(q0))
print("query end:            ", pct(q3))
print("query duration:       ", pct(q3 - q0))
print("  runs loaded after:  ", pct(q1 - q0))
print("  candidates after:   ", pct(q2 - q1))
print("  ranked+written:     ", pct(q3 - q2))
print(f"radius iterations: {dict(zip(*np.unique(it, return_counts=True)))}; candidates p50 {np.median(cnt):.0f} "
      f"p90 {np.quantile(cnt, .9):.0f} max {cnt.max()}")
order = np.argsort(q3)[::-1][:5]
print("last queries:", [(int(d), round(us(q0[d]), 2), round(us(q3[d]), 2), int(it[d]), int(cnt[d])) for d in order])
