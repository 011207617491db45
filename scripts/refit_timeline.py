"""Phase timeline of the fused single-track refit (k_refit): builds a diagnostics copy of
libepp.so with -DEPP_REFIT_TL into scripts/dbg/ (not the product library), runs 50
refits and prints the median time of every phase boundary (s_memrealtime, 100 MHz)
relative to the kernel's first stamp.  Solver (wg0): 0 entry,
1 times / powers / vertex values, 5 assembly, 6 block solve, 7 coefficients, 8 inputs staged, 13 rows
written; slots 14/15 hold the shader clock (s_memtime) around the block solve."""
import ctypes as C
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "efficient-path-planner_amd")]
from eppamd import synth  # noqa: E402

out = os.path.join(ROOT, "scripts", "tl")  # built here on the CPU side (make below); travels with the tree
os.makedirs(out, exist_ok=True)
pkg = os.path.join(ROOT, "efficient-path-planner_amd")
if not os.path.exists(f"{out}/libepp_tl.so") or "--rebuild" in sys.argv:  # (prebuilt on the CPU side)
    subprocess.run(["make", "-s", "-j16", "-C", pkg, f"BUILD={out}/build", f"LIB={out}/libepp_tl.so",
                    "EXTRA=-DEPP_REFIT_TL", f"{out}/libepp_tl.so"], check=True)
L = C.CDLL(os.path.join(out, "libepp_tl.so"))
wp = np.ascontiguousarray(synth.random_track_waypoints(10_000, 12))
v = np.zeros(3)
rows = C.POINTER(C.c_double)()
n = C.c_int64()
tl = np.zeros(32 + 128, np.uint64)
stamps = []
for r in range(60):
    rc = L.epp_generate_trajectory_host(C.c_void_p(wp.ctypes.data), len(wp), C.c_double(1.0), C.c_double(2.0),
                                        C.c_double(0.1), C.c_double(0.0), C.c_void_p(v.ctypes.data),
                                        C.c_void_p(v.ctypes.data), C.byref(rows), C.byref(n))
    assert rc == 0
    L.epp_host_free(C.cast(rows, C.c_void_p))
    L.epp_dbg_refit_tl(C.c_void_p(tl.ctypes.data))
    stamps.append(tl.astype(np.int64).copy())
allst = np.array(stamps[10:])
it = allst[:, 32:32 + 64]  # wg0's per-iteration shader clocks of the block solve
W = len(wp)
nin = W - 2
nstep = nin - (nin + 1) // 2  # the twisted solve's steps per sweep (slots 1.. forward, 33.. back)
fw = np.diff(it[:, 1:nstep + 1], axis=1)
print("block solve forward, cycles per step (median):", np.median(fw, axis=0).astype(int).tolist())
bw = np.diff(it[:, 32:32 + nstep + 1], axis=1)
print("back substitution, cycles per step (median):", np.median(bw, axis=0).astype(int).tolist())
print("last forward step -> back start (middle solve):", int(np.median(it[:, 32] - it[:, nstep])),
      "cycles; back end -> phase end:", int(np.median(it[:, 63] - it[:, 32 + nstep])), "cycles")
st = allst[:, :32].reshape(-1, 2, 16)
t0 = st[:, :, 0].min(axis=1)
for wg in range(2):
    clk = (st[:, wg, 15] - st[:, wg, 14]) / ((st[:, wg, 6] - st[:, wg, 5]) * 10e-9) / 1e6
    print(f"wg{wg} shader clock during the block solve: median {np.median(clk):.0f} MHz")
    for k in range(14):
        d = (st[:, wg, k] - t0) * 10  # ns
        if (st[:, wg, k] > 0).all():
            print(f"wg{wg} stamp {k:2d}: median {np.median(d) / 1000:7.2f} us")
print("rows", n.value)
