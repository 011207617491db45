"""Phase timeline of k_knn_tile (diagnostics; not the product): builds a diagnostics copy of
libepp.so with -DEPP_KNN_DIAG into scripts/dbg/, runs the planner's k-NN (one C4 segment's
~63k nodes, k = 16) and prints, over the blocks, percentiles of each phase's duration
(thread 0's s_memrealtime stamps, 10 ns): halo sizes + scan, halo copy, first query
round's pass 1 (histogram), pass 2 (list), exact phase, the other rounds, the tail."""
import ctypes as C
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "efficient-path-planner_amd")]
from eppamd import capi, config, synth  # noqa: E402

out = os.path.join(ROOT, "scripts", "dbg")
lib_path = os.path.join(out, "libepp_knndiag.so")
if not os.path.exists(lib_path):
    subprocess.run(["make", "-s", "-j16", "-C", os.path.join(ROOT, "efficient-path-planner_amd"),
                    f"BUILD={out}/build_knn", f"LIB={lib_path}", "EXTRA=-DEPP_KNN_DIAG", lib_path], check=True)
capi.LIB_PATH = lib_path
L = capi.lib()
L.epp_dbg_knn_tl.argtypes = [C.c_void_p, C.c_int64]
cfg = config.load(os.path.join(ROOT, "configs", "config.json"))
geom = config.geometry(cfg)
rg, ro = config.inflate_radii(cfg)
gates, obstacles = synth.track_world(100)
w = capi.World(capi.build_obbs(geom, gates, obstacles), rg, ro)
s = synth.sample_states(1234, *synth.C2_BOUNDS, 65536)
nodes = np.ascontiguousarray(s[w.check_states(s, False).astype(bool)])
n, k = len(nodes), 16
d_n = capi.DeviceBuffer.from_array(nodes)
d_k = capi.DeviceBuffer(4 * n * k)
ws = int(L.epp_knn_workspace_size(n))
d_ws = capi.DeviceBuffer(ws)


def report(recs):
    t = np.concatenate(recs)
    names = ["scan", "copy", "pass1", "pass2", "exact", "rounds", "tail"]
    print(f"blocks per launch {len(recs[0])}, queries per block p50 {np.median(t[:, 8]):.0f} max {t[:, 8].max()}, "
          f"halo candidates p50 {np.median(t[:, 9]):.0f} max {t[:, 9].max()}")
    for i, nm in enumerate(names):
        a, b = t[:, i], t[:, i + 1]
        ok = (a > 0) & (b > 0)
        v = (b[ok] - a[ok]) * 10 / 1000.0
        print(f"{nm:7s} p10 {np.percentile(v, 10):7.2f} p50 {np.percentile(v, 50):7.2f} p90 {np.percentile(v, 90):7.2f} "
              f"max {v.max():7.2f} us")
    if (t[:, 11] > 0).any():  # k_knn_wave (EPP_KNN_TILE=2): wave 0's queries and its query-loop cycles
        ok = t[:, 11] > 0
        cpq = t[ok, 12] / t[ok, 11]
        print(f"wave 0: queries p50 {np.median(t[ok, 11]):.0f}, s_memtime cycles per query p10 {np.percentile(cpq, 10):.0f} "
              f"p50 {np.median(cpq):.0f} p90 {np.percentile(cpq, 90):.0f}")
    tot = (t[:, 7] - t[:, 0]) * 10 / 1000.0
    print(f"block   p10 {np.percentile(tot, 10):7.2f} p50 {np.percentile(tot, 50):7.2f} p90 {np.percentile(tot, 90):7.2f} "
          f"max {tot.max():7.2f} us")
    # the slowest blocks: what they hold and where they are (grid from the workspace's KnnGrid)
    gw = d_ws.download(np.uint8, 64)
    dims = np.frombuffer(gw[40:52].tobytes(), np.int32)
    nbx, nby = (dims[0] + 3) // 4, (dims[1] + 3) // 4
    r0 = recs[0]
    tb = (r0[:, 7] - r0[:, 0]) * 10 / 1000.0
    b_ = idxs[0]  # block numbers
    print(f"grid dims {dims.tolist()}, blocks {nbx}x{nby}x{(dims[2] + 3) // 4}; corr(time, queries) "
          f"{np.corrcoef(tb, r0[:, 8])[0, 1]:.2f}, corr(time, halo) {np.corrcoef(tb, r0[:, 9])[0, 1]:.2f}")
    for i in np.argsort(tb)[::-1][:10]:
        bx, by, bz = b_[i] % nbx, (b_[i] // nbx) % nby, b_[i] // (nbx * nby)
        ph = [(r0[i, j + 1] - r0[i, j]) * 10 / 1000.0 if r0[i, j] and r0[i, j + 1] else -1 for j in range(7)]
        print(f"  block {b_[i]} ({bx},{by},{bz}) {tb[i]:.1f} us  queries {r0[i, 8]} halo {r0[i, 9]}  phases "
              + " ".join(f"{x:.1f}" for x in ph))
    for r in recs[:3]:
        st = (r[:, 0] - r[:, 0].min()) * 10 / 1000.0
        en = (r[:, 7] - r[:, 0].min()) * 10 / 1000.0
        print(f"launch: block starts p50 {np.median(st):.2f} max {st.max():.2f} us, ends max {en.max():.2f} us")


modes = sys.argv[1:] or ["1"]  # EPP_KNN_TILE values (2: k_knn_wave, its phases: scan, copy, first query, wave 0's rest, wait for the other waves)
for m in modes:
    os.environ["EPP_KNN_TILE"] = m
    recs, idxs = [], []
    for r in range(12):
        capi.check(L.epp_knn_grid_ws(d_n.ptr, n, k, 0.0, d_k.ptr, d_ws.ptr, ws, None))
        capi.sync()
        if r >= 2:
            tl = np.zeros((1024, 16), np.uint64)
            capi.check(L.epp_dbg_knn_tl(tl.ctypes.data, 1024))
            keep = tl[:, 7] != 0
            recs.append(tl[keep].astype(np.int64))
            idxs.append(np.nonzero(keep)[0])
    print(f"== EPP_KNN_TILE={m}")
    report(recs)
    # the last launch's retried queries (k_knn_retry): duration, start/end from the first
    # retry's start, bound in h^2
    hdr = d_ws.download(np.uint8, 80)
    nretry = int(hdr[60:64].view(np.int32)[0])
    hh = float(hdr[24:32].view(np.float64)[0])
    if nretry > 0 and hasattr(L, "epp_dbg_knn_retry_tl"):
        L.epp_dbg_knn_retry_tl.argtypes = [C.c_void_p, C.c_int64]
        rt = np.zeros((min(nretry, 4096), 4), np.uint64)
        capi.check(L.epp_dbg_knn_retry_tl(rt.ctypes.data, len(rt)))
        t0 = rt[:, 0].astype(np.int64)
        dur = (rt[:, 1].astype(np.int64) - t0) * 10 / 1000.0
        st = (t0 - t0.min()) * 10 / 1000.0
        b2 = rt[:, 2].view(np.float64) / (hh * hh)
        print(f"retry: {nretry} queries, duration p50 {np.median(dur):.2f} p90 {np.percentile(dur, 90):.2f} max {dur.max():.2f} us, "
              f"starts span {st.max():.2f} us, last end {(st + dur).max():.2f} us")
        for i in np.argsort(dur)[::-1][:6]:
            print(f"  retry node {int(rt[i, 3])}: {dur[i]:.2f} us from {st[i]:.2f}, bound {b2[i]:.2f} h^2")
