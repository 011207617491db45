"""Row-restriction bound factor (EPP_PLAN_ELLIPSE) over many C4 tracks (diagnostics): per
factor, in its own process, pre_compute_traj on world seeds 100..100+N-1 (65,536 samples,
16 planner threads), twice per track; prints restricted rows, fallbacks and the p50 time."""
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "efficient-path-planner_amd")]

if len(sys.argv) > 1 and sys.argv[1] == "--child":
    import numpy as np
    import online_traj_planner as otp
    from eppamd import config, synth
    n = int(sys.argv[2])
    cfg = config.load(os.path.join(ROOT, "configs", "config.json"))
    cfg["world_properties"]["lower_bound"] = [-6, -6, 0]
    cfg["world_properties"]["upper_bound"] = [6, 6, 2]
    cfg["path_planner_properties"]["samples_fmt"] = 65536
    geom = config.geometry(cfg)
    fd, path = tempfile.mkstemp(suffix=".json")
    with os.fdopen(fd, "w") as f:
        json.dump(cfg, f)
    ts, fb, rows, segs_fb = [], 0, 0, []
    for seed in range(100, 100 + n):
        gates, obstacles = synth.track_world(seed)
        cps = synth.gate_checkpoints(gates, geom.gate_height, 0.55)
        otg = otp.OnlineTrajGenerator(cps[0], cps[-1], gates, obstacles, path)
        for rep in range(2):
            t = time.perf_counter()
            otg.pre_compute_traj(0.0)
            ts.append((time.perf_counter() - t) * 1e3)
            s = otg.planner_stats()
            fb += s["fallbacks"]
            rows += s["restricted_rows"]
            if s["fallbacks"]:
                segs_fb.append((seed, rep, s["fallbacks"]))
    os.unlink(path)
    print(f"EPP_PLAN_ELLIPSE={os.environ.get('EPP_PLAN_ELLIPSE', 'default')}: {len(ts)} calls, p50 {np.median(ts):.3f} ms, "
          f"mean {np.mean(ts):.3f} ms, fallbacks {fb} ({fb / len(ts):.3f} per call), restricted rows per call "
          f"{rows / len(ts):.0f}; calls with fallbacks {segs_fb}", flush=True)
else:
    n = sys.argv[1] if len(sys.argv) > 1 else "32"
    for fac in sys.argv[2:] or ["1.5", "1.3", "1.2"]:
        env = dict(os.environ, EPP_PLAN_ELLIPSE=fac, EPP_PLAN_THREADS="16", EPP_PATH_WRITER="0")
        r = subprocess.run([sys.executable, __file__, "--child", n], env=env, timeout=600)
        if r.returncode:
            sys.exit(r.returncode)
