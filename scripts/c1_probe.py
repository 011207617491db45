"""C1 plan latency under planner knobs (diagnostics): bench.py's c1_plan (single gate + 4
obstacles, pre_compute_traj) in a child process per environment given, alternating twice.
usage: python scripts/c1_probe.py "ENV=a ENV2=b" "ENV=c" ..."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if len(sys.argv) > 1 and sys.argv[1] == "--child":
    sys.path[:0] = [ROOT, os.path.join(ROOT, "efficient-path-planner_amd")]
    import bench
    r = bench.c1_plan(reps=60)
    print(json.dumps({k: r[k] for k in ("ms_per_plan", "ms_per_plan_p50")}))
else:
    for rep in range(2):
        for envs in sys.argv[1:] or [""]:
            env = dict(os.environ)
            for kv in envs.split():
                k, v = kv.split("=", 1)
                env[k] = v
            out = subprocess.run([sys.executable, __file__, "--child"], env=env, capture_output=True, text=True,
                                 timeout=300)
            if out.returncode:
                print(out.stderr[-2000:])
                sys.exit(out.returncode)
            print(f"{envs or 'default'} (rep {rep + 1}): {out.stdout.strip().splitlines()[-1]}", flush=True)
