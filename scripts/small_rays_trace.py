"""Kernel durations of scripts/rays_latency_probe.py's batches from its kernel trace (the
calls in order: 50 warm + 500 timed per batch size, then 500 single rays).
    python scripts/small_rays_trace.py gpurun_out/sr/prof/rl_kernel_trace.csv"""
import csv
import sys

import numpy as np

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
d = np.array([int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows])
for k, n in enumerate((1, 16, 64, 256, 512, 768, 1024, "one ray (check_ray_valid)")):
    seg = d[k * 550 + 50:(k + 1) * 550] if k < 7 else d[7 * 550:]
    print(f"{n}: kernel p50 {np.median(seg) / 1e3:.1f} us, p90 {np.percentile(seg, 90) / 1e3:.1f} us")
