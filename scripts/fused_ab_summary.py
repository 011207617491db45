"""Summary of scripts/gpu_fused_ab.sh: per run, the median wall time of the shortcut's and
the pruning's ray batches (pairs_trace lines) and pre_compute_traj's p50 / mean.
    python scripts/fused_ab_summary.py [gpurun_out/fused]"""
import glob
import os
import re
import sys

import numpy as np

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/fused"
for f in sorted(glob.glob(os.path.join(d, "o*_*.log"))):
    txt = open(f).read()
    sc = [float(x) for x in re.findall(r"pairs_trace: shortcut .*? ([\d.]+) us", txt)]
    pr = [float(x) for x in re.findall(r"pairs_trace: prune .*? ([\d.]+) us", txt)]
    pairs = [int(x) for x in re.findall(r"pairs_trace: shortcut paths \d+ pairs (\d+)", txt)]
    m = re.search(r"pre_compute_traj p50 ([\d.]+) ms \(mean ([\d.]+)", txt)
    sc, pr = sc[2:], pr[2:]  # (the warm-up calls)
    print(f"{os.path.basename(f)}: shortcut rays p50 {np.median(sc):.1f} us (pairs p50 {np.median(pairs):.0f}), "
          f"pruning rays p50 {np.median(pr):.1f} us, sum p50 {np.median(np.add(sc, pr)):.1f} us; "
          f"pre_compute_traj p50 {m.group(1)} ms mean {m.group(2)} ms")
