#!/bin/bash
# k_knn_wave bring-up (diagnostics): the k-NN GPU tests (every kernel variant against the
# all-pairs kernel and numpy), then time per 63k-node table for k_knn_tile (1) and
# k_knn_wave (2), each table compared with the all-pairs one.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop_on_fault() { case "$1" in 0) return 0 ;; *) echo "step $2 ended with $1: stopping"; exit "$1" ;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_planner.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "knn" > gpurun_out/pytest_knn.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_knn.log; stop_on_fault $rc pytest
timeout -k 10 120 python scripts/knn_probe.py 1 2 1 2 > gpurun_out/kprobe.log 2>&1; rc=$?
cat gpurun_out/kprobe.log; stop_on_fault $rc knn_probe
rm -rf gpurun_out/kprof
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kprof -o run -- python3 scripts/knn_probe.py 2 > gpurun_out/kprof.log 2>&1; rc=$?
stop_on_fault $rc kprof
python3 - <<'PY'
import csv
for r in list(csv.DictReader(open("gpurun_out/kprof/run_kernel_stats.csv")))[:6]:
    n = r["Name"]; n = n[:n.find("(")] if "(" in n else n
    print(f"{n[-40:]:40s} {r['Calls']:>4} avg {float(r['AverageNs'])/1e3:8.2f} min {float(r['MinNs'])/1e3:8.2f} max {float(r['MaxNs'])/1e3:8.2f} us")
PY
echo "all done"
