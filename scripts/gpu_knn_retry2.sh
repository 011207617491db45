#!/bin/bash
# k-NN retry trial bound (diagnostics): the k-NN / planner tests, the timelines (blocks and
# retried queries) and the isolated planner trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop_on_fault() { case "$1" in 0) return 0 ;; *) echo "step $2 ended with $1: stopping"; exit "$1" ;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_planner.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "knn or plan" > gpurun_out/pytest_knn.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_knn.log; stop_on_fault $rc pytest
timeout -k 10 180 python scripts/knn_timeline.py 1 > gpurun_out/knn_tl.log 2>&1; rc=$?
grep "^retry\|^  retry\|^block" gpurun_out/knn_tl.log; stop_on_fault $rc knn_tl
rm -rf gpurun_out/prof_plan
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_plan -o run -- python3 scripts/planner_isolated.py > gpurun_out/prof_plan.json 2> gpurun_out/prof_plan.err; rc=$?
cat gpurun_out/prof_plan.json; stop_on_fault $rc prof_plan
python3 - <<'PY'
import csv
for r in list(csv.DictReader(open("gpurun_out/prof_plan/run_kernel_stats.csv")))[:5]:
    n = r["Name"].split("(anonymous namespace)::")[-1][:40]
    print(f"{n:40s} {r['Calls']:>4} avg {float(r['AverageNs'])/1e3:8.2f} min {float(r['MinNs'])/1e3:8.2f} max {float(r['MaxNs'])/1e3:8.2f} us")
PY
echo "all done"
