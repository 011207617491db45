#!/bin/bash
# k-NN iteration session (diagnostics): the k-NN / planner GPU tests, the k_knn_tile phase
# timeline (scripts/knn_timeline.py) and the isolated planner trace (scripts/planner_isolated.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop_on_fault() { case "$1" in 0|1) return 0 ;; *) echo "step $2 ended with $1: stopping"; exit "$1" ;; esac; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_planner.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "${PYTEST_K:-knn or plan or scan}" > gpurun_out/pytest_knn.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_knn.log; stop_on_fault $rc pytest
timeout -k 10 180 python scripts/knn_timeline.py > gpurun_out/knn_tl.log 2>&1; rc=$?
grep -v "^launch" gpurun_out/knn_tl.log | head -14; stop_on_fault $rc knn_tl
rm -rf gpurun_out/prof_plan
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_plan -o run -- python3 scripts/planner_isolated.py > gpurun_out/prof_plan.json 2> gpurun_out/prof_plan.err; rc=$?
cat gpurun_out/prof_plan.json; stop_on_fault $rc prof_plan
python3 - <<'PY'
import csv
for r in list(csv.DictReader(open("gpurun_out/prof_plan/run_kernel_stats.csv")))[:8]:
    n = r["Name"]; n = n[:n.find("(")] if "(" in n else n
    print(f"{n[-40:]:40s} {r['Calls']:>4} avg {float(r['AverageNs'])/1e3:8.2f} min {float(r['MinNs'])/1e3:8.2f} max {float(r['MaxNs'])/1e3:8.2f} us")
PY
if [ -n "${MOTIONS_PMC:-}" ]; then
  bash scripts/gpu_pmc_motions.sh; rc=$?; stop_on_fault $rc pmc_motions
  python3 scripts/pmc_summary.py gpurun_out/mpmc3 k_motions_v5
fi
echo done
