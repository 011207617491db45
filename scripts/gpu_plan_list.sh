#!/bin/bash
# Row-restricted k-NN as listed retry queries: the planner tests, the isolated planner trace,
# then the C4 full-plan probe with the restriction (1.5) and without (0), twice.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop_on_fault() { case "$1" in 0) return 0 ;; *) echo "step $2 ended with $1: stopping"; exit "$1" ;; esac; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_planner.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_pl.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_pl.log; stop_on_fault $rc pytest
rm -rf gpurun_out/prof_plan
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_plan -o run -- python3 scripts/planner_isolated.py > gpurun_out/prof_plan.json 2> gpurun_out/prof_plan.err; rc=$?
cat gpurun_out/prof_plan.json; stop_on_fault $rc prof_plan
python3 - <<'PY'
import csv
for r in list(csv.DictReader(open("gpurun_out/prof_plan/run_kernel_stats.csv")))[:12]:
    n = r["Name"].split("(anonymous namespace)::")[-1][:40]
    print(f"{n:40s} {r['Calls']:>4} avg {float(r['AverageNs'])/1e3:8.2f} min {float(r['MinNs'])/1e3:8.2f} max {float(r['MaxNs'])/1e3:8.2f} us")
PY
for rep in 1 2; do
  for e in 1.5 0; do
    EPP_PLAN_ELLIPSE=$e timeout -k 10 200 python3 scripts/plan_probe.py 4 > gpurun_out/sweep_$e.log 2>&1; rc=$?
    head -1 gpurun_out/sweep_$e.log; stop_on_fault $rc sweep_$e
  done
done
echo "all done"
