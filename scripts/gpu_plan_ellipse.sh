#!/bin/bash
# Row-restricted k-NN table download: the planner tests, then the isolated planner with the
# ellipsoid (default) and with the whole table (EPP_PLAN_ELLIPSE=0), then the bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop_on_fault() { case "$1" in 0) return 0 ;; *) echo "step $2 ended with $1: stopping"; exit "$1" ;; esac; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_planner.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_pl.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_pl.log; stop_on_fault $rc pytest
for e in 1.5 0 1.5 0; do
  EPP_PLAN_ELLIPSE=$e timeout -k 10 300 python3 scripts/planner_isolated.py > gpurun_out/pl_$e.json 2>&1; rc=$?
  echo "ellipse $e: $(tail -c 400 gpurun_out/pl_$e.json)"; stop_on_fault $rc pl_$e
done
timeout -k 10 600 python bench.py > gpurun_out/bench_pl.json 2> gpurun_out/bench_pl.err; rc=$?
python3 -c "
import json; d=json.loads(open('gpurun_out/bench_pl.json').read().strip().splitlines()[-1])
f=d['full_plan']; print('full_plan', f['ms_per_track'], f['ms_per_track_p50'], f['one_segment'])
print('c1', d.get('c1_plan', {}).get('ms_per_plan'), d['value'])"; stop_on_fault $rc bench
echo "all done"
