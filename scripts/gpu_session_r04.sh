#!/bin/bash
# Round-4 GPU session: parity tests, smoke, the bench, rocprofv3 kernel traces of the bench
# headline and of one planner thread alone (scripts/planner_isolated.py).  Every GPU step has
# its own time limit; a fault/abort/timeout stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop_on_fault() { case "$1" in 0|1) return 0 ;; *) echo "step $2 ended with $1: stopping"; exit "$1" ;; esac; }
if [ -z "${SKIP_TESTS:-}" ]; then
  echo "== pytest -m gpu"
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1; rc=$?
  tail -15 gpurun_out/pytest_gpu.log; stop_on_fault $rc pytest
  echo "== smoke"
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
  tail -3 gpurun_out/smoke.log; stop_on_fault $rc smoke
fi
echo "== bench (driver shape: 20 steps)"
timeout -k 10 600 python bench.py --steps 20 --warmup 5 ${BENCH_ARGS:-} > gpurun_out/bench20.json 2> gpurun_out/bench20.err; rc=$?
tail -c 600 gpurun_out/bench20.json; tail -3 gpurun_out/bench20.err; stop_on_fault $rc bench20
echo "== bench (default)"
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?
tail -c 600 gpurun_out/bench.json; tail -3 gpurun_out/bench.err; stop_on_fault $rc bench
if [ -z "${SKIP_PROF:-}" ]; then
  echo "== rocprofv3 kernel trace of the bench headline"
  rm -rf gpurun_out/prof gpurun_out/prof_plan
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --no-cpu --no-plan --no-side > gpurun_out/prof_bench.json 2> gpurun_out/prof.err; rc=$?
  tail -3 gpurun_out/prof.err; stop_on_fault $rc rocprof
  echo "== rocprofv3 kernel trace of one planner thread, 20 segments"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_plan -o run -- python3 scripts/planner_isolated.py > gpurun_out/prof_plan.json 2> gpurun_out/prof_plan.err; rc=$?
  tail -3 gpurun_out/prof_plan.err; cat gpurun_out/prof_plan.json; stop_on_fault $rc rocprof_plan
fi
echo done
