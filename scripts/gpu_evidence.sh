#!/bin/bash
# Round-5 evidence session: every GPU test, smoke, the bench (driver shape and default),
# rocprofv3 kernel traces (headline alone, whole bench, the batched planner alone) and the
# PMC FETCH_SIZE / WRITE_SIZE passes of the headline (separate runs) -> gpurun_out/ev/.
# Every GPU step has its own time limit; a fault/abort/timeout stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ev
export TMPDIR=/tmp
stop() { case "$1" in 0) return 0 ;; *) echo "step $2 ended with $1: stopping"; exit "$1" ;; esac; }
if [ -z "${SKIP_TESTS:-}" ]; then
  echo "== pytest -m gpu"
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/ev/pytest_gpu.log 2>&1; rc=$?
  tail -4 gpurun_out/ev/pytest_gpu.log; stop $rc pytest
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/ev/smoke.log 2>&1; rc=$?
  tail -1 gpurun_out/ev/smoke.log; stop $rc smoke
fi
echo "== bench (driver shape: 20 steps)"
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/ev/bench20.json 2> gpurun_out/ev/bench20.err; rc=$?
stop $rc bench20
echo "== bench (default)"
timeout -k 10 600 python bench.py > gpurun_out/ev/bench.json 2> gpurun_out/ev/bench.err; rc=$?
stop $rc bench
if [ -z "${SKIP_PROF:-}" ]; then
  echo "== rocprofv3: headline, whole bench, planner"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ev/prof -o run -- python3 bench.py --no-cpu --no-plan --no-side > gpurun_out/ev/prof_bench.json 2> gpurun_out/ev/prof.err; rc=$?
  stop $rc rocprof
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ev/prof_full -o run -- python3 bench.py --no-cpu > gpurun_out/ev/prof_full_bench.json 2> gpurun_out/ev/prof_full.err; rc=$?
  stop $rc rocprof_full
  EPP_PROBE_CALLS=30 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ev/prof_plan -o run -- python3 scripts/plan_probe.py --child > gpurun_out/ev/prof_plan.log 2>&1; rc=$?
  stop $rc rocprof_plan
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d gpurun_out/ev/pmc_$c -o run -- python3 bench.py --no-cpu --no-plan --no-side --steps 200 --warmup 20 > gpurun_out/ev/pmc_$c.json 2> gpurun_out/ev/pmc_$c.err; rc=$?
    stop $rc pmc_$c
  done
fi
echo done
