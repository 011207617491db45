#!/bin/bash
# One GPU session: parity tests, smoke, a short bench, a rocprofv3 kernel-trace summary.
# Every GPU step has its own time limit; a fault/abort/timeout stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop_on_fault() {  # $1 = exit code, $2 = step name
  case "$1" in
    0|1) return 0 ;;   # pass / test failures: keep going
    *) echo "step $2 ended with $1: stopping (no further GPU work)"; exit "$1" ;;
  esac
}
echo "== pytest -m gpu"
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_gpu.log; stop_on_fault $rc pytest
echo "== smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
tail -3 gpurun_out/smoke.log; stop_on_fault $rc smoke
echo "== bench"
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?
tail -c 3000 gpurun_out/bench.json; tail -3 gpurun_out/bench.err; stop_on_fault $rc bench
echo "== rocprofv3 kernel trace"
rm -rf gpurun_out/prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 50 --no-cpu > gpurun_out/prof_bench.json 2> gpurun_out/prof.err; rc=$?
tail -3 gpurun_out/prof.err; stop_on_fault $rc rocprof
find gpurun_out/prof -name "*stats*" | head
echo done
