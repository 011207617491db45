#!/bin/bash
# Quick GPU validation: parity tests, smoke, one bench run (each step time-limited;
# stops at the first fault/abort/timeout).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop_on_fault() { case "$1" in 0|1) return 0 ;; *) echo "step $2 ended with $1: stopping"; exit "$1" ;; esac; }
echo "== pytest -m gpu"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_gpu.log; stop_on_fault $rc pytest
echo "== smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
tail -3 gpurun_out/smoke.log; stop_on_fault $rc smoke
echo "== bench"
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?
tail -c 3000 gpurun_out/bench.json; tail -3 gpurun_out/bench.err; stop_on_fault $rc bench
echo done
