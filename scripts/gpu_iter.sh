#!/bin/bash
# Development loop on the GPU: parity tests, planner end to end, kernel microbench, timeline.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop_on_fault() { case "$1" in 0|1) return 0 ;; *) echo "step $2 ended with $1: stopping"; exit "$1" ;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_gpu.log; stop_on_fault $rc pytest
[ $rc -eq 0 ] || exit 1
timeout -k 10 120 python -u scripts/diag_plan2.py 3 > gpurun_out/plan2.log 2>&1; rc=$?
tail -3 gpurun_out/plan2.log; stop_on_fault $rc plan
[ $rc -eq 0 ] || exit 1
timeout -k 10 600 python scripts/kbench.py "${KB:-.}" > gpurun_out/kbench.log 2>&1; rc=$?
cat gpurun_out/kbench.log | grep -v "^\s*$" | tail -40; stop_on_fault $rc kbench
timeout -k 10 300 python scripts/timeline.py > gpurun_out/timeline.log 2>&1; rc=$?
head -c 1500 gpurun_out/timeline.log; stop_on_fault $rc timeline
