#!/bin/bash
# Development loop on the GPU: parity tests, kernel microbench, per-wave timeline.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop_on_fault() { case "$1" in 0|1) return 0 ;; *) echo "step $2 ended with $1: stopping"; exit "$1" ;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_gpu.log; stop_on_fault $rc pytest
[ $rc -eq 0 ] || exit 1
timeout -k 10 600 python scripts/kbench.py > gpurun_out/kbench.log 2>&1; rc=$?
cat gpurun_out/kbench.log | grep -v "^\s*$" | tail -40; stop_on_fault $rc kbench
timeout -k 10 300 python scripts/timeline.py > gpurun_out/timeline.log 2>&1; rc=$?
cat gpurun_out/timeline.log; stop_on_fault $rc timeline
