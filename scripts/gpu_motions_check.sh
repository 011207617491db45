#!/bin/bash
# Motion-kernel parity after a change (diagnostics): the collision tests (every motion
# variant, the C3 full-size test) and the planner tests, then C3 timing against the
# previous revision (scripts/ab_build.sh HEAD prev).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop_on_fault() { case "$1" in 0) return 0 ;; *) echo "step $2 ended with $1: stopping"; exit "$1" ;; esac; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_collision.py tests/test_gpu_planner.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_mo.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_mo.log; stop_on_fault $rc pytest
for r in 1 2 3; do
  for lib in "" ${AB_LIB:-scripts/dbg/libepp_prev.so}; do
    timeout -k 10 120 python scripts/motions_ab.py $lib > gpurun_out/ab.log 2>&1; rc=$?
    tail -1 gpurun_out/ab.log; stop_on_fault $rc "motions $lib"
  done
done
echo "all done"
