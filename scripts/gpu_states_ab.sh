#!/bin/bash
# k_states_v5 launch-shape A/B on one box (diagnostics): the state-kernel parity tests,
# then scripts/states_ab.py alternating the default shape and EPP_V5_BLOCK=${ALT:-256}.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop_on_fault() { case "$1" in 0) return 0 ;; *) echo "step $2 ended with $1: stopping"; exit "$1" ;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_collision.py -m gpu -q -x --timeout 120 --timeout-method thread \
  -k "${PYTEST_K:-every_kernel_variant or states_full_size or racing}" > gpurun_out/pytest_states.log 2>&1; rc=$?
tail -4 gpurun_out/pytest_states.log; stop_on_fault $rc pytest
for r in 1 2 3; do
  for v in "" "EPP_V5_BLOCK=${ALT:-256}"; do
    echo "== states_ab ${v:-default} ($r)"
    timeout -k 10 120 python scripts/states_ab.py $v > gpurun_out/states_ab.log 2>&1; rc=$?
    tail -2 gpurun_out/states_ab.log; stop_on_fault $rc states_ab
  done
done
