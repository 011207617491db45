#!/bin/bash
# Round-4 diagnostics session: GPU tests, k_states_v5 build variants (scripts/gpu_states_variants.sh)
# and the k_knn_tile phase timeline with its slowest blocks (scripts/knn_timeline.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop_on_fault() { case "$1" in 0|1) return 0 ;; *) echo "step $2 ended with $1: stopping"; exit "$1" ;; esac; }
echo "== pytest -m gpu"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -4 gpurun_out/pytest_gpu.log; stop_on_fault $rc pytest
echo "== states variants"
bash scripts/gpu_states_variants.sh; rc=$?; stop_on_fault $rc variants
echo "== knn timeline"
timeout -k 10 180 python scripts/knn_timeline.py > gpurun_out/knn_tl.log 2>&1; rc=$?
cat gpurun_out/knn_tl.log | grep -v "^launch"; stop_on_fault $rc knn_tl
echo done
