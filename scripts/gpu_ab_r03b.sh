#!/bin/bash
# Same-box A/B of the current libepp.so against scripts/dbg/libepp_head.so (ab_build.sh /
# c5_ab_build.sh): k-NN probe (alternating, twice each) and the native C5 loops.  Each GPU
# step has its own time limit; a fault / abort / timeout stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop_on_fault() { case "$1" in 0) return 0 ;; *) echo "step $2 ended with $1: stopping"; exit "$1" ;; esac; }
if [ -n "${PYTEST_K:-}${PYTEST_FILES:-}" ]; then
  timeout -k 10 600 python -u -m pytest ${PYTEST_FILES:-tests} -m gpu -q -x --timeout 120 --timeout-method thread \
    ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_ab.log 2>&1; rc=$?
  tail -8 gpurun_out/pytest_ab.log; stop_on_fault $rc pytest
fi
for r in 1 2; do
  for lib in scripts/dbg/libepp_head.so efficient-path-planner_amd/libepp.so; do
    echo "== knn_probe $lib ($r)"
    EPP_LIB=$PWD/$lib timeout -k 10 180 python scripts/knn_probe.py 1 > gpurun_out/knn_ab.log 2>&1; rc=$?
    tail -4 gpurun_out/knn_ab.log; stop_on_fault $rc knn_probe
  done
done
echo "== c5 A/B"
timeout -k 10 300 python scripts/c5_ab.py scripts/dbg/c5_native_head tools/c5_native > gpurun_out/c5_ab.log 2>&1; rc=$?
cat gpurun_out/c5_ab.log; stop_on_fault $rc c5_ab
echo done
