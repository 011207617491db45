#!/bin/bash
# k-NN A/B (diagnostics): the product against ${AB_LIB} (default: one retry workgroup per
# CU, -DEPP_KNN_RETRY_PER_CU=1), time per table + equality with
# the all-pairs table.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop_on_fault() { case "$1" in 0) return 0 ;; *) echo "step $2 ended with $1: stopping"; exit "$1" ;; esac; }
for r in 1 2 3; do
  for lib in efficient-path-planner_amd/libepp.so ${AB_LIB:-scripts/dbg/libepp_r1.so}; do
    timeout -k 10 120 python scripts/knn_probe.py $lib 1 > gpurun_out/kprobe.log 2>&1; rc=$?
    tail -1 gpurun_out/kprobe.log; stop_on_fault $rc knn_probe
  done
done
echo "all done"
