#!/bin/bash
# k_motions_v5 A/B (diagnostics): the AABB prefilter in the queued test for the analytic
# mode only (-DEPP_MOTIONS_PF0) against the product, four rounds, same flags required.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop_on_fault() { case "$1" in 0) return 0 ;; *) echo "step $2 ended with $1: stopping"; exit "$1" ;; esac; }
for r in 1 2 3 4; do
  for lib in "" scripts/dbg/libepp_pf0.so; do
    timeout -k 10 120 python scripts/motions_ab.py $lib > gpurun_out/ab.log 2>&1; rc=$?
    tail -1 gpurun_out/ab.log; stop_on_fault $rc "motions $lib"
  done
done
echo "all done"
