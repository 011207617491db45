#!/bin/bash
# Round-4 A/B probes (diagnostics): k_states_v5 staging / exact-path cost probes (WRONG
# answers by design: capped staging, no exact path) and the motion-kernel prefilter
# variant (same answers), each against the product build on one box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop_on_fault() { case "$1" in 0) return 0 ;; *) echo "step $2 ended with $1: stopping"; exit "$1" ;; esac; }
for r in 1 2; do
  for lib in "" scripts/dbg/libepp_dense.so scripts/dbg/libepp_noexact.so; do
    timeout -k 10 120 python scripts/states_ab.py $lib > gpurun_out/ab.log 2>&1; rc=$?
    tail -1 gpurun_out/ab.log; stop_on_fault $rc "states $lib"
  done
  timeout -k 10 120 python scripts/states_ab.py EPP_V5_BLOCK=256 > gpurun_out/ab.log 2>&1; rc=$?
  tail -1 gpurun_out/ab.log; stop_on_fault $rc "states 256"
  for lib in "" scripts/dbg/libepp_pfflush.so scripts/dbg/libepp_w1mask.so scripts/dbg/libepp_w1pf.so; do
    timeout -k 10 120 python scripts/motions_ab.py $lib > gpurun_out/ab.log 2>&1; rc=$?
    tail -1 gpurun_out/ab.log; stop_on_fault $rc "motions $lib"
  done
done
echo done
