#!/bin/bash
# k_states_v5 A/B (diagnostics): two states per lane at eight waves per SIMD (-DEPP_V5_SPL2)
# against the product, same flags (sha1) required.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop_on_fault() { case "$1" in 0) return 0 ;; *) echo "step $2 ended with $1: stopping"; exit "$1" ;; esac; }
for r in 1 2 3; do
  for lib in "" scripts/dbg/libepp_spl2.so; do
    timeout -k 10 120 python scripts/states_ab.py $lib > gpurun_out/ab.log 2>&1; rc=$?
    tail -1 gpurun_out/ab.log; stop_on_fault $rc "states $lib"
  done
done
echo "all done"
