#!/bin/bash
# k_states_v5 A/B (diagnostics): records read from L2 in the exact path, only lists and
# classes staged (-DEPP_V5_GREC) against the product, same flags (sha1) required.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop_on_fault() { case "$1" in 0) return 0 ;; *) echo "step $2 ended with $1: stopping"; exit "$1" ;; esac; }
for r in 1 2 3; do
  for lib in "" scripts/dbg/libepp_grec.so; do
    timeout -k 10 120 python scripts/states_ab.py $lib > gpurun_out/ab.log 2>&1; rc=$?
    tail -1 gpurun_out/ab.log; stop_on_fault $rc "states $lib"
  done
done
echo "all done"
