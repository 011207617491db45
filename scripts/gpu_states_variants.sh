#!/bin/bash
# k_states_v5 build variants on one box (diagnostics): scripts/dbg/libepp_<V>.so built with
# -DEPP_V5_<V> (efficient-path-planner_amd/Makefile EXTRA=...), timed alternately with the
# product build by scripts/states_ab.py; the flag digests must agree.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop_on_fault() { case "$1" in 0) return 0 ;; *) echo "step $2 ended with $1: stopping"; exit "$1" ;; esac; }
for r in 1 2 3; do
  for v in "" ${VARIANTS:-SPL8 TWOPHASE PRIO}; do
    lib=""; [ -n "$v" ] && lib="scripts/dbg/libepp_$v.so"
    timeout -k 10 120 python scripts/states_ab.py $lib > gpurun_out/states_ab.log 2>&1; rc=$?
    tail -1 gpurun_out/states_ab.log; stop_on_fault $rc "states_ab $v"
  done
done
