#!/bin/bash
# k-NN A/B over diagnostics builds (scripts/dbg/libepp_<name>.so, VARIANTS) against the
# in-tree library: scripts/knn_probe.py for each, alternating, twice (each checks its
# table against the all-pairs kernel).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2; do
  for v in cur ${VARIANTS:-}; do
    lib=$PWD/efficient-path-planner_amd/libepp.so; [ "$v" != cur ] && lib=$PWD/scripts/dbg/libepp_$v.so
    EPP_LIB=$lib timeout -k 10 180 python scripts/knn_probe.py 1 > gpurun_out/knn_v.log 2>&1; rc=$?
    echo "$v: $(grep 'per call' gpurun_out/knn_v.log)"
    [ $rc -eq 0 ] || { tail -5 gpurun_out/knn_v.log; exit $rc; }
  done
done
