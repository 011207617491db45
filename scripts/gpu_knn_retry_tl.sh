#!/bin/bash
# k-NN timelines (diagnostics build): k_knn_tile's blocks and k_knn_retry's queries.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 180 python scripts/knn_timeline.py 1 > gpurun_out/knn_tl.log 2>&1; rc=$?
grep -v "^launch\|^  block" gpurun_out/knn_tl.log; exit $rc
