#!/bin/bash
# k_knn_wave phase timeline (diagnostics build, scripts/knn_timeline.py 2 1).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 180 python scripts/knn_timeline.py 2 1 > gpurun_out/knn_tl.log 2>&1; rc=$?
grep -v "^launch" gpurun_out/knn_tl.log; exit $rc
