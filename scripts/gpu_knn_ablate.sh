#!/bin/bash
# k_knn_tile exact-phase ablation (diagnostics build): timeline with the product kernel (1)
# and with the exact phase's inserts skipped (5: gathers only, no answer, no retries).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 180 python scripts/knn_timeline.py 1 5 > gpurun_out/knn_tl.log 2>&1; rc=$?
grep -v "^launch\|^  block" gpurun_out/knn_tl.log; exit $rc
