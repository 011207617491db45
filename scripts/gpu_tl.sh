#!/bin/bash
# Per-wave timeline of the default k_states variant (diagnostics).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python scripts/timeline.py > gpurun_out/timeline.log 2>&1; rc=$?
cat gpurun_out/timeline.log; exit $rc
