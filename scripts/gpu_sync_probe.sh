#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 120 python scripts/sync_probe.py > gpurun_out/sync_probe.log 2>&1; rc=$?
cat gpurun_out/sync_probe.log; exit $rc
