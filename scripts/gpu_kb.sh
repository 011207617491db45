#!/bin/bash
# Kernel microbench only (KB = name filter regex).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python scripts/kbench.py "${KB:-.}" > gpurun_out/kbench.log 2>&1; rc=$?
grep -v "^\s*$" gpurun_out/kbench.log | tail -40; exit $rc
