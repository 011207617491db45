#!/bin/bash
# Parity tests + kernel microbench (diagnostics session).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -8 gpurun_out/pytest_gpu.log
case $rc in 0|1) ;; *) echo "pytest ended with $rc: stopping"; exit $rc;; esac
timeout -k 10 600 python scripts/kbench.py > gpurun_out/kbench.log 2>&1; rc=$?
cat gpurun_out/kbench.log | tail -20
exit $rc
