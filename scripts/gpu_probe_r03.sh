#!/bin/bash
# Round-3 probe session (diagnostics): min-snap / planner GPU tests, refit A/B against
# scripts/dbg/libepp_prev.so, refit timeline.
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out
PYTEST_FILES="tests/test_gpu_minsnap.py tests/test_gpu_planner.py" AB_LIBS="prev" bash scripts/gpu_refit_ab.sh || exit $?
echo "== refit timeline"; timeout -k 10 120 python3 scripts/refit_timeline.py > gpurun_out/refit_tl.log 2>&1 || exit $?
tail -16 gpurun_out/refit_tl.log
echo "== C5 latency split"
PYTEST_K=minsnap_batch_golden bash scripts/gpu_c5probe.sh 2>&1 | grep -v "^\.\|passed" | head -60
