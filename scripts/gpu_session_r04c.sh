#!/bin/bash
# Round-4 combined session: every GPU test, then the k-NN timeline + isolated planner trace +
# motions VALU mix (scripts/gpu_knn_session.sh without its test step), the A/B probes
# (scripts/gpu_ab_r04.sh) and the world-creation cost probe.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
# (the k-NN tests first: the previous session faulted in test_knn_grid_large)
timeout -k 10 300 python -u -m pytest tests/test_gpu_planner.py -m gpu -x -q --timeout 120 --timeout-method thread -k knn > gpurun_out/pytest_knn.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_knn.log
[ $rc -ne 0 ] && { echo "pytest (knn) ended with $rc: stopping"; exit $rc; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -4 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && { echo "pytest ended with $rc: stopping"; exit $rc; }
MOTIONS_PMC=1 PYTEST_K="knn_vs_bruteforce" bash scripts/gpu_knn_session.sh || exit $?
bash scripts/gpu_ab_r04.sh || exit $?
timeout -k 10 60 ./scripts/world_create_probe || exit $?
echo all done
