# k_pb_sample taking the batch's problems without an upload dispatch: the planner's GPU
# tests, then plan_probe against ab/pkg_base (the previous revision), alternating.
set -o pipefail
mkdir -p gpurun_out/sa
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_planner.py > gpurun_out/sa/tests.log 2>&1 &&
for r in 1 2 3 4; do
  EPP_PROBE_CALLS=300 timeout -k 10 120 python scripts/plan_probe.py 16 > gpurun_out/sa/cur$r.log 2>&1 &&
  EPP_PKG=ab/pkg_base EPP_PROBE_CALLS=300 timeout -k 10 120 python scripts/plan_probe.py 16 > gpurun_out/sa/base$r.log 2>&1 || exit 1
done
