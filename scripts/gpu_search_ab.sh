# Host search change A/B: the planner's GPU tests, then plan_probe against ab/pkg_base (the
# previous revision), alternating; the slowest problem's restricted search and the
# searches phase are the figures to compare.
set -o pipefail
mkdir -p gpurun_out/se
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_planner.py > gpurun_out/se/tests.log 2>&1 &&
for r in 1 2 3; do
  EPP_PROBE_CALLS=300 timeout -k 10 120 python scripts/plan_probe.py 16 > gpurun_out/se/cur$r.log 2>&1 &&
  EPP_PKG=ab/pkg_base EPP_PROBE_CALLS=300 timeout -k 10 120 python scripts/plan_probe.py 16 > gpurun_out/se/base$r.log 2>&1 || exit 1
done
