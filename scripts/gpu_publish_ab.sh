# Same-box A/B of the completion publish (one system-scope release per workgroup,
# completion.h) against ab/pkg_base (the previous revision): the GPU tests of every
# kernel that publishes (small queries, refit / check + refit, the planner's emit), then
# the C4 plan, the C5 step and the small ray batches, alternating builds.
set -o pipefail
mkdir -p gpurun_out/pub
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_collision.py tests/test_gpu_planner.py tests/test_gpu_minsnap.py > gpurun_out/pub/tests.log 2>&1 &&
for r in 1 2; do
  EPP_PROBE_CALLS=200 timeout -k 10 120 python scripts/plan_probe.py 16 > gpurun_out/pub/plan_cur$r.log 2>&1 &&
  EPP_PKG=ab/pkg_base EPP_PROBE_CALLS=200 timeout -k 10 120 python scripts/plan_probe.py 16 > gpurun_out/pub/plan_base$r.log 2>&1 &&
  timeout -k 10 120 python scripts/c5_step_probe.py > gpurun_out/pub/c5_cur$r.log 2>&1 &&
  EPP_PKG=ab/pkg_base timeout -k 10 120 python scripts/c5_step_probe.py > gpurun_out/pub/c5_base$r.log 2>&1 || exit 1
done
