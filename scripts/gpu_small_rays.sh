# The small ray kernel after a change: its parity tests (collision + planner), then the
# batch-size latency probe under the kernel trace, this build and ab/pkg_base alternating.
set -o pipefail
mkdir -p gpurun_out/sr
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_collision.py tests/test_gpu_planner.py -k "motion or ray or shortcut or include_gates2 or precompute or plan" > gpurun_out/sr/tests.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT &&
for r in 1 2; do
  timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/sr/cur$r -o rl -- python scripts/rays_latency_probe.py > gpurun_out/sr/cur$r.log 2>&1 &&
  EPP_PKG=ab/pkg_base timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/sr/base$r -o rl -- python scripts/rays_latency_probe.py > gpurun_out/sr/base$r.log 2>&1 || exit 1
done
