# k_pb_compact with its loads and membership issued before the look-back: the planner's GPU
# tests, a kernel trace of both builds, then plan_probe against ab/pkg_base, alternating.
set -o pipefail
mkdir -p gpurun_out/ca
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_planner.py > gpurun_out/ca/tests.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT &&
EPP_PROBE_CALLS=60 timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ca/pcur -o k -- python scripts/plan_probe.py --child > gpurun_out/ca/pcur.log 2>&1 &&
EPP_PKG=ab/pkg_base EPP_PROBE_CALLS=60 timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ca/pbase -o k -- python scripts/plan_probe.py --child > gpurun_out/ca/pbase.log 2>&1 &&
for r in 1 2 3; do
  EPP_PROBE_CALLS=300 timeout -k 10 120 python scripts/plan_probe.py 16 > gpurun_out/ca/cur$r.log 2>&1 &&
  EPP_PKG=ab/pkg_base EPP_PROBE_CALLS=300 timeout -k 10 120 python scripts/plan_probe.py 16 > gpurun_out/ca/base$r.log 2>&1 || exit 1
done
