#!/bin/bash
# Round-3 probe session: min-snap tests, refit A/B (current vs scripts/dbg/libepp_prev.so), refit timeline.
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out
PYTEST_FILES="tests/test_gpu_minsnap.py tests/test_gpu_planner.py" AB_LIBS="prev" bash scripts/gpu_refit_ab.sh || exit $?
echo "== refit timeline"; timeout -k 10 120 python3 scripts/refit_timeline.py > gpurun_out/refit_tl.log 2>&1 || exit $?
tail -30 gpurun_out/refit_tl.log
echo "== planner timeline (1 thread)"
rm -rf gpurun_out/prof_plan
EPP_PLAN_THREADS=1 timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/prof_plan -o run -- python3 scripts/plan_probe.py --child > gpurun_out/plan_tl_run.log 2>&1 || exit $?
python3 scripts/plan_timeline.py gpurun_out/prof_plan > gpurun_out/plan_tl.log 2>&1; tail -60 gpurun_out/plan_tl.log
