#!/bin/bash
# Round-3 probe session (diagnostics): planner / min-snap GPU tests, k-NN probe, full-plan
# probe (1 and 4 planner threads), planner timeline (1 thread), refit A/B and timeline.
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out
PYTEST_FILES="tests/test_gpu_minsnap.py tests/test_gpu_planner.py" PROBES="knn_probe" PROBE_ARGS="1" bash scripts/gpu_iter.sh || exit $?
echo "== plan probe"; timeout -k 10 300 python3 scripts/plan_probe.py 1 4 > gpurun_out/plan_probe.log 2>&1 || exit $?
cat gpurun_out/plan_probe.log
echo "== planner timeline (1 thread)"
rm -rf gpurun_out/prof_plan
EPP_PLAN_THREADS=1 timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/prof_plan -o run -- python3 scripts/plan_probe.py --child > gpurun_out/plan_tl_run.log 2>&1 || exit $?
python3 scripts/plan_timeline.py gpurun_out/prof_plan > gpurun_out/plan_tl.log 2>&1; tail -40 gpurun_out/plan_tl.log
AB_LIBS="${AB_LIBS:-}" bash scripts/gpu_refit_ab.sh || exit $?
echo "== refit timeline"; timeout -k 10 120 python3 scripts/refit_timeline.py > gpurun_out/refit_tl.log 2>&1 || exit $?
tail -16 gpurun_out/refit_tl.log
