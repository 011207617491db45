# C5 latency diagnostics: minsnap/planner parity tests, round-trip floors, the A11 split,
# the C5 step split and the refit phase timeline (each step time-limited).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -15 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 scripts/latency_probe > gpurun_out/latency_probe.log 2>&1; rc=$?; cat gpurun_out/latency_probe.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python scripts/c5_probe.py > gpurun_out/c5_probe.log 2>&1; rc=$?; cat gpurun_out/c5_probe.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python scripts/a11_probe.py > gpurun_out/a11_probe.log 2>&1; rc=$?; cat gpurun_out/a11_probe.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python scripts/c5_breakdown.py > gpurun_out/c5_breakdown.log 2>&1; rc=$?; cat gpurun_out/c5_breakdown.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python scripts/refit_timeline.py > gpurun_out/refit_tl.log 2>&1; rc=$?; cat gpurun_out/refit_tl.log; [ $rc -eq 0 ] || exit $rc
if [ -n "${WITH_BENCH:-}" ]; then
  timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?; tail -c 2500 gpurun_out/bench.json; exit $rc
fi
