# Same-box A/B of planPathsIncludeGates2's fused pruning (EPP_FUSED_PRUNE=0: the shortcut's
# and the pruning's ray batches apart): GPU tests of the path, then plan_probe runs with the
# batches' own wall times (EPP_PAIRS_TRACE) alternating on / off.
set -o pipefail
mkdir -p gpurun_out/fused
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_planner.py -k "rays_both or include_gates2 or precompute_traj" > gpurun_out/fused/tests.log 2>&1 &&
for r in 1 2 3; do
  EPP_PAIRS_TRACE=1 EPP_PROBE_CALLS=300 timeout -k 10 120 python scripts/plan_probe.py 16 > gpurun_out/fused/on_$r.log 2>&1 &&
  EPP_PAIRS_TRACE=1 EPP_FUSED_PRUNE=0 EPP_PROBE_CALLS=300 timeout -k 10 120 python scripts/plan_probe.py 16 > gpurun_out/fused/off_$r.log 2>&1 || exit 1
done
