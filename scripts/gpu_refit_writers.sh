# Refit writer workgroups (EPP_REFIT_ROWS_PER_WRITER): the min-snap GPU tests at 64, then
# the C5 step probe and a kernel trace of it at 128 / 64 / 43 / 32 rows per writer.
# (a diagnostics A/B of round 6: the knob it sets was removed again after it measured slower)
set -u -o pipefail
mkdir -p gpurun_out/wr
EPP_REFIT_ROWS_PER_WRITER=64 timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_minsnap.py > gpurun_out/wr/tests.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for w in 128 64 43 32 128 64; do
  EPP_REFIT_ROWS_PER_WRITER=$w timeout -k 10 120 python scripts/c5_step_probe.py > gpurun_out/wr/c5_$w.$RANDOM.log 2>&1 || exit 1
done
for w in 128 64 32; do
  EPP_REFIT_ROWS_PER_WRITER=$w timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/wr/p$w -o k -- python scripts/c5_step_probe.py > gpurun_out/wr/p$w.log 2>&1 || exit 1
done
