# Motion-kernel study on C3 (diagnostics): A/B of the tree's build against a reference
# build (scripts/dbg/libepp_head.so), the per-wave timeline build, and the SQ counter passes.
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "motion" > gpurun_out/pytest_motion.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_motion.log; [ $rc -eq 0 ] || exit $rc
for cfg in "scripts/dbg/libepp_head.so" "" "scripts/dbg/libepp_head.so" ""; do
  timeout -k 10 120 python scripts/motions_ab.py $cfg || exit $?
done
[ "${STUDY_QUICK:-0}" = 1 ] && exit 0
timeout -k 10 120 python scripts/motions_timeline.py v5 || exit $?
bash scripts/gpu_pmc_motions.sh || exit $?
