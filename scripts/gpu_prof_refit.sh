set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python scripts/refit_prof.py && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_refit -o run -- python3 scripts/refit_prof.py > gpurun_out/prof_refit.log 2>&1; rc=$?
tail -3 gpurun_out/prof_refit.log
find gpurun_out/prof_refit -name "*kernel_stats.csv" | head -1 | xargs cat | cut -d, -f1-8
exit $rc
