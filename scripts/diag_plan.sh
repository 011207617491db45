set -u
mkdir -p gpurun_out
echo "== brute"; EPP_KNN_IMPL=1 timeout -k 10 120 python -u scripts/diag_plan2.py 3 > gpurun_out/d1.log 2>&1; rc=$?; tail -4 gpurun_out/d1.log; [ $rc -eq 0 ] || exit $rc
echo "== default"; timeout -k 10 120 python -u scripts/diag_plan2.py 3 > gpurun_out/d2.log 2>&1; rc=$?; tail -4 gpurun_out/d2.log; [ $rc -eq 0 ] || exit $rc
echo "== bench"; timeout -k 10 300 python -u bench.py --no-side --no-cpu --steps 5 --warmup 1 > gpurun_out/d3.log 2>&1; rc=$?; tail -c 600 gpurun_out/d3.log; exit $rc
