set -o pipefail
mkdir -p gpurun_out/sa2
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT &&
EPP_PROBE_CALLS=60 timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sa2/pcur -o k -- python scripts/plan_probe.py --child > gpurun_out/sa2/pcur.log 2>&1 &&
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_planner.py -k "plan_once or bench_tracks or include_gates2" > gpurun_out/sa2/tests.log 2>&1
