#!/bin/bash
# One GPU session: parity tests, smoke, the bench, a rocprofv3 kernel-trace summary of the
# bench, and the two PMC passes (FETCH_SIZE, WRITE_SIZE) for the roofline traffic figure.
# Every GPU step has its own time limit; a fault/abort/timeout stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop_on_fault() {  # $1 = exit code, $2 = step name
  case "$1" in
    0|1) return 0 ;;   # pass / test failures: keep going
    *) echo "step $2 ended with $1: stopping (no further GPU work)"; exit "$1" ;;
  esac
}
echo "== pytest -m gpu"
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_gpu.log; stop_on_fault $rc pytest
echo "== smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
tail -3 gpurun_out/smoke.log; stop_on_fault $rc smoke
echo "== bench"
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?
tail -c 1500 gpurun_out/bench.json; tail -3 gpurun_out/bench.err; stop_on_fault $rc bench
echo "== rocprofv3 kernel trace of the bench headline (no plan / side legs: one launch shape)"
rm -rf gpurun_out/prof gpurun_out/prof_full
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --no-cpu --no-plan --no-side > gpurun_out/prof_bench.json 2> gpurun_out/prof.err; rc=$?
tail -3 gpurun_out/prof.err; stop_on_fault $rc rocprof
echo "== rocprofv3 kernel trace of the whole bench (plan + side legs)"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_full -o run -- python3 bench.py --no-cpu > gpurun_out/prof_full_bench.json 2> gpurun_out/prof_full.err; rc=$?
tail -3 gpurun_out/prof_full.err; stop_on_fault $rc rocprof_full
for c in FETCH_SIZE WRITE_SIZE; do
  echo "== rocprofv3 --pmc $c"
  rm -rf gpurun_out/pmc_$c
  timeout -k 10 600 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc_$c -o run -- python3 bench.py --no-cpu --no-side --no-plan > gpurun_out/pmc_$c.json 2> gpurun_out/pmc_$c.err; rc=$?
  tail -2 gpurun_out/pmc_$c.err; stop_on_fault $rc pmc_$c
done
# (summaries are written locally afterwards — only gpurun_out/ comes back from the box:
#   python3 scripts/profile_summary.py gpurun_out rNN && cp gpurun_out/bench.json profiles/rNN_bench.json)
echo done
