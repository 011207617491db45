#!/bin/bash
# One iteration session on the GPU box: selected parity tests (PYTEST_FILES / PYTEST_K),
# then optional probes (PROBES: a space-separated list of scripts/*.py to run under
# rocprofv3 --kernel-trace --stats, each into gpurun_out/prof_<name>).  Every GPU step
# has its own time limit; a fault / abort / timeout stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop_on_fault() { case "$1" in 0|1) return 0 ;; *) echo "step $2 ended with $1: stopping"; exit "$1" ;; esac; }
if [ -n "${PYTEST_FILES:-}" ]; then
  echo "== pytest ${PYTEST_FILES} ${PYTEST_K:-}"
  timeout -k 10 600 python -u -m pytest ${PYTEST_FILES} -m gpu -q -x --timeout 120 --timeout-method thread \
    ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_iter.log 2>&1; rc=$?
  tail -15 gpurun_out/pytest_iter.log; stop_on_fault $rc pytest
fi
for p in ${PROBES:-}; do
  name=$(basename "$p" .py)
  echo "== probe $p ${PROBE_ARGS:-}"
  rm -rf "gpurun_out/prof_$name"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "gpurun_out/prof_$name" -o run -- \
    python3 "scripts/$name.py" ${PROBE_ARGS:-} > "gpurun_out/$name.log" 2>&1; rc=$?
  tail -12 "gpurun_out/$name.log"; stop_on_fault $rc "$name"
  f=$(ls gpurun_out/prof_$name/*kernel_stats.csv 2>/dev/null | head -1)
  [ -n "$f" ] && python3 - "$f" <<'EOF'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:14]:
    print(f'{r["Name"][:70]:70s} calls {r["Calls"]:>6s} avg_us {float(r["AverageNs"])/1e3:9.2f} total_ms {float(r["TotalDurationNs"])/1e6:8.3f}')
EOF
done
echo done
