#!/bin/bash
# One GPU session: the -m gpu tests (optionally a -k filter), smoke(), then bench.py with its
# defaults; logs under gpurun_out/.  Usage: scripts/gpu_round.sh [pytest -k expr] [--no-bench]
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
K="${1:-}"
BENCH=1
[ "${2:-}" = "--no-bench" ] && BENCH=0
args=(-u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider)
[ -n "$K" ] && args+=(-k "$K")
timeout -k 10 900 python "${args[@]}" > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log | tail -20; exit 1; }
tail -1 gpurun_out/smoke.log
if [ $BENCH = 1 ]; then
  timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -30 gpurun_out/bench.err; exit 1; }
  python - <<'PY'
import json
d = json.load(open("gpurun_out/bench.json"))
print("value", d["value"], "frac", d["roofline"]["frac"], "kernel_ms", d["roofline"]["kernel_ms"])
fp = d["full_plan"]
print("full_plan", fp["ms_per_track"], fp["ms_per_track_p50"], fp.get("comm_n_ranks"))
print("parity", json.dumps(d.get("parity")))
PY
fi
