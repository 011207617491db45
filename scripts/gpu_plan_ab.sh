#!/bin/bash
# Same-box A/B of planner knobs (scripts/plan_probe.py, 16 planner threads): each line an
# environment, run twice in alternation.  Usage: scripts/gpu_plan_ab.sh "ENV=a" "ENV=b" ...
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in 1 2; do
  for e in "$@"; do
    echo "== $e (rep $rep)"
    env $e EPP_PROBE_CALLS=${EPP_PROBE_CALLS:-30} timeout -k 10 100 python scripts/plan_probe.py 16 | grep -v "all (ms)\|slowest" || exit 1
  done
done
