#!/bin/bash
# Full-plan A/B on one box (diagnostics): planner GPU tests, then scripts/plan_probe.py for
# the in-tree package and each scripts/dbg/pkg_<name> in AB_PKGS (scripts/ab_pkg.sh), with
# the planner thread counts in PLAN_THREADS (default "4 1"); optional k-NN probe.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -n "${PYTEST_FILES:-}" ]; then
  timeout -k 10 600 python -u -m pytest ${PYTEST_FILES} -m gpu -q -x --timeout 120 --timeout-method thread \
    ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_ab.log 2>&1; rc=$?
  tail -5 gpurun_out/pytest_ab.log
  case $rc in 0) ;; *) echo "pytest ended with $rc: stopping"; exit $rc ;; esac
fi
for rep in 1 2; do
  for name in cur ${AB_PKGS:-}; do
    pkg=""; [ "$name" != cur ] && pkg="$PWD/scripts/dbg/pkg_$name"
    EPP_PKG="$pkg" timeout -k 10 300 python3 scripts/plan_probe.py ${PLAN_THREADS:-4 1} > "gpurun_out/plan_ab_$name.log" 2>&1; rc=$?
    grep -v slowest "gpurun_out/plan_ab_$name.log"
    case $rc in 0) ;; *) echo "$name ended with $rc: stopping"; exit $rc ;; esac
  done
done
if [ -n "${KNN:-}" ]; then
  PROBES="knn_probe" PROBE_ARGS="1" bash scripts/gpu_iter.sh || exit $?
fi
echo done
