#!/bin/bash
# Refit A/B on one box: the min-snap GPU tests, then refit_prof.py under rocprofv3 for the
# in-tree libepp and each scripts/dbg/libepp_<name>.so named in AB_LIBS.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -n "${PYTEST_FILES:-}" ]; then
  timeout -k 10 600 python -u -m pytest ${PYTEST_FILES} -m gpu -q -x --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_ab.log 2>&1; rc=$?
  tail -5 gpurun_out/pytest_ab.log
  case $rc in 0) ;; *) echo "pytest ended with $rc: stopping"; exit $rc ;; esac
fi
for name in cur ${AB_LIBS:-}; do
  lib=""; [ "$name" != cur ] && lib="$PWD/scripts/dbg/libepp_$name.so"
  rm -rf "gpurun_out/prof_ab_$name"
  EPP_LIB="$lib" timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "gpurun_out/prof_ab_$name" -o run -- \
    python3 scripts/refit_prof.py > "gpurun_out/ab_$name.log" 2>&1; rc=$?
  echo "$name $(tail -1 gpurun_out/ab_$name.log)"
  case $rc in 0) ;; *) echo "$name ended with $rc: stopping"; exit $rc ;; esac
  f=$(ls gpurun_out/prof_ab_$name/*kernel_stats.csv | head -1)
  grep refit "$f" | cut -d, -f1-4 | sed "s/^/$name /"
done
echo done
