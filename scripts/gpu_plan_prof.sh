#!/bin/bash
# Kernel trace of the full plan alone (scripts/plan_probe.py, 4 planner threads): per-kernel
# time of the batched planner's stages -> gpurun_out/plan_prof/.
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/plan_prof
EPP_PROBE_CALLS=${EPP_PROBE_CALLS:-30} timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/plan_prof -o plan -- python3 scripts/plan_probe.py --child > gpurun_out/plan_prof/probe.log 2>&1
rc=$?
tail -4 gpurun_out/plan_prof/probe.log
f=$(find gpurun_out/plan_prof -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && python3 -c "
import csv,sys
rows=list(csv.DictReader(open('$f')))
for r in rows[:25]: print(r['Name'][:80].ljust(80), r['Calls'].rjust(6), '%9.1f'%(float(r['AverageNs'])/1e3), '%9.1f'%(float(r['MaxNs'])/1e3), r['Percentage'])
"
exit $rc
