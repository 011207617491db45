#!/bin/bash
# k_pb_rows launch width A/B (diagnostics): the planner probe's stage trace under several
# EPP_PB_ROWS_WG values (one-wave workgroups per CU), twice each.
set -u
for rep in 1 2; do
  for wg in 28 16 12 40; do
    EPP_PB_ROWS_WG=$wg EPP_PB_TRACE=1 EPP_PLAN_THREADS=16 EPP_PROBE_CALLS=30 timeout -k 10 120 python scripts/plan_probe.py --child > /tmp/pr.log 2> /tmp/pr.err || exit 1
    echo "wg $wg rep $rep: $(python3 -c "
import re, numpy as np
d={}
for l in open('/tmp/pr.err'):
    if l.startswith('pb_trace:'):
        for k,v in re.findall(r'(\w+)=(\d+)', l): d.setdefault(k,[]).append(int(v))
print(' '.join(f'{k}={np.median(v[3:]):.0f}' for k,v in d.items()))")"
  done
done
