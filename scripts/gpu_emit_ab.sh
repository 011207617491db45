#!/bin/bash
# k_pb_emit workgroup count sweep (diagnostics): the planner probe under several
# EPP_PB_EMIT_BLOCKS values, each under a kernel trace (k_pb_emit's own duration) and
# with the planner's phases.
set -u -o pipefail
mkdir -p gpurun_out/emit
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for eb in 64 128 256 512; do
  EPP_PB_EMIT_BLOCKS=$eb EPP_PROBE_CALLS=60 timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/emit/eb$eb -o k -- python scripts/plan_probe.py --child > gpurun_out/emit/eb$eb.log 2>&1 || exit 1
done
