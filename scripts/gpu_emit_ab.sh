#!/bin/bash
# k_pb_emit workgroup count sweep (diagnostics): the planner probe with the stage trace
# (EPP_PB_TRACE=1) under several EPP_PB_EMIT_BLOCKS values.
set -u
for eb in 16 32 64 128 256 32; do
  EPP_PB_EMIT_BLOCKS=$eb EPP_PB_TRACE=1 EPP_PLAN_THREADS=16 EPP_PROBE_CALLS=30 timeout -k 10 120 python scripts/plan_probe.py --child > gpurun_out/pbt_$eb.log 2> gpurun_out/pbt_$eb.err || exit 1
  echo "eb $eb: $(grep phases gpurun_out/pbt_$eb.log)"
done
