#!/bin/bash
# SQ counter passes over the k-NN kernels (scripts/knn_probe.py, tiled), one pass per run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_WAVES SQ_INSTS_BRANCH SQ_INSTS_SMEM"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  rm -rf gpurun_out/kpmc$i
  timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d gpurun_out/kpmc$i -o run -- python3 scripts/knn_probe.py 1 > gpurun_out/kpmc$i.log 2>&1; rc=$?
  tail -1 gpurun_out/kpmc$i.log
  [ $rc -ne 0 ] && { echo "pass $i ended with $rc"; exit $rc; }
  python3 scripts/pmc_summary.py gpurun_out/kpmc$i "k_knn_tile|k_knn_retry"
done
echo done
