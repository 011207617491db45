#!/bin/bash
# SQ PMC passes over 20 launches of k_states on 1M states, default vs exact-path ablation.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmc1m
export TMPDIR=/tmp
CT="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU"
CT2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_BUSY_CYCLES"
for v in 1 2; do
  i=0
  for ctrs in "$CT" "$CT2"; do
    i=$((i+1))
    EPP_V5_PAIRS=$v timeout -s KILL 90 rocprofv3 --pmc $ctrs --output-format csv -d gpurun_out/pmc1m/v${v}p$i -o run -- python3 scripts/run_states.py 1m > gpurun_out/pmc1m/v${v}p$i.log 2>&1; rc=$?
    [ $rc -eq 0 ] || { echo "pmc pass v$v $i failed rc=$rc"; tail -5 gpurun_out/pmc1m/v${v}p$i.log; }
  done
done
echo pmc done
