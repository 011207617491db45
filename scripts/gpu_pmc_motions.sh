#!/bin/bash
# SQ counter passes over the C3 motion kernels (scripts/motions_run.py), one pass per run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_INSTS_BRANCH SQ_INSTS_SMEM"
# the VALU mix: FP64 arithmetic vs integer / conversion work (per-SE sums; the rest of
# SQ_INSTS_VALU is compares, selects, moves, bit and lane operations)
P3="SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  rm -rf gpurun_out/mpmc$i
  timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d gpurun_out/mpmc$i -o run -- python3 scripts/motions_run.py > gpurun_out/mpmc$i.log 2>&1; rc=$?
  tail -2 gpurun_out/mpmc$i.log
  [ $rc -ne 0 ] && { echo "pass $i ended with $rc"; exit $rc; }
done
rm -rf gpurun_out/mkt
timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/mkt -o run -- python3 scripts/motions_run.py > gpurun_out/mkt.log 2>&1 || { echo "kernel trace failed"; exit 1; }
python3 scripts/pmc_summary.py gpurun_out/mpmc1 k_motions_v5 > gpurun_out/motions_pmc.txt
python3 scripts/pmc_summary.py gpurun_out/mpmc2 k_motions_v5 >> gpurun_out/motions_pmc.txt
python3 scripts/pmc_summary.py gpurun_out/mpmc3 k_motions_v5 >> gpurun_out/motions_pmc.txt
python3 scripts/motions_valu.py gpurun_out/motions_valu.json
echo done
