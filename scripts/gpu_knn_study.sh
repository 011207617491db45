#!/bin/bash
# k-NN study session (diagnostics): SQ counter passes over k_knn_tile (3 passes: cycles,
# instruction / LDS counts, LDS stalls + VALU mix), the phase timeline with the no-insert
# ablations (diagnostics build), and the fixed-point candidate variant against the product
# (scripts/knn_probe.py: time per table + equality with the all-pairs table).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
stop_on_fault() { case "$1" in 0) return 0 ;; *) echo "step $2 ended with $1: stopping"; exit "$1" ;; esac; }
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_WAVES SQ_INSTS_BRANCH SQ_LDS_IDX_ACTIVE"
P3="SQ_LDS_UNALIGNED_STALL SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT64 SQ_ACTIVE_INST_SCA"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  rm -rf gpurun_out/kpmc$i
  timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d gpurun_out/kpmc$i -o run -- python3 scripts/knn_probe.py 1 > gpurun_out/kpmc$i.log 2>&1; rc=$?
  tail -1 gpurun_out/kpmc$i.log
  stop_on_fault $rc "pmc pass $i"
  python3 scripts/pmc_summary.py gpurun_out/kpmc$i "k_knn_tile|k_knn_retry"
done
timeout -k 10 240 python scripts/knn_timeline.py 1 5 6 > gpurun_out/knn_tl.log 2>&1; rc=$?
grep -v "^launch" gpurun_out/knn_tl.log | grep -v "^  block" ; stop_on_fault $rc knn_tl
for lib in efficient-path-planner_amd/libepp.so scripts/dbg/libepp_pack8.so efficient-path-planner_amd/libepp.so scripts/dbg/libepp_pack8.so; do
  timeout -k 10 120 python scripts/knn_probe.py $lib 1 > gpurun_out/kprobe.log 2>&1; rc=$?
  echo "$lib: $(tail -2 gpurun_out/kprobe.log | tr '\n' ' ')"; stop_on_fault $rc knn_probe
done
echo "all done"
