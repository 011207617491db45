#!/bin/bash
# Parity tests, kernel microbench, then rocprofv3 PMC passes over k_states.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -4 gpurun_out/pytest_gpu.log
case $rc in 0|1) ;; *) echo "pytest ended with $rc: stopping"; exit $rc;; esac
timeout -k 10 600 python scripts/kbench.py > gpurun_out/kbench.log 2>&1; rc=$?
grep -E "c2_|empty|c3_" gpurun_out/kbench.log
[ $rc -eq 0 ] || exit $rc
i=0
for ctrs in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" \
            "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR" \
            "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $ctrs --output-format csv -d gpurun_out/pmc/p$i -o run -- python3 scripts/run_states.py > gpurun_out/pmc/p$i.log 2>&1; rc=$?
  [ $rc -eq 0 ] || { echo "pmc pass $i failed rc=$rc"; tail -5 gpurun_out/pmc/p$i.log; exit $rc; }
done
echo pmc done
