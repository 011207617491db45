# k_pb_rows one-wave workgroups per CU (EPP_PB_ROWS_WG) under a kernel trace each: the
# kernel's own duration per C4 batch.
set -u -o pipefail
mkdir -p gpurun_out/rw
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for w in 16 20 24 28 32 40; do
  EPP_PB_ROWS_WG=$w EPP_PROBE_CALLS=40 timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rw/w$w -o k -- python scripts/plan_probe.py --child > gpurun_out/rw/w$w.log 2>&1 || exit 1
done
