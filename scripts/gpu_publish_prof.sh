# Kernel durations (rocprofv3 kernel trace) of the C5 step and the C4 plan, this build and
# ab/pkg_base: the kernels that publish completion slots (k_check_refit, k_pb_emit,
# k_motions_small).
set -o pipefail
mkdir -p gpurun_out/pubp
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT &&
for b in cur base; do
  if [ $b = base ]; then export EPP_PKG=ab/pkg_base; else unset EPP_PKG; fi
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pubp/c5_$b -o k -- python scripts/c5_step_probe.py > gpurun_out/pubp/c5_$b.log 2>&1 &&
  EPP_PROBE_CALLS=100 timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pubp/plan_$b -o k -- python scripts/plan_probe.py 16 > gpurun_out/pubp/plan_$b.log 2>&1 || exit 1
done
