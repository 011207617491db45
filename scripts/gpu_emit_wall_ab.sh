set -o pipefail
mkdir -p gpurun_out/emit2
for r in 1 2 3; do
  EPP_PB_EMIT_BLOCKS=64 EPP_PROBE_CALLS=200 timeout -k 10 120 python scripts/plan_probe.py 16 > gpurun_out/emit2/e64_$r.log 2>&1 &&
  EPP_PROBE_CALLS=200 timeout -k 10 120 python scripts/plan_probe.py 16 > gpurun_out/emit2/e128_$r.log 2>&1 || exit 1
done
