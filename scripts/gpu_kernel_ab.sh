#!/bin/bash
# Same-box A/B of the planner's kernels: rocprofv3 kernel stats of scripts/plan_probe.py
# (--child, EPP_PROBE_CALLS calls) under each package built by scripts/ab_pkg.sh, twice in
# alternation.  Usage: scripts/gpu_kernel_ab.sh NAME... (ab/pkg_NAME); prints the kernels
# matching $KERNELS (a regex; default the batch's k_pb_ and k_states kernels).
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for rep in 1 2; do
  for n in "$@"; do
    out=gpurun_out/kab_${n}_$rep
    EPP_PKG=ab/pkg_$n EPP_PROBE_CALLS=${EPP_PROBE_CALLS:-20} timeout -k 10 120 rocprofv3 --kernel-trace --stats \
      --output-format csv -d $out -o run -- python3 scripts/plan_probe.py --child > $out.log 2>&1 || exit 1
    echo "== $n (rep $rep): $(grep -o 'pre_compute_traj p50 [0-9.]* ms' $out.log)"
    python3 - "$out/run_kernel_stats.csv" "${KERNELS:-k_pb_|k_states}" <<'PY'
import csv, re, sys
for r in csv.DictReader(open(sys.argv[1])):
    if re.search(sys.argv[2], r["Name"]):
        print(f'   {r["Name"][:60]:60s} {int(r["Calls"]):5d} {float(r["AverageNs"]) / 1e3:7.2f} us')
PY
  done
done
