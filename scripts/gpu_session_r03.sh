#!/bin/bash
# Round-3 session: the full check (tests, smoke, bench, rocprof, PMC), then the motion
# kernels' A/B against scripts/dbg/libepp_head.so and the k-NN probe.
set -u
cd "${GRAFT_REPO_ROOT}"
bash scripts/gpu_check.sh || exit $?
echo "== motions A/B (head, cur, head, cur)"
bash scripts/gpu_motions_ab.sh || exit $?
PROBES="knn_probe" PROBE_ARGS="1" bash scripts/gpu_iter.sh || exit $?
