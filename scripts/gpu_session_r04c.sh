#!/bin/bash
# Round-4 combined diagnostics session: k-NN tests + timeline + isolated planner trace +
# motions VALU mix (scripts/gpu_knn_session.sh), the A/B probes (scripts/gpu_ab_r04.sh) and
# the world-creation cost probe.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
MOTIONS_PMC=1 bash scripts/gpu_knn_session.sh || exit $?
bash scripts/gpu_ab_r04.sh || exit $?
timeout -k 10 60 ./scripts/world_create_probe || exit $?
echo all done
