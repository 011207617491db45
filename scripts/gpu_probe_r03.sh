#!/bin/bash
# Round-3 probe session (diagnostics): k-NN grid density (EPP_KNN_NPC) vs k_knn_tile time.
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for npc in 1.5 1.25 1.1 1.0 1.35 1.5; do
  EPP_KNN_NPC=$npc timeout -k 10 120 python3 scripts/knn_probe.py 1 > gpurun_out/knn_v.log 2>&1 || { tail -5 gpurun_out/knn_v.log; exit 1; }
  grep "per call" gpurun_out/knn_v.log | sed "s|^|npc $npc |"
done
for npc in 1.25 1.1; do
  echo "== timeline npc $npc"
  EPP_KNN_NPC=$npc timeout -k 10 120 python3 scripts/knn_timeline.py > gpurun_out/knn_tl.log 2>&1 || exit 1
  grep -v "^launch" gpurun_out/knn_tl.log | tail -10
done
