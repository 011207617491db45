#!/bin/bash
# Motion-kernel A/B on one box (diagnostics): the collision + planner parity tests, then
# scripts/motions_ab.py on the product library and on ab/libepp_rounds.so (built with
# EXTRA=-DEPP_MOTIONS_ROUNDS), three rounds in alternation, then a short bench.
set -u
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_collision.py tests/test_gpu_planner.py > gpurun_out/mt.log 2>&1 || { tail -20 gpurun_out/mt.log; exit 1; }
tail -2 gpurun_out/mt.log
for r in 1 2 3; do
  timeout -k 10 120 python scripts/motions_ab.py || exit 1
  timeout -k 10 120 python scripts/motions_ab.py ab/libepp_rounds.so || exit 1
done
timeout -k 10 300 python bench.py --no-cpu --steps 20 --warmup 5 > gpurun_out/b20.json
