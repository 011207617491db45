#!/bin/bash
# bench headline: graph replay vs host loop, and a rocprofv3 kernel trace of the default
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for a in "" "--host-loop" ""; do
  timeout -k 10 120 python bench.py --no-cpu --no-plan --no-side $a > gpurun_out/g.json || exit 1
  python -c "import json;d=json.load(open('gpurun_out/g.json'));print('$a', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['config']['launch'])"
done
rm -rf gpurun_out/prof_g
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_g -o run -- python3 bench.py --no-cpu --no-plan --no-side > gpurun_out/prof_g.json 2> gpurun_out/prof_g.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/prof_g.json'));print('under rocprof', d['roofline']['kernel_ms'])"
head -2 gpurun_out/prof_g/run_kernel_stats.csv | cut -c1-60,150-400
