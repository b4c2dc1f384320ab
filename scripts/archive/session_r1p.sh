#!/bin/bash
# End-of-milestone GPU session: full parity suite, default bench (with CPU baseline), cfg3 and
# cfg5 bench lines, rocprof kernel trace/stats and PMC traffic passes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=r1p bash scripts/gpu_check.sh || exit $?
for c in cfg3 cfg5; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > gpurun_out/bench_${c}_r1p.json 2> gpurun_out/bench_${c}_r1p.err || exit $?
  cut -c1-200 gpurun_out/bench_${c}_r1p.json
done
