#!/bin/bash
# End-of-milestone GPU session (part 1): full parity suite, cfg2 bench, rocprof kernel
# trace/stats and PMC traffic for cfg2, cfg3 and cfg5.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=r1q BENCH_ARGS="--no-cpu-baseline" bash scripts/gpu_check.sh || exit $?
for c in cfg3 cfg5; do
  TAG=r1q_$c SKIP_TESTS=1 BENCH_ARGS="--config $c --no-cpu-baseline" bash scripts/gpu_check.sh || exit $?
done
