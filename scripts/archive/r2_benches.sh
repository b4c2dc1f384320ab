#!/bin/bash
# Round 2 bench lines for cfg2 / cfg3 / cfg5 (default arguments, whole-model e2e field included)
# and rocprofv3 kernel stats of cfg5; logs under gpurun_out/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
for C in cfg2 cfg3 cfg5; do
  echo "== bench $C"
  timeout -k 10 400 python -u bench.py --config $C > $OUT/bench_$C.json 2> $OUT/bench_$C.err || { tail -5 $OUT/bench_$C.err; exit 1; }
  cut -c1-300 $OUT/bench_$C.json
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_cfg5 -o run -- python3 bench.py --config cfg5 --steps 20 --warmup 5 --no-cpu-baseline --e2e-steps 0 > $OUT/prof_cfg5.log 2>&1 && echo "== done"
