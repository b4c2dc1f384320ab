#!/bin/bash
# Round-1 profiles of the whole-model step: bench lines (cfg2/cfg3 geometric + e2e), the
# per-layer MLP timings, rocprofv3 kernel stats of the --model step, MLP phase stamps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r1mlp
mkdir -p $OUT
export TMPDIR=/tmp
for c in cfg2 cfg3; do
  timeout -k 10 300 python bench.py --config $c > $OUT/bench_$c.json 2> $OUT/bench_$c.err || exit 1
  timeout -k 10 200 python tools/bench_mlp.py --config $c > $OUT/bench_mlp_$c.jsonl 2> $OUT/bench_mlp_$c.err || exit 1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_model_$c -o run -- python3 bench.py --config $c --model --steps 20 --warmup 5 > $OUT/prof_model_$c.log 2>&1 || exit 1
done
timeout -k 10 200 python tools/stamp_mlp.py --fp > $OUT/stamp_mlp.jsonl 2> $OUT/stamp_mlp.err || exit 1
echo done
