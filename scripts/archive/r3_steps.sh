#!/bin/bash
# default-layout bench lines at several step counts, interleaved (fill/drain amortisation)
set -o pipefail
OUT=gpurun_out/r3/steps
mkdir -p $OUT
for r in 1 2; do
  for c in ${CONFIGS:-cfg2}; do
    for k in ${STEPS:-50:10 400:40 1000:50}; do
      set -- ${k//:/ }
      tag=${c}_$1_$r
      timeout -k 10 300 python3 bench.py --config $c --steps $1 --warmup $2 --no-cpu-baseline --e2e-steps 0 ${ARGS:-} > $OUT/b_$tag.json 2> $OUT/b_$tag.err || { tail -20 $OUT/b_$tag.err; exit 1; }
      python3 -c "import json; d=json.load(open('$OUT/b_$tag.json')); print('$tag', round(d['value']), round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms'],4))"
    done
  done
done
