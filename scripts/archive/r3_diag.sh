#!/bin/bash
# what bounds the multi-lane pipeline: samplers alone, side work alone, both
set -o pipefail
OUT=gpurun_out/r3/diag
mkdir -p $OUT
for c in ${CONFIGS:-cfg2 cfg3 cfg5}; do
  for v in ${VARIANTS:-"2 5 6" "3 6 9" "4 7 8"}; do
    set -- $v
    for only in full samplers side; do
      D=""; [ "$only" != "full" ] && D="--diag-only $only"
      tag=${c}_$1_$2_$3_$only
      timeout -k 10 200 python3 bench.py --config $c --steps 400 --warmup 30 --no-cpu-baseline --e2e-steps 0 \
        --sampler-lanes $1 --hw-queues $2 --sets $3 $D > $OUT/b_$tag.json 2> $OUT/b_$tag.err || { tail -20 $OUT/b_$tag.err; exit 1; }
      python3 -c "import json; d=json.load(open('$OUT/b_$tag.json')); print('$tag', round(d['value']), round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms'],4))"
    done
  done
done
