#!/bin/bash
# side-lane layouts a / b with several sampler lanes (full steps and side work alone)
set -o pipefail
OUT=gpurun_out/r3/layout
mkdir -p $OUT
for c in ${CONFIGS:-cfg2 cfg3}; do
  for lay in a b; do
    for v in ${VARIANTS:-3:6:9 3:7:9 4:8:8}; do
      set -- ${v//:/ }
      for only in ${ONLY:-full side}; do
        D=""; [ "$only" != "full" ] && D="--diag-only $only"
        tag=${c}_${lay}_$1_$2_$3_$only
        PN2_SIDE_LAYOUT=$lay timeout -k 10 200 python3 bench.py --config $c --steps 400 --warmup 30 --no-cpu-baseline --e2e-steps 0 \
          --sampler-lanes $1 --hw-queues $2 --sets $3 $D > $OUT/b_$tag.json 2> $OUT/b_$tag.err || { tail -20 $OUT/b_$tag.err; exit 1; }
        python3 -c "import json; d=json.load(open('$OUT/b_$tag.json')); print('$tag', round(d['value']), round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms'],4))"
      done
    done
  done
done
