#!/bin/bash
# private side streams per buffer set x sampler lanes x hardware queues
set -o pipefail
OUT=gpurun_out/r3/private
mkdir -p $OUT
for c in ${CONFIGS:-cfg2 cfg3 cfg5}; do
  for v in ${VARIANTS:-"3 6 9 -" "3 12 6 p" "4 12 4 p" "4 16 8 p" "6 20 6 p" "8 28 8 p"}; do
    set -- $v
    P=""; [ "$4" = "p" ] && P="--private-side"
    tag=${c}_$1_$2_$3_$4
    timeout -k 10 200 python3 bench.py --config $c --steps 400 --warmup 30 --no-cpu-baseline --e2e-steps 0 \
      --sampler-lanes $1 --hw-queues $2 --sets $3 $P > $OUT/b_$tag.json 2> $OUT/b_$tag.err || { tail -20 $OUT/b_$tag.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/b_$tag.json')); print('$tag', round(d['value']), round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms'],4))"
  done
done
