#!/bin/bash
# native plan: buffer sets x sampler lanes x hardware queues
set -o pipefail
OUT=gpurun_out/r3/plansets
mkdir -p $OUT
for c in ${CONFIGS:-cfg2 cfg3 cfg5}; do
  for v in ${VARIANTS:-"2 4 4" "2 4 6" "3 5 6" "3 6 6" "3 6 9" "4 6 8" "4 8 8" "4 8 12"}; do
    set -- $v
    timeout -k 10 200 python3 bench.py --config $c --steps 400 --warmup 30 --no-cpu-baseline --e2e-steps 0 \
      --sampler-lanes $1 --hw-queues $2 --sets $3 > $OUT/b_${c}_$1_$2_$3.json 2> $OUT/b_${c}_$1_$2_$3.err || { tail -20 $OUT/b_${c}_$1_$2_$3.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/b_${c}_$1_$2_$3.json')); print('$c lanes $1 queues $2 sets $3', round(d['value']), round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms'],4))"
  done
done
