#!/bin/bash
# more sampler lanes (and hardware queues): cfg2/cfg3/cfg5
set -o pipefail
OUT=gpurun_out/r3
mkdir -p $OUT
for c in cfg2 cfg3 cfg5; do
  for v in "2 4" "3 5" "3 8" "4 6" "4 8"; do
    set -- $v
    timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --e2e-steps 0 --sampler-lanes $1 --hw-queues $2 --sets 4 > $OUT/sl2_${c}_$1_$2.json 2> $OUT/sl2_${c}_$1_$2.err || { tail -20 $OUT/sl2_${c}_$1_$2.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/sl2_${c}_$1_$2.json')); print('$c lanes $1 queues $2', round(d['value']), round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms'],4))"
  done
done
