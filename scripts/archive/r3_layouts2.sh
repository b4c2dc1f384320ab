#!/bin/bash
# side layouts (PN2_SIDE_LAYOUT) x sampler lanes, interleaved repetitions on one box;
# VARIANTS = cfg:layout:lanes:queues:sets ...
set -o pipefail
OUT=gpurun_out/r3/layouts2
mkdir -p $OUT
for r in $(seq ${REPS:-2}); do
  for v in ${VARIANTS:-cfg2:a:3:5:9 cfg2:b:3:6:9 cfg2:c:3:6:9 cfg2:d:3:7:9 cfg3:a:3:6:9 cfg3:c:3:7:9 cfg3:d:3:8:9 cfg3:a:2:5:6}; do
    set -- ${v//:/ }
    tag=$1_$2_$3_$4_$5_$r
    PN2_SIDE_LAYOUT=$2 timeout -k 10 200 python3 bench.py --config $1 --steps 400 --warmup 30 --no-cpu-baseline --e2e-steps 0 \
      --sampler-lanes $3 --hw-queues $4 --sets $5 ${ARGS:-} > $OUT/b_$tag.json 2> $OUT/b_$tag.err || { tail -20 $OUT/b_$tag.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/b_$tag.json')); print('$tag', round(d['value']), round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms'],4))"
  done
done
