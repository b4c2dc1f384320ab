#!/bin/bash
# Round 4: the driver's 20-step window against the number of buffer sets (9 = default, 12, 16),
# interleaved, five runs each.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4/sets20
mkdir -p $OUT
for i in 1 2 3 4 5; do
  for s in 9 12 16; do
    timeout -k 10 300 python3 bench.py --no-cpu-baseline --e2e-steps 0 --latency-reps 0 --steps 20 --warmup 5 --sets $s > $OUT/b_s${s}_$i.json 2> $OUT/b_s${s}_$i.err || { tail -20 $OUT/b_s${s}_$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/b_s${s}_$i.json')); print('s$s run $i', round(d['value']), d.get('verified'))"
  done
done
