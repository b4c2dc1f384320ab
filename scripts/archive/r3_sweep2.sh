#!/bin/bash
# layouts again after the per-lane end events
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r3/sweep2
mkdir -p $OUT
for L in "cfg2:3:b:7:9:own" "cfg2:4:b:8:12:own" "cfg2:3:a:6:9:own" "cfg2:3:b:7:6:own" "cfg3:2:a:6:6:own" "cfg3:3:a:7:9:own" "cfg3:3:b:8:9:own" "cfg5:5:a:8:10:behind" "cfg5:4:a:8:10:own"; do
  IFS=: read c l s q n ch <<< "$L"
  A="--config $c --sampler-lanes $l --side-layout $s --hw-queues $q --sets $n --chain $ch --no-cpu-baseline --e2e-steps 0"
  timeout -k 10 200 python3 bench.py $A > $OUT/b.json 2> $OUT/err.log || { tail -5 $OUT/err.log; exit 1; }
  timeout -k 10 200 python3 bench.py $A --steps 20 --warmup 5 > $OUT/d.json 2> $OUT/err.log || { tail -5 $OUT/err.log; exit 1; }
  python3 -c "
import json; a=json.load(open('$OUT/b.json')); b=json.load(open('$OUT/d.json'))
print('$L', round(a['value']), round(a['roofline']['avg_launch_ms'],3), '| 20 steps', round(b['value']))"
done
