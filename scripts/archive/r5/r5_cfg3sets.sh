#!/bin/bash
# Round 5: cfg3 buffer sets 6 / 8 / 10 / 12 (2 sampler streams), 500 steps, interleaved twice,
# and the driver-style 20-step window at the best two.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r5/cfg3sets
mkdir -p $OUT
run() { n=$1; shift; timeout -k 10 300 python3 bench.py --config cfg3 --e2e-steps 0 --no-cpu-baseline "$@" > $OUT/b_$n.json 2> $OUT/b_$n.err || { tail -20 $OUT/b_$n.err; exit 1; }
  echo "$n $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(round(d['value']), round(d['ms_per_step'],4), d.get('verified'))" $OUT/b_$n.json)"; }
for rep in 1 2; do
  for s in 6 8 10 12; do run s${s}_$rep --steps 500 --warmup 50 --sets $s; done
done
for rep in 1 2 3; do
  for s in 6 8 10; do run d20s${s}_$rep --steps 20 --warmup 5 --sets $s; done
done
