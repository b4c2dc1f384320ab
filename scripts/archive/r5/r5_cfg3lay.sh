#!/bin/bash
# Round 5: cfg3 layouts after the attention / FP4 changes: 2 vs 3 sampler streams, sets,
# side layouts (500 steps), interleaved twice.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r5/cfg3lay
mkdir -p $OUT
run() { n=$1; shift; timeout -k 10 300 python3 bench.py --config cfg3 --steps 500 --warmup 50 --e2e-steps 0 --no-cpu-baseline "$@" > $OUT/b_$n.json 2> $OUT/b_$n.err || { tail -20 $OUT/b_$n.err; exit 1; }
  echo "$n $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(round(d['value']), round(d['ms_per_step'],4), d.get('verified'), d['config'].get('hw_queues'))" $OUT/b_$n.json)"; }
for rep in 1 2; do
  run def_$rep
  run l3s9q7_$rep --sampler-lanes 3 --sets 9 --hw-queues 7
  run l3s9q7b_$rep --sampler-lanes 3 --sets 9 --hw-queues 7 --side-layout b
  run l3s9q8_$rep --sampler-lanes 3 --sets 9 --hw-queues 8
  run l2s8q6_$rep --sets 8
done
