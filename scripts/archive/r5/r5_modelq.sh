#!/bin/bash
# Round 5: the whole-model step with more hardware queues (each buffer set's private lane-1
# stream on its own queue) and more buffer sets.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r5/modelq
mkdir -p $OUT
run() { n=$1; shift; timeout -k 10 300 python3 bench.py --model --steps 20 --warmup 5 --no-cpu-baseline --e2e-steps 0 "$@" > $OUT/b_$n.json 2> $OUT/b_$n.err || { tail -20 $OUT/b_$n.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['value']), round(d['ms_per_step'],4), d.get('verified'), d['config'].get('hw_queues'))" $OUT/b_$n.json $n; }
for c in cfg2 cfg3; do
  run ${c}_q4 --config $c
  run ${c}_q8 --config $c --hw-queues 8
  run ${c}_q16 --config $c --hw-queues 16
  run ${c}_q16_s4 --config $c --hw-queues 16 --sets 4
  run ${c}_q24_s6 --config $c --hw-queues 24 --sets 6
done
