#!/bin/bash
# Round 5: one, two or three chain streams (the SA2-4 samplers) beside three sampler streams,
# at the driver's 20 steps (interleaved, twice) and at 500 steps.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r5/chains
mkdir -p $OUT
run() { n=$1; shift; timeout -k 10 300 python3 bench.py --no-cpu-baseline --e2e-steps 0 --no-verify "$@" > $OUT/b_$n.json 2> $OUT/b_$n.err || { tail -20 $OUT/b_$n.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/b_$n.json')); print('$n', round(d['value']), round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms'],4), d['config']['hw_queues'])"; }
for i in 1 2 3; do
run d_own_$i --steps 20 --warmup 5
run d_own3_$i --steps 20 --warmup 5 --chain own3 --hw-queues 9
run d_own2_$i --steps 20 --warmup 5 --chain own2 --hw-queues 8
done
run own3 --steps 500 --chain own3 --hw-queues 9
run own --steps 500
echo done
