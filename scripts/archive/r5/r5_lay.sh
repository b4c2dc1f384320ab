#!/bin/bash
# Round 5: sampler streams x chain streams, full step and the halves alone (500 steps), and the
# driver's 20 steps.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r5/lay
mkdir -p $OUT
run() { n=$1; shift; timeout -k 10 300 python3 bench.py --no-cpu-baseline --e2e-steps 0 --no-verify "$@" > $OUT/b_$n.json 2> $OUT/b_$n.err || { tail -20 $OUT/b_$n.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/b_$n.json')); print('$n', round(d['value']), round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms'],4), d['config']['hw_queues'])"; }
run l3 --steps 500
run l3own2 --steps 500 --chain own2 --hw-queues 8
run l4own2 --steps 500 --chain own2 --sampler-lanes 4 --hw-queues 9
run l4own2_samp --steps 500 --chain own2 --sampler-lanes 4 --hw-queues 9 --diag-only samplers
run l3own2_samp --steps 500 --chain own2 --hw-queues 8 --diag-only samplers
run l5own2_samp --steps 500 --chain own2 --sampler-lanes 5 --hw-queues 10 --diag-only samplers
run l4own2_side --steps 500 --chain own2 --sampler-lanes 4 --hw-queues 9 --diag-only side
run d_l3 --steps 20 --warmup 5
run d_l4own2 --steps 20 --warmup 5 --chain own2 --sampler-lanes 4 --hw-queues 9
run d_l3 --steps 20 --warmup 5
run d_l4own2 --steps 20 --warmup 5 --chain own2 --sampler-lanes 4 --hw-queues 9
echo done
