#!/bin/bash
# Round 4: the cfg2 pipeline layout re-swept with the one-launch FP4 (side layout a-d, the
# later samplers' stream(s), queues, sets), 500 steps each.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4/sweep
mkdir -p $OUT
run() {  # name, bench args
  n=$1; shift
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --e2e-steps 0 --latency-reps 0 "$@" > $OUT/b_$n.json 2> $OUT/b_$n.err || { tail -20 $OUT/b_$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b_$n.json')); print('$n', round(d['value']), round(d['ms_per_step']*1e3,1), d.get('verified'))"
}
run default
run la --side-layout a --hw-queues 6
run lc --side-layout c
run ld --side-layout d --hw-queues 8
run own2 --chain own2 --hw-queues 8
run behind --chain behind --hw-queues 6
run s7 --sets 7
run q8 --hw-queues 8
run default2
run la2 --side-layout a --hw-queues 6
run lc2 --side-layout c
