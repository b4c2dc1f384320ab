#!/bin/bash
# Round 4: marginal cost of each side task in the pipelined cfg2 step -- the task runs twice
# in its graph (PN2_DUP_TASKS, same results), the step time difference is what one more copy
# costs beside everything else.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4/dup
mkdir -p $OUT
run() {  # name, dup list, bench args
  n=$1; d=$2; shift 2
  PN2_DUP_TASKS=$d timeout -k 10 300 python3 bench.py --no-cpu-baseline --e2e-steps 0 --latency-reps 0 "$@" > $OUT/b_$n.json 2> $OUT/b_$n.err || { tail -20 $OUT/b_$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b_$n.json')); print('$n', round(d['value']), round(d['ms_per_step']*1e3,1), d['verified'])"
}
run default ""
run grid1 grid1
run sa1 sa1
run sa234 sa234
run fp4 fp4
run fp123 fp123
run default2 ""
run c3_default "" --config cfg3
for t in sa1 sa234 fp4 fp123 att1; do run c3_$t $t --config cfg3; done
