#!/bin/bash
# Round 4: what limits the step period once FP4 is one launch -- per-task marginal costs
# again, the timeline's per-lane lags, more sampler lanes.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4/lim
mkdir -p $OUT
run() {  # name, bench args
  n=$1; shift
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --e2e-steps 0 --latency-reps 0 "$@" > $OUT/b_$n.json 2> $OUT/b_$n.err || { tail -20 $OUT/b_$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b_$n.json')); print('$n', round(d['value']), round(d['ms_per_step']*1e3,1), d['verified'])"
}
run default
for t in grid1 sa1 sa234 fp4 fp123; do export PN2_DUP_TASKS=$t; run dup_$t; done; unset PN2_DUP_TASKS
run l4 --sampler-lanes 4 --hw-queues 8 --sets 12
run l4s16 --sampler-lanes 4 --hw-queues 8 --sets 16
run l3s12 --sets 12
run l2 --sampler-lanes 2 --hw-queues 6
timeout -k 10 300 python3 bench.py --no-cpu-baseline --e2e-steps 0 --latency-reps 0 --steps 300 --timeline $OUT/timeline.json > $OUT/b_tl.json 2> $OUT/b_tl.err || { tail -20 $OUT/b_tl.err; exit 1; }
python3 tools/timeline_report.py $OUT/timeline.json --show 0 --lanes
