#!/bin/bash
# Round 4: samplers alone / side work alone / both (fused FP4), and the driver's 20-step
# window against the number of buffer sets (its fill + drain is ~0.6 ms of ~4 ms).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4/diag
mkdir -p $OUT
run() {  # name, bench args
  n=$1; shift
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --e2e-steps 0 --latency-reps 0 "$@" > $OUT/b_$n.json 2> $OUT/b_$n.err || { tail -20 $OUT/b_$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b_$n.json')); print('$n', round(d['value']), round(d['ms_per_step']*1e3,1), d.get('verified'))"
}
run full
run samplers --diag-only samplers --no-verify
run side --diag-only side --no-verify
run samplers_l4 --diag-only samplers --no-verify --sampler-lanes 4 --hw-queues 8 --sets 12
for s in 9 6 7 8 9 6 7 8; do run drv_s$s --steps 20 --warmup 5 --sets $s; done
run s6 --sets 6
run s7 --sets 7
