#!/bin/bash
# Round 4: the later samplers' chain lane at high stream priority (PN2_CHAIN_PRIO=1), the SA1
# sampler streams and side lanes at normal priority.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4/cprio
mkdir -p $OUT
run() {  # name, bench args
  n=$1; shift
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --e2e-steps 0 --latency-reps 5 "$@" > $OUT/b_$n.json 2> $OUT/b_$n.err || { tail -20 $OUT/b_$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b_$n.json')); print('$n', round(d['value']), round(d['ms_per_step']*1e3,1), d.get('verified'), round(d.get('latency_ms_per_batch',0),3))"
}
run base
export PN2_CHAIN_PRIO=1; run cprio; unset PN2_CHAIN_PRIO
run drv_base --steps 20 --warmup 5
export PN2_CHAIN_PRIO=1; run drv_cprio --steps 20 --warmup 5; unset PN2_CHAIN_PRIO
run base2
export PN2_CHAIN_PRIO=1; run cprio2; unset PN2_CHAIN_PRIO
run drv_base2 --steps 20 --warmup 5
export PN2_CHAIN_PRIO=1; run drv_cprio2 --steps 20 --warmup 5; unset PN2_CHAIN_PRIO
export PN2_CHAIN_PRIO=1; run cfg3_cprio --config cfg3; unset PN2_CHAIN_PRIO
run cfg3_base --config cfg3
