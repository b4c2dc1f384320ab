#!/bin/bash
# Round 6: interleaved A/B of bench.py argument sets (ARGS_A, ARGS_B, ... and environments
# ENV_A, ...: named by ABS, each run REPS times, STEPS steps), then their values.
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r6/ab}
mkdir -p $OUT
for r in $(seq 1 ${REPS:-2}); do
  for n in ${ABS:-A B}; do
    v="ARGS_$n"; e="ENV_$n"
    env ${!e} timeout -k 10 300 python3 bench.py --steps ${STEPS:-500} --no-cpu-baseline --e2e-steps 0 ${!v} > $OUT/ab_${n}_$r.json 2> $OUT/ab_${n}_$r.err || { tail -20 $OUT/ab_${n}_$r.err; exit 1; }
  done
done
for f in $OUT/ab_*.json; do
  python3 -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', round(d['value']), round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms'],4), d.get('verified'))"
done
