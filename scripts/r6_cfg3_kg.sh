#!/bin/bash
# cfg3: FP4's known grid built on FP4's lane (the default) or by the SA1 sampler's workgroups,
# at 500 steps and with the driver's 20-step window, interleaved REP times (all verified).
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r6/cfg3_kg}
mkdir -p $OUT
for n in $(seq 1 ${REP:-3}); do
  for m in lane sampler; do
    for st in 500 20; do
      f=$OUT/cfg3_${m}_s${st}_$n.json
      timeout -k 10 300 python3 bench.py --config cfg3 --steps $st --warmup 5 --fp4-known-grid $m --no-cpu-baseline --e2e-steps 0 > $f 2> $f.err || { tail -20 $f.err; exit 1; }
      python3 -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('cfg3 $m s$st $n', round(d['value']), d.get('verified'))"
    done
  done
done
