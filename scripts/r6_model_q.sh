#!/bin/bash
# Whole-model step: hardware queues x buffer sets sweep (bench.py --model, 20 steps), cfg2 and
# cfg3, now that lane 1 carries only the MLP kernels.
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r6/model_q}
mkdir -p $OUT
for c in ${CFGS:-cfg2 cfg3}; do
  for q in ${QS:-4 6 8}; do
    for s in ${SETS:-3 4}; do
      f=$OUT/${c}_q${q}_s${s}.json
      timeout -k 10 300 python3 bench.py --model --config $c --hw-queues $q --sets $s --no-cpu-baseline > $f 2> $f.err || { tail -20 $f.err; exit 1; }
      python3 -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$c q$q s$s', round(d['value']), round(d['ms_per_step'], 4))"
    done
  done
done
