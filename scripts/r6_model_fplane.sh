#!/bin/bash
# Whole-model step A/B: the FP MLP chain on lane 1 behind the SA chain (default) or on a lane of
# its own (lane 5), so one step's FP layers can overlap the next step's SA layers.
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r6/model_fplane}
mkdir -p $OUT
PN2_MODEL_FP_LANE=5 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_model.py > $OUT/pytest_model.log 2>&1 || { tail -30 $OUT/pytest_model.log; exit 1; }
tail -1 $OUT/pytest_model.log
for n in 1 2; do
 for lane in 1 5; do
  for q in 4 5 6; do
   [ $lane = 1 ] && [ $q != 4 ] && continue
   for c in cfg2 cfg3; do
    f=$OUT/${c}_l${lane}_q${q}_$n.json
    PN2_MODEL_FP_LANE=$lane timeout -k 10 300 python3 bench.py --model --config $c --hw-queues $q --no-cpu-baseline > $f 2> $f.err || { tail -20 $f.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$c lane$lane q$q', $n, round(d['value']), round(d['ms_per_step'], 4))"
   done
  done
 done
done
