#!/bin/bash
# sampler lanes A/B: bench cfg2/cfg3/cfg5 with 1 and 2 sampler streams (3 and 4 sets), then the
# full-size pipeline parity tests
set -o pipefail
OUT=gpurun_out/r3
mkdir -p $OUT
for c in cfg2 cfg3 cfg5; do
  for v in "1 3" "2 3" "2 4"; do
    set -- $v
    timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --e2e-steps 0 --sampler-lanes $1 --sets $2 > $OUT/sl_${c}_$1_$2.json 2> $OUT/sl_${c}_$1_$2.err || { tail -20 $OUT/sl_${c}_$1_$2.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/sl_${c}_$1_$2.json')); print('$c lanes $1 sets $2', round(d['value']), round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms'],4))"
  done
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_a_fullsize.py -x -q -k pipeline --timeout 300 --timeout-method thread > $OUT/slanes_fullsize.log 2>&1 || { tail -40 $OUT/slanes_fullsize.log; exit 1; }
tail -1 $OUT/slanes_fullsize.log
