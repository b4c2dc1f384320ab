#!/bin/bash
# lane 3 for attention (cfg3) / MSG radius 2 (cfg5) with several sampler lanes
set -o pipefail
OUT=gpurun_out/r3/lane3
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 280 --timeout-method thread -m gpu \
  tests/test_gpu_a_fullsize.py -k "pipeline" > $OUT/pytest_pipeline.log 2>&1 \
  || { tail -30 $OUT/pytest_pipeline.log; exit 1; }
tail -2 $OUT/pytest_pipeline.log
for c in ${CONFIGS:-cfg3 cfg5 cfg2}; do
  for v in ${VARIANTS:-"2 5 6" "3 6 9" "3 7 9" "4 7 8"}; do
    set -- $v
    tag=${c}_$1_$2_$3
    timeout -k 10 200 python3 bench.py --config $c --steps 400 --warmup 30 --no-cpu-baseline --e2e-steps 0 \
      --sampler-lanes $1 --hw-queues $2 --sets $3 > $OUT/b_$tag.json 2> $OUT/b_$tag.err || { tail -20 $OUT/b_$tag.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/b_$tag.json')); print('$tag', round(d['value']), round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms'],4))"
  done
done
