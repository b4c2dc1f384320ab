#!/bin/bash
# native plan with segment graphs: pipeline parity, then sampler lanes x hardware queues
set -o pipefail
OUT=gpurun_out/r3/planq
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 280 --timeout-method thread -m gpu \
  tests/test_gpu_a_fullsize.py -k "pipeline" > $OUT/pytest_pipeline.log 2>&1 \
  || { tail -30 $OUT/pytest_pipeline.log; exit 1; }
tail -2 $OUT/pytest_pipeline.log
for c in cfg2 cfg3 cfg5; do
  timeout -k 10 200 python3 tools/host_overhead.py --config $c --steps 100 --geometry-only --sampler-lanes 2 | tee $OUT/host_$c.json
  for v in ${VARIANTS:-"1 4" "2 4" "3 5" "3 6" "4 6" "4 8"}; do
    set -- $v
    timeout -k 10 200 python3 bench.py --config $c --steps 300 --warmup 20 --no-cpu-baseline --e2e-steps 0 \
      --sampler-lanes $1 --hw-queues $2 > $OUT/b_${c}_$1_$2.json 2> $OUT/b_${c}_$1_$2.err || { tail -20 $OUT/b_${c}_$1_$2.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/b_${c}_$1_$2.json')); print('$c lanes $1 queues $2', round(d['value']), round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms'],4))"
  done
done
