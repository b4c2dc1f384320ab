#!/bin/bash
# native plan executor: pipeline parity (poisoned buffers, 1/2 sampler lanes), then bench lines
# with 1-3 sampler lanes and the host cost of one step's enqueue
set -o pipefail
OUT=gpurun_out/r3/plan
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 280 --timeout-method thread -m gpu \
  tests/test_gpu_a_fullsize.py -k "pipeline" > $OUT/pytest_pipeline.log 2>&1 \
  || { tail -30 $OUT/pytest_pipeline.log; exit 1; }
tail -3 $OUT/pytest_pipeline.log
for c in cfg2 cfg3 cfg5; do
  for l in ${LANES:-1 2 3}; do
    timeout -k 10 200 python3 bench.py --config $c --steps 200 --warmup 20 --no-cpu-baseline --e2e-steps 0 \
      --sampler-lanes $l > $OUT/b_${c}_$l.json 2> $OUT/b_${c}_$l.err || { tail -20 $OUT/b_${c}_$l.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/b_${c}_$l.json')); print('$c lanes $l', round(d['value']), round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms'],4))"
  done
  timeout -k 10 200 python3 tools/host_overhead.py --config $c --steps 100 --geometry-only --sampler-lanes 2 | tee $OUT/host_$c.json
done
