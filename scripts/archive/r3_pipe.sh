#!/bin/bash
# parity of the fused layers + full-size steps, the layers micro-bench, bench lines
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r3/${TAG:-pipe}
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_fused_layers.py tests/test_gpu_a_fullsize.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 200 python3 tools/bench_layers.py --json $OUT/layers.json || exit 1
for c in ${CONFIGS:-cfg2 cfg3}; do
  for rep in 1 2; do
  timeout -k 10 300 python3 bench.py --config $c --no-cpu-baseline --e2e-steps 0 ${BENCH_ARGS:-} > $OUT/bench_${c}_$rep.json 2> $OUT/bench_$c.err || { tail -20 $OUT/bench_$c.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_${c}_$rep.json')); print('$c', round(d['value']), round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms'],4), d['config']['streams'][:40])"
  done
  for m in side samplers; do
  timeout -k 10 300 python3 bench.py --config $c --no-cpu-baseline --e2e-steps 0 --diag-only $m ${BENCH_ARGS:-} > $OUT/${m}_$c.json 2> $OUT/${m}_$c.err || { tail -20 $OUT/${m}_$c.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/${m}_$c.json')); print('$c $m-only', round(d['value']), round(d['ms_per_step'],4))"
  done
done
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_driver.json 2> $OUT/bench_driver.err || { tail -20 $OUT/bench_driver.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench_driver.json')); print('driver-cmd', round(d['value']), round(d['ms_per_step'],4))"
