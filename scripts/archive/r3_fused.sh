#!/bin/bash
# fused multi-layer launches: parity, then the default bench lines + a kernel trace
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r3/${TAG:-fused}
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_fused_layers.py tests/test_gpu_a_fullsize.py > $OUT/pytest_fused.log 2>&1 || { tail -30 $OUT/pytest_fused.log; exit 1; }
tail -1 $OUT/pytest_fused.log
for c in ${CONFIGS:-cfg2 cfg3}; do
  timeout -k 10 300 python3 bench.py --config $c --no-cpu-baseline --e2e-steps 0 ${BENCH_ARGS:-} > $OUT/bench_$c.json 2> $OUT/bench_$c.err || { tail -20 $OUT/bench_$c.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_$c.json')); print('$c', round(d['value']), round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms'],4))"
  timeout -k 10 300 python3 bench.py --config $c --no-cpu-baseline --e2e-steps 0 --diag-only side ${BENCH_ARGS:-} > $OUT/side_$c.json 2> $OUT/side_$c.err || { tail -20 $OUT/side_$c.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/side_$c.json')); print('$c side-only', round(d['value']), round(d['ms_per_step'],4))"
done
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_driver.json 2> $OUT/bench_driver.err || { tail -20 $OUT/bench_driver.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench_driver.json')); print('driver-cmd', round(d['value']), round(d['ms_per_step'],4))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_cfg2 -o run -- python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --e2e-steps 0 > $OUT/prof_cfg2.json 2> $OUT/prof_cfg2.err || { tail -20 $OUT/prof_cfg2.err; exit 1; }
echo done
