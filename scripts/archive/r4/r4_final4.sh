#!/bin/bash
# End-of-round check of the final build (after the walk's merged first pass and the radii LDS
# bound): the whole GPU suite, smoke, the driver's command twice, cfg3 and cfg5 once.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4/${FINAL_DIR:-final4}
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 280 --timeout-method thread -m gpu tests > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_drv_1.json 2> $OUT/bench_drv_1.err || { tail -20 $OUT/bench_drv_1.err; exit 1; }
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_drv_2.json 2> $OUT/bench_drv_2.err || { tail -20 $OUT/bench_drv_2.err; exit 1; }
timeout -k 10 400 python3 bench.py --steps 500 --no-cpu-baseline --e2e-steps 0 > $OUT/bench_cfg2_500.json 2> $OUT/bench_cfg2_500.err || { tail -20 $OUT/bench_cfg2_500.err; exit 1; }
timeout -k 10 400 python3 bench.py --config cfg3 --no-cpu-baseline --e2e-steps 0 > $OUT/bench_cfg3.json 2> $OUT/bench_cfg3.err || { tail -20 $OUT/bench_cfg3.err; exit 1; }
timeout -k 10 400 python3 bench.py --config cfg5 --no-cpu-baseline --e2e-steps 0 > $OUT/bench_cfg5.json 2> $OUT/bench_cfg5.err || { tail -20 $OUT/bench_cfg5.err; exit 1; }
# first use of a buffer set's graphs inside the timed window? (9 sets; warm-up 5 leaves 4 unused)
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 9 --no-cpu-baseline --e2e-steps 0 > $OUT/bench_drv_w9.json 2> $OUT/bench_drv_w9.err || { tail -20 $OUT/bench_drv_w9.err; exit 1; }
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --e2e-steps 0 > $OUT/bench_drv_w5.json 2> $OUT/bench_drv_w5.err || { tail -20 $OUT/bench_drv_w5.err; exit 1; }
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 18 --no-cpu-baseline --e2e-steps 0 > $OUT/bench_drv_w18.json 2> $OUT/bench_drv_w18.err || { tail -20 $OUT/bench_drv_w18.err; exit 1; }
for c in drv_1 drv_2 cfg2_500 cfg3 cfg5 drv_w9 drv_w5 drv_w18; do
  python3 -c "import json; d=json.load(open('$OUT/bench_$c.json')); print('$c', round(d['value']), round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms'],4), d.get('verified'), d.get('fault_status'), round(d.get('latency_ms_per_batch', 0), 3), d['roofline'].get('traffic_source'))"
done
echo done
