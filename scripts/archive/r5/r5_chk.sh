#!/bin/bash
# Round 5: a build check -- the GPU suite, then the driver's command three times, cfg2 at 500
# steps, cfg3, cfg5 (value, ms/step, sampler launch ms, verified, fault status, latency).
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r5/chk}
mkdir -p $OUT
if [ -z "$NOSUITE" ]; then
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 280 --timeout-method thread -m gpu tests \
  > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
fi
for n in 1 2 3; do
  timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --e2e-steps 0 > $OUT/bench_drv_$n.json 2> $OUT/bench_drv_$n.err || { tail -20 $OUT/bench_drv_$n.err; exit 1; }
done
timeout -k 10 400 python3 bench.py --steps 500 --no-cpu-baseline --e2e-steps 0 > $OUT/bench_cfg2_500.json 2> $OUT/bench_cfg2.err || { tail -20 $OUT/bench_cfg2.err; exit 1; }
timeout -k 10 400 python3 bench.py --config cfg3 --no-cpu-baseline --e2e-steps 0 > $OUT/bench_cfg3.json 2> $OUT/bench_cfg3.err || { tail -20 $OUT/bench_cfg3.err; exit 1; }
timeout -k 10 400 python3 bench.py --config cfg5 --no-cpu-baseline --e2e-steps 0 > $OUT/bench_cfg5.json 2> $OUT/bench_cfg5.err || { tail -20 $OUT/bench_cfg5.err; exit 1; }
for c in drv_1 drv_2 drv_3 cfg2_500 cfg3 cfg5; do
  python3 -c "import json; d=json.loads(open('$OUT/bench_$c.json').read().strip().splitlines()[-1]); print('$c', round(d['value']), round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms'],4), d.get('verified'), d.get('fault_status'), round(d.get('latency_ms_per_batch') or 0, 3))"
done
