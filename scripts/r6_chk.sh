#!/bin/bash
# Round 6 build check: focused GPU tests (TESTS=...), the pipeline stress (ROT rotations), the
# driver's command NDRV times, cfg2 at 500 steps, cfg3, cfg5. Every GPU step has its own time
# limit and the first failure ends the script.
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r6/chk}
mkdir -p $OUT
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-900} python3 -u -m pytest -x -v -rP --timeout 280 --timeout-method thread -m gpu $TESTS \
    > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
  grep -E 'passed|failed|torn reads' $OUT/pytest_gpu.log | tail -5
fi
if [ -n "${ROT:-}" ]; then
  timeout -k 10 600 python3 -u tools/pipe_stress.py --rotations $ROT > $OUT/pipe_stress.json 2> $OUT/pipe_stress.err \
    || { tail -20 $OUT/pipe_stress.err; exit 1; }
  tail -2 $OUT/pipe_stress.json
fi
[ -n "${NOBENCH:-}" ] && exit 0
for n in $(seq 1 ${NDRV:-3}); do
  timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --e2e-steps 0 > $OUT/bench_drv_$n.json 2> $OUT/bench_drv_$n.err || { tail -20 $OUT/bench_drv_$n.err; exit 1; }
done
timeout -k 10 400 python3 bench.py --steps 500 --no-cpu-baseline --e2e-steps 0 > $OUT/bench_cfg2_500.json 2> $OUT/bench_cfg2.err || { tail -20 $OUT/bench_cfg2.err; exit 1; }
timeout -k 10 400 python3 bench.py --config cfg3 --no-cpu-baseline --e2e-steps 0 > $OUT/bench_cfg3.json 2> $OUT/bench_cfg3.err || { tail -20 $OUT/bench_cfg3.err; exit 1; }
timeout -k 10 400 python3 bench.py --config cfg5 --no-cpu-baseline --e2e-steps 0 > $OUT/bench_cfg5.json 2> $OUT/bench_cfg5.err || { tail -20 $OUT/bench_cfg5.err; exit 1; }
for c in $(seq -f 'drv_%g' 1 ${NDRV:-3}) cfg2_500 cfg3 cfg5; do
  python3 -c "import json; d=json.loads(open('$OUT/bench_$c.json').read().strip().splitlines()[-1]); print('$c', round(d['value']), round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms'],4), d.get('verified'), d.get('fault_status'), round(d.get('latency_ms_per_batch') or 0, 3))"
done
