#!/bin/bash
# End-of-round evidence (round 6), part 1: GPU suite, smoke, the driver's command five times
# (the first with its CPU baseline and e2e fields), cfg2 at 500 steps, cfg3, cfg5, the
# side-only diagnostic. Part 2: scripts/r6_final2.sh.
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r6/final}
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 280 --timeout-method thread -m gpu tests \
  > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 500 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_drv_1.json 2> $OUT/bench_drv_1.err || { tail -20 $OUT/bench_drv_1.err; exit 1; }
for n in 2 3 4 5; do
  timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --e2e-steps 0 > $OUT/bench_drv_$n.json 2> $OUT/bench_drv_$n.err || { tail -20 $OUT/bench_drv_$n.err; exit 1; }
done
timeout -k 10 400 python3 bench.py --steps 500 --no-cpu-baseline --e2e-steps 0 > $OUT/bench_cfg2_500.json 2> $OUT/bench_cfg2.err || { tail -20 $OUT/bench_cfg2.err; exit 1; }
timeout -k 10 400 python3 bench.py --config cfg3 --no-cpu-baseline > $OUT/bench_cfg3.json 2> $OUT/bench_cfg3.err || { tail -20 $OUT/bench_cfg3.err; exit 1; }
timeout -k 10 400 python3 bench.py --config cfg5 --no-cpu-baseline --e2e-steps 0 > $OUT/bench_cfg5.json 2> $OUT/bench_cfg5.err || { tail -20 $OUT/bench_cfg5.err; exit 1; }
timeout -k 10 400 python3 bench.py --steps 500 --no-cpu-baseline --e2e-steps 0 --diag-only side > $OUT/bench_side_only.json 2> $OUT/bench_side_only.err || { tail -20 $OUT/bench_side_only.err; exit 1; }
for c in drv_1 drv_2 drv_3 drv_4 drv_5 cfg2_500 cfg3 cfg5 side_only; do
  python3 -c "import json; d=json.loads(open('$OUT/bench_$c.json').read().strip().splitlines()[-1]); print('$c', round(d['value']), round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms'],4), d.get('verified'), d.get('fault_status'), round(d.get('latency_ms_per_batch') or 0, 3), (d.get('e2e') or {}).get('value'), (d.get('cpu_baseline') or {}).get('value'))"
done
echo done
