#!/bin/bash
# Round 4: the changed GPU tests (pipeline with per-set clouds, grouped_xyz of the multi-layer
# grouping), smoke, the driver's bench command twice and the 500-step default.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4/check
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 280 --timeout-method thread -m gpu tests/test_gpu_a_fullsize.py tests/test_gpu_fused_layers.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_drv_$i.json 2> $OUT/bench_drv_$i.err || { tail -20 $OUT/bench_drv_$i.err; exit 1; }
done
timeout -k 10 300 python3 bench.py --no-cpu-baseline --e2e-steps 0 > $OUT/bench_500.json 2> $OUT/bench_500.err || { tail -20 $OUT/bench_500.err; exit 1; }
for f in $OUT/bench_*.json; do
  python3 -c "import json,sys; d=json.load(open('$f')); print('$f', round(d['value']), round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms'],4), d['verified'], d['fault_status'], d['latency_ms_per_batch'], (d.get('verify') or {}).get('seconds'), d.get('host'))"
done
