#!/bin/bash
# Round 4 start: the driver's bench command three times and the 500-step default, on the
# round-3 code (the reference point for this round's changes).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4/start
mkdir -p $OUT
for i in 1 2 3; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --e2e-steps 0 > $OUT/bench_drv_$i.json 2> $OUT/bench_drv_$i.err || { tail -20 $OUT/bench_drv_$i.err; exit 1; }
done
timeout -k 10 300 python3 bench.py --no-cpu-baseline --e2e-steps 0 > $OUT/bench_500.json 2> $OUT/bench_500.err || { tail -20 $OUT/bench_500.err; exit 1; }
for f in $OUT/bench_*.json; do
  python3 -c "import json,sys; d=json.load(open('$f')); print('$f', round(d['value']), round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms'],4), d.get('host'))"
done
