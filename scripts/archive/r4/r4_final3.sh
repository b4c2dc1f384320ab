#!/bin/bash
# End-of-round evidence (round 4), part 3 (after MSG SA1's one-launch radii): cfg5's bench
# line, kernel stats and traffic again; the driver's command three more times (its spread).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4/final3
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 280 --timeout-method thread -m gpu tests/test_gpu_a_fullsize.py tests/test_gpu_fused_layers.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 400 python3 bench.py --config cfg5 --no-cpu-baseline --e2e-steps 0 > $OUT/bench_cfg5.json 2> $OUT/bench_cfg5.err || { tail -20 $OUT/bench_cfg5.err; exit 1; }
timeout -k 10 400 python3 bench.py --config cfg5 --steps 20 --warmup 5 --no-cpu-baseline --e2e-steps 0 > $OUT/bench_cfg5_20.json 2> $OUT/bench_cfg5_20.err || { tail -20 $OUT/bench_cfg5_20.err; exit 1; }
for i in 1 2 3; do
  timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_drv_$i.json 2> $OUT/bench_drv_$i.err || { tail -20 $OUT/bench_drv_$i.err; exit 1; }
done
for c in cfg5 cfg5_20 drv_1 drv_2 drv_3; do
  python3 -c "import json; d=json.load(open('$OUT/bench_$c.json')); print('$c', round(d['value']), round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms'],4), d.get('verified'), d.get('fault_status'), round(d.get('latency_ms_per_batch', 0), 3))"
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_cfg5 -o run -- python3 bench.py --config cfg5 --steps 200 --warmup 20 --no-cpu-baseline --e2e-steps 0 --latency-reps 0 --no-verify > $OUT/prof_cfg5.json 2> $OUT/prof_cfg5.err || { tail -20 $OUT/prof_cfg5.err; exit 1; }
find $OUT -name "*kernel_trace.csv" -delete
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $OUT/pmc_${C}_cfg5 -o run -- python3 bench.py --config cfg5 --steps 5 --warmup 2 --no-cpu-baseline --e2e-steps 0 --latency-reps 0 --no-verify > $OUT/pmc_${C}_cfg5.log 2>&1 || { tail -5 $OUT/pmc_${C}_cfg5.log; exit 1; }
done
python3 tools/pmc_summary.py $OUT/pmc_FETCH_SIZE_cfg5 $OUT/pmc_WRITE_SIZE_cfg5 > $OUT/pmc_traffic_cfg5_B8.json || exit 1
rm -rf $OUT/pmc_FETCH_SIZE_cfg5 $OUT/pmc_WRITE_SIZE_cfg5
du -sh $OUT
echo done
