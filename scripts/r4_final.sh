#!/bin/bash
# End-of-round evidence (round 4): GPU suite, smoke, bench lines (cfg2 default + the driver's
# command, cfg3, cfg5), rocprofv3 kernel stats per config, the cfg2 critical path and lane
# report from that trace, PMC HBM traffic (one counter per pass).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4/final
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 280 --timeout-method thread -m gpu tests \
  > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_cfg2_driver_cmd.json 2> $OUT/bench_d.err || { tail -20 $OUT/bench_d.err; exit 1; }
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_cfg2_driver_cmd2.json 2> $OUT/bench_d2.err || { tail -20 $OUT/bench_d2.err; exit 1; }
timeout -k 10 400 python3 bench.py --steps 500 --no-cpu-baseline > $OUT/bench_cfg2_500.json 2> $OUT/bench_cfg2.err || { tail -20 $OUT/bench_cfg2.err; exit 1; }
timeout -k 10 400 python3 bench.py --config cfg3 --no-cpu-baseline > $OUT/bench_cfg3.json 2> $OUT/bench_cfg3.err || { tail -20 $OUT/bench_cfg3.err; exit 1; }
timeout -k 10 400 python3 bench.py --config cfg5 --no-cpu-baseline --e2e-steps 0 > $OUT/bench_cfg5.json 2> $OUT/bench_cfg5.err || { tail -20 $OUT/bench_cfg5.err; exit 1; }
for c in cfg2_driver_cmd cfg2_driver_cmd2 cfg2_500 cfg3 cfg5; do
  python3 -c "import json; d=json.load(open('$OUT/bench_$c.json')); print('$c', round(d['value']), round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms'],4), d.get('verified'), d.get('fault_status'), round(d.get('latency_ms_per_batch', 0), 3), (d.get('e2e') or {}).get('value'), (d.get('cpu_baseline') or {}).get('value'))"
done
for c in cfg2 cfg3 cfg5; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$c -o run -- python3 bench.py --config $c --steps 200 --warmup 20 --no-cpu-baseline --e2e-steps 0 --latency-reps 0 --no-verify > $OUT/prof_$c.json 2> $OUT/prof_$c.err || { tail -20 $OUT/prof_$c.err; exit 1; }
done
T=$(ls $OUT/prof_cfg2/*/run_kernel_trace.csv 2>/dev/null | head -1)
[ -n "$T" ] || T=$(find $OUT/prof_cfg2 -name "*kernel_trace.csv" | head -1)
python3 tools/critical_path.py "$T" > $OUT/critical_path_cfg2.txt || exit 1
python3 tools/lane_report.py "$T" > $OUT/lanes_cfg2.txt || exit 1
for cb in cfg2:16 cfg3:16 cfg5:8; do
  c=${cb%%:*}; b=${cb##*:}
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $OUT/pmc_${C}_$c -o run -- python3 bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline --e2e-steps 0 --latency-reps 0 --no-verify > $OUT/pmc_${C}_$c.log 2>&1 || { tail -5 $OUT/pmc_${C}_$c.log; exit 1; }
  done
  python3 tools/pmc_summary.py $OUT/pmc_FETCH_SIZE_$c $OUT/pmc_WRITE_SIZE_$c > $OUT/pmc_traffic_${c}_B$b.json || exit 1
done
echo done
