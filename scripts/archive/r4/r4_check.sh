#!/bin/bash
# Round 4: the changed GPU tests (pipeline with per-set clouds, grouped_xyz of the multi-layer
# grouping, grid builds / flattened grid query, samplers), the driver's bench command twice,
# the 500-step default, cfg5, side work alone, a kernel trace with its critical path.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4/check
mkdir -p $OUT
B=pointcloud-segmentation-attention_amd/csrc/build
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 280 --timeout-method thread -m gpu tests/test_gpu_a_fullsize.py tests/test_gpu_fused_layers.py tests/test_gpu_parity.py -k "fps or chain or grid or ball or pipeline or stack or golden or group" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_drv_$i.json 2> $OUT/bench_drv_$i.err || { tail -20 $OUT/bench_drv_$i.err; exit 1; }
done
timeout -k 10 300 python3 bench.py --no-cpu-baseline --e2e-steps 0 > $OUT/bench_500.json 2> $OUT/bench_500.err || { tail -20 $OUT/bench_500.err; exit 1; }
timeout -k 10 300 python3 bench.py --config cfg5 --no-cpu-baseline --e2e-steps 0 > $OUT/bench_cfg5.json 2> $OUT/bench_cfg5.err || { tail -20 $OUT/bench_cfg5.err; exit 1; }
timeout -k 10 300 python3 bench.py --no-cpu-baseline --e2e-steps 0 --diag-only side --steps 200 > $OUT/bench_side.json 2> $OUT/bench_side.err || { tail -20 $OUT/bench_side.err; exit 1; }
for f in $OUT/bench_*.json; do
  python3 -c "import json,sys; d=json.load(open('$f')); print('$f', round(d['value']), round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms'],4), d['verified'], d['fault_status'], d['latency_ms_per_batch'], (d.get('verify') or {}).get('seconds'), d.get('host'))" || true
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace_cfg2 -o run -- python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --e2e-steps 0 --no-verify --latency-reps 0 > $OUT/trace_cfg2.log 2>&1 || { tail -20 $OUT/trace_cfg2.log; exit 1; }
T=$(find $OUT/trace_cfg2 -name "*kernel_trace.csv" | head -1)
python3 tools/critical_path.py $T --out $OUT/critical_path_cfg2.txt | head -8
python3 tools/lane_report.py $T > $OUT/lanes_cfg2.txt; head -30 $OUT/lanes_cfg2.txt
