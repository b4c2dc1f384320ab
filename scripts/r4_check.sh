#!/bin/bash
# Round 4: the changed GPU tests (pipeline with per-set clouds, grouped_xyz of the multi-layer
# grouping, grid builds / flattened grid query), micro-benchmarks with A/B builds (grid query
# row loop vs flattened; grouping U = 4 / 8 / 16), the driver's bench command twice, the
# 500-step default, cfg5.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4/check
mkdir -p $OUT
B=pointcloud-segmentation-attention_amd/csrc/build
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 280 --timeout-method thread -m gpu tests/test_gpu_a_fullsize.py tests/test_gpu_fused_layers.py tests/test_gpu_parity.py -k "fps or chain or grid or ball or pipeline or stack or golden or group" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 120 python3 tools/bench_msg_grid.py > $OUT/msg_grid_flat.json 2>&1 || { tail -20 $OUT/msg_grid_flat.json; exit 1; }
PN2HIP_LIB=$B/libpn2hip_v_gqrows.so timeout -k 10 120 python3 tools/bench_msg_grid.py > $OUT/msg_grid_rows.json 2>&1 || { tail -20 $OUT/msg_grid_rows.json; exit 1; }
paste $OUT/msg_grid_flat.json $OUT/msg_grid_rows.json
PN2HIP_LIB=$B/libpn2hip_sg_vec.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_fused_layers.py -k ball_group_layers > $OUT/pytest_sgvec.log 2>&1 || { tail -30 $OUT/pytest_sgvec.log; exit 1; }
tail -1 $OUT/pytest_sgvec.log
for v in main u8 u16 vec vecu8; do
  L=""; [ $v != main ] && L=$B/libpn2hip_sg_$v.so
  PN2HIP_LIB=$L timeout -k 10 120 python3 tools/bench_layers.py > $OUT/layers_$v.json 2>&1 || { tail -20 $OUT/layers_$v.json; exit 1; }
  echo $v; cat $OUT/layers_$v.json
done
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
timeout -k 10 120 python3 tools/bench_chain.py > $OUT/chain_wc1.json 2>&1 || { tail -20 $OUT/chain_wc1.json; exit 1; }
PN2HIP_LIB=$B/libpn2hip_v_wc0.so timeout -k 10 120 python3 tools/bench_chain.py > $OUT/chain_wc0.json 2>&1 || { tail -20 $OUT/chain_wc0.json; exit 1; }
cat $OUT/chain_wc1.json $OUT/chain_wc0.json
for v in cb128 cb512; do
  PN2HIP_LIB=$B/libpn2hip_v_$v.so timeout -k 10 120 python3 tools/bench_chain.py > $OUT/chain_$v.json 2>&1 || { tail -20 $OUT/chain_$v.json; exit 1; }
  echo $v; cat $OUT/chain_$v.json
done
for v in main gcu8 gcu8t4k gcu16t4k; do
  L=""; [ $v != main ] && L=$B/libpn2hip_v_$v.so
  PN2HIP_LIB=$L timeout -k 10 120 python3 tools/bench_group.py > $OUT/group_$v.json 2>&1 || { tail -20 $OUT/group_$v.json; exit 1; }
  echo $v; cat $OUT/group_$v.json
done
