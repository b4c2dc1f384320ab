#!/bin/bash
# Round 4 A/B: micro-benchmarks of alternative builds (grid query row loop vs flattened,
# grouping in-flight depth / vector write phase, group_concat tiles, chain block size and
# winner coordinates) and a cfg2 layout sweep (second chain stream, four sampler streams).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4/ab
mkdir -p $OUT
B=pointcloud-segmentation-attention_amd/csrc/build
run() {  # name, bench args
  n=$1; shift
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --e2e-steps 0 "$@" > $OUT/b_$n.json 2> $OUT/b_$n.err || { tail -20 $OUT/b_$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b_$n.json')); print('$n', round(d['value']), round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms'],4), d['verified'], d['latency_ms_per_batch'], d['host'])"
}
run default
run cup64 --cu-partition 64
run cup80 --cu-partition 80
run cup96 --cu-partition 96
run l4cup80 --sampler-lanes 4 --hw-queues 8 --sets 12 --cu-partition 80
run own2cup80 --chain own2 --hw-queues 8 --cu-partition 80
run drv_default --steps 20 --warmup 5
run drv_cup64 --steps 20 --warmup 5 --cu-partition 64
run drv_cup80 --steps 20 --warmup 5 --cu-partition 80
PN2HIP_LIB=$B/libpn2hip_sg_vec.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_fused_layers.py -k ball_group_layers > $OUT/pytest_sgvec.log 2>&1 || { tail -30 $OUT/pytest_sgvec.log; exit 1; }
tail -1 $OUT/pytest_sgvec.log
timeout -k 10 120 python3 tools/bench_msg_grid.py > $OUT/msg_grid_flat.json 2>&1 || { tail -20 $OUT/msg_grid_flat.json; exit 1; }
PN2HIP_LIB=$B/libpn2hip_v_gqrows.so timeout -k 10 120 python3 tools/bench_msg_grid.py > $OUT/msg_grid_rows.json 2>&1 || { tail -20 $OUT/msg_grid_rows.json; exit 1; }
paste $OUT/msg_grid_flat.json $OUT/msg_grid_rows.json
for v in main u8 u16 vec vecu8; do
  L=""; [ $v != main ] && L=$B/libpn2hip_sg_$v.so
  PN2HIP_LIB=$L timeout -k 10 120 python3 tools/bench_layers.py > $OUT/layers_$v.json 2>&1 || { tail -20 $OUT/layers_$v.json; exit 1; }
  echo $v; tail -1 $OUT/layers_$v.json
done
for v in main wc0 cb128 cb512; do
  L=""; [ $v != main ] && L=$B/libpn2hip_v_$v.so
  PN2HIP_LIB=$L timeout -k 10 120 python3 tools/bench_chain.py > $OUT/chain_$v.json 2>&1 || { tail -20 $OUT/chain_$v.json; exit 1; }
  echo $v; tail -1 $OUT/chain_$v.json
done
for v in main gcu8 gcu8t4k gcu16t4k; do
  L=""; [ $v != main ] && L=$B/libpn2hip_v_$v.so
  PN2HIP_LIB=$L timeout -k 10 120 python3 tools/bench_group.py > $OUT/group_$v.json 2>&1 || { tail -20 $OUT/group_$v.json; exit 1; }
  echo $v; tail -1 $OUT/group_$v.json
done
