#!/bin/bash
# Round 4 A/B 2: the new defaults (vector write phase of the multi-layer grouping incl. split
# queries, hybrid grid-query walk, chain without carried coordinates) checked bit-exact, their
# micro-benchmarks against A/B builds, and high-priority sampler streams.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4/ab2
mkdir -p $OUT
B=pointcloud-segmentation-attention_amd/csrc/build
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 280 --timeout-method thread -m gpu tests/test_gpu_a_fullsize.py tests/test_gpu_fused_layers.py -k "stack or ball_group or grid or pipeline" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
run() {  # name, bench args
  n=$1; shift
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --e2e-steps 0 "$@" > $OUT/b_$n.json 2> $OUT/b_$n.err || { tail -20 $OUT/b_$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b_$n.json')); print('$n', round(d['value']), round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms'],4), d['verified'], round(d['latency_ms_per_batch'],3), d['host'])"
}
run default
run prio --sampler-priority high
run prio_own2 --sampler-priority high --chain own2 --hw-queues 8
run prio_l4 --sampler-priority high --sampler-lanes 4 --hw-queues 8 --sets 12
run drv_default --steps 20 --warmup 5
run drv_prio --steps 20 --warmup 5 --sampler-priority high
run cfg5 --config cfg5
run cfg5_prio --config cfg5 --sampler-priority high
run cfg3 --config cfg3
run cfg3_prio --config cfg3 --sampler-priority high
for v in main vec0; do
  L=""; [ $v != main ] && L=$B/libpn2hip_sg_$v.so
  PN2HIP_LIB=$L timeout -k 10 120 python3 tools/bench_layers.py > $OUT/layers_$v.json 2>&1 || { tail -20 $OUT/layers_$v.json; exit 1; }
  echo $v; tail -1 $OUT/layers_$v.json
done
for v in main gqrows gqlr16 gqlr48; do
  L=""; [ $v != main ] && L=$B/libpn2hip_v_$v.so
  PN2HIP_LIB=$L timeout -k 10 120 python3 tools/bench_msg_grid.py > $OUT/msg_grid_$v.json 2>&1 || { tail -20 $OUT/msg_grid_$v.json; exit 1; }
done
paste $OUT/msg_grid_main.json $OUT/msg_grid_gqrows.json $OUT/msg_grid_gqlr16.json $OUT/msg_grid_gqlr48.json | cut -c1-240
timeout -k 10 120 python3 tools/bench_chain.py > $OUT/chain_main.json 2>&1 || { tail -20 $OUT/chain_main.json; exit 1; }
tail -1 $OUT/chain_main.json
