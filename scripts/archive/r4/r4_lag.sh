#!/bin/bash
# Round 4: lag-aware cold-wave priority in the SA1 sampler (PN2_FPS_COLD_LAGPRIO=1: a cold wave
# with another group waiting outranks the ones keeping up) -- exactness, standalone time,
# round structure, pipeline; plus cfg3-shaped FP4 timings (tools/bench_nn.py).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4/lag
mkdir -p $OUT
B=pointcloud-segmentation-attention_amd/csrc/build
timeout -k 10 300 python3 tools/fps_hot_check.py --algos 0 --lib lagprio=$B/libpn2hip_v_lagprio.so --reps 30 > $OUT/hot_check.log 2>&1 || { tail -20 $OUT/hot_check.log; exit 1; }
tail -1 $OUT/hot_check.log
timeout -k 10 300 python3 tools/fps_hot_check.py --msg --algos 0 --lib lagprio=$B/libpn2hip_v_lagprio.so --reps 20 --shape 8,16384,512 > $OUT/hot_check_msg.log 2>&1 || { tail -20 $OUT/hot_check_msg.log; exit 1; }
tail -1 $OUT/hot_check_msg.log
for v in base lagprio; do
  l=tools/fps_stamp/libpn2fpsstamp.so; [ $v = lagprio ] && l=tools/fps_stamp/libpn2fpsstamp_lagprio.so
  PN2_STAMP_LIB=$l timeout -k 10 200 python3 tools/stamp_fps_cull.py --json $OUT/stamps_$v.json > $OUT/stamps_$v.log 2>&1 || { tail -20 $OUT/stamps_$v.log; exit 1; }
  PN2_STAMP_LIB=$l timeout -k 10 200 python3 tools/fps_stamp/lag_events.py > $OUT/lag_$v.log 2>&1 || { tail -20 $OUT/lag_$v.log; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/stamps_$v.json')); print('$v', d['kernel_cycles'], d['round_cycles'], d['median_round_events']['hot_end_to_last_cold'])"
  tail -1 $OUT/lag_$v.log
done
run() {  # name, lib, bench args
  n=$1; l=$2; shift 2
  PN2HIP_LIB=$l timeout -k 10 300 python3 bench.py --no-cpu-baseline --e2e-steps 0 --latency-reps 5 "$@" > $OUT/b_$n.json 2> $OUT/b_$n.err || { tail -20 $OUT/b_$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b_$n.json')); print('$n', round(d['value']), round(d['ms_per_step']*1e3,1), round(d['roofline']['avg_launch_ms'],4), d.get('verified'), round(d.get('latency_ms_per_batch',0),3))"
}
run base ""
run lagprio $B/libpn2hip_v_lagprio.so
run base2 ""
run lagprio2 $B/libpn2hip_v_lagprio.so
run drv_base "" --steps 20 --warmup 5
run drv_lagprio $B/libpn2hip_v_lagprio.so --steps 20 --warmup 5
timeout -k 10 120 python3 tools/bench_nn.py > $OUT/nn.json 2> $OUT/nn.err || { tail -20 $OUT/nn.err; exit 1; }
grep "cfg3\|fp4" $OUT/nn.json
