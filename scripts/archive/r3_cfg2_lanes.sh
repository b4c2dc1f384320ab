#!/bin/bash
# defer2 A/B (SA1, MSG), then cfg2 bench twice and a cfg2 kernel trace (queue mapping)
set -o pipefail
OUT=gpurun_out/r3
mkdir -p $OUT
export TMPDIR=/tmp
L="--lib defer2=pointcloud-segmentation-attention_amd/csrc/build/libpn2hip_defer2.so"
timeout -k 10 300 python -u tools/fps_hot_check.py --reps 30 --algos 0 $L > $OUT/ab_defer2_sa1.log 2>&1 || { tail -30 $OUT/ab_defer2_sa1.log; exit 1; }
tail -1 $OUT/ab_defer2_sa1.log
timeout -k 10 300 python -u tools/fps_hot_check.py --msg --shape 8,16384,512 --reps 30 --algos 0 $L > $OUT/ab_defer2_msg.log 2>&1 || { tail -30 $OUT/ab_defer2_msg.log; exit 1; }
tail -1 $OUT/ab_defer2_msg.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --e2e-steps 0 > $OUT/bench_cfg2_l$i.json 2> $OUT/bench_cfg2_l$i.err || { tail -20 $OUT/bench_cfg2_l$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_cfg2_l$i.json')); print('cfg2', round(d['value']), d['ms_per_step'], d['roofline']['avg_launch_ms'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_lanes_cfg2 -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --e2e-steps 0 > $OUT/prof_lanes_cfg2.log 2>&1 || { tail -20 $OUT/prof_lanes_cfg2.log; exit 1; }
echo prof ok
