#!/bin/bash
# wave-cooperative three_nn: GPU suite, three_nn micro-benchmark A/B, bench lines
set -o pipefail
OUT=gpurun_out/r3/nnwave
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 280 --timeout-method thread -m gpu tests \
  > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 200 python3 tools/bench_nn.py > $OUT/bench_nn_wave.json 2>&1 || { tail -20 $OUT/bench_nn_wave.json; exit 1; }
PN2HIP_LIB=$PWD/pointcloud-segmentation-attention_amd/csrc/build/libpn2hip_nn0.so timeout -k 10 200 python3 tools/bench_nn.py > $OUT/bench_nn_nn0.json 2>&1 || { tail -20 $OUT/bench_nn_nn0.json; exit 1; }
grep -h "edge=0.0 sorted\|scan" $OUT/bench_nn_wave.json $OUT/bench_nn_nn0.json
for c in cfg2 cfg3; do
  for v in "3 6 9"; do
    set -- $v
    for only in full side; do
      D=""; [ "$only" != "full" ] && D="--diag-only $only"
      tag=${c}_$1_$2_$3_$only
      timeout -k 10 200 python3 bench.py --config $c --steps 400 --warmup 30 --no-cpu-baseline --e2e-steps 0 \
        --sampler-lanes $1 --hw-queues $2 --sets $3 $D > $OUT/b_$tag.json 2> $OUT/b_$tag.err || { tail -20 $OUT/b_$tag.err; exit 1; }
      python3 -c "import json; d=json.load(open('$OUT/b_$tag.json')); print('$tag', round(d['value']), round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms'],4))"
    done
  done
done
