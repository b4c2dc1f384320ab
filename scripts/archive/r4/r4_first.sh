#!/bin/bash
# Round 4: the grid three_nn walk's first pass as the whole 3x3x3 block (shells 0 and 1, one
# merge and test) against shell 0 alone first (first0), and the fused FP4 grid at 1.5 points
# per cell (ppc15) on top.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4/first
mkdir -p $OUT
B=pointcloud-segmentation-attention_amd/csrc/build
for v in main ppc15; do
  l=""; [ $v != main ] && l=$B/libpn2hip_v_$v.so
  PN2HIP_LIB=$l timeout -k 10 600 python3 -u -m pytest -x -q --timeout 280 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_a_fullsize.py -k "fp_grid_fused or three_nn or fp_fused or stack_full_size" > $OUT/pytest_$v.log 2>&1 || { tail -30 $OUT/pytest_$v.log; exit 1; }
  tail -1 $OUT/pytest_$v.log
done
for v in main first0 ppc15; do
  l=""; [ $v != main ] && l=$B/libpn2hip_v_$v.so
  PN2HIP_LIB=$l timeout -k 10 120 python3 tools/bench_nn.py > $OUT/nn_$v.json 2> $OUT/nn_$v.err || { tail -20 $OUT/nn_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/nn_$v.json')); print('$v', {k: d[k] for k in ('grid edge=0.0 sorted', 'grid edge=0.2 sorted', 'fp4 grid fused', 'cfg3 fp4 grid fused')})"
done
run() {  # name, lib, bench args
  n=$1; l=$2; shift 2
  PN2HIP_LIB=$l timeout -k 10 300 python3 bench.py --no-cpu-baseline --e2e-steps 0 --latency-reps 5 "$@" > $OUT/b_$n.json 2> $OUT/b_$n.err || { tail -20 $OUT/b_$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b_$n.json')); print('$n', round(d['value']), round(d['ms_per_step']*1e3,1), d.get('verified'), round(d.get('latency_ms_per_batch',0),3))"
}
run main ""
run first0 $B/libpn2hip_v_first0.so
run ppc15 $B/libpn2hip_v_ppc15.so
run side_main "" --diag-only side --no-verify
run side_first0 $B/libpn2hip_v_first0.so --diag-only side --no-verify
run main2 ""
run first02 $B/libpn2hip_v_first0.so
