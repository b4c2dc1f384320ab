#!/bin/bash
# Round 4: the fused FP4 kernel with its LDS trimmed to 8 workgroups a CU (uint16 offsets, one
# atomic pass; main) against the previous build (prev), its LDS grid at 2 / 1.5 / 1 points per
# cell, and the wave box again (mg60).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4/ppc
mkdir -p $OUT
B=pointcloud-segmentation-attention_amd/csrc/build
for v in main prev ppc15 ppc1; do
  l=""; [ $v != main ] && l=$B/libpn2hip_v_$v.so
  PN2HIP_LIB=$l timeout -k 10 600 python3 -u -m pytest -x -q --timeout 280 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "fp_grid_fused or three_nn or fp_fused" > $OUT/pytest_$v.log 2>&1 || { tail -30 $OUT/pytest_$v.log; exit 1; }
  tail -1 $OUT/pytest_$v.log
done
for v in main prev ppc15 ppc1 mg60; do
  l=""; [ $v != main ] && l=$B/libpn2hip_v_$v.so
  PN2HIP_LIB=$l timeout -k 10 120 python3 tools/bench_nn.py > $OUT/nn_$v.json 2> $OUT/nn_$v.err || { tail -20 $OUT/nn_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/nn_$v.json')); print('$v', {k: d[k] for k in ('grid edge=0.0 sorted', 'fp4 three launches', 'fp4 grid fused', 'fp4 grid fused +nn', 'fp4 apply only')})"
done
run() {  # name, lib, bench args
  n=$1; l=$2; shift 2
  PN2HIP_LIB=$l timeout -k 10 300 python3 bench.py --no-cpu-baseline --e2e-steps 0 --latency-reps 5 "$@" > $OUT/b_$n.json 2> $OUT/b_$n.err || { tail -20 $OUT/b_$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b_$n.json')); print('$n', round(d['value']), round(d['ms_per_step']*1e3,1), d.get('verified'), round(d.get('latency_ms_per_batch',0),3))"
}
run main ""
run prev $B/libpn2hip_v_prev.so
run ppc1 $B/libpn2hip_v_ppc1.so
run side_main "" --diag-only side --no-verify
run side_prev $B/libpn2hip_v_prev.so --diag-only side --no-verify
run side_ppc1 $B/libpn2hip_v_ppc1.so --diag-only side --no-verify
run main2 ""
run prev2 $B/libpn2hip_v_prev.so
