#!/bin/bash
# Round 4: the grid three_nn's wave box (grid_nn3_wave: one candidate box per wave of
# unknowns, shell walk only for the uncertified) against the walk alone (margin 0) and other
# margins.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4/box
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 280 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "fp_grid_fused or three_nn or fp_fused or step" > $OUT/pytest_parity.log 2>&1 || { tail -30 $OUT/pytest_parity.log; exit 1; }
tail -1 $OUT/pytest_parity.log
B=pointcloud-segmentation-attention_amd/csrc/build
for v in main mg0 mg45 mg80; do
  l=""; [ $v != main ] && l=$B/libpn2hip_v_$v.so
  PN2HIP_LIB=$l timeout -k 10 120 python3 tools/bench_nn.py > $OUT/nn_$v.json 2> $OUT/nn_$v.err || { tail -20 $OUT/nn_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/nn_$v.json')); print('$v', {k: d[k] for k in ('grid edge=0.0 rand', 'grid edge=0.0 sorted', 'grid edge=0.2 sorted', 'fp4 grid fused', 'fp4 apply only')})"
done
run() {  # name, lib, bench args
  n=$1; l=$2; shift 2
  PN2HIP_LIB=$l timeout -k 10 300 python3 bench.py --no-cpu-baseline --e2e-steps 0 --latency-reps 5 "$@" > $OUT/b_$n.json 2> $OUT/b_$n.err || { tail -20 $OUT/b_$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b_$n.json')); print('$n', round(d['value']), round(d['ms_per_step']*1e3,1), d.get('verified'), round(d.get('latency_ms_per_batch',0),3))"
}
run box ""
run walk $B/libpn2hip_v_mg0.so
run side_box "" --diag-only side --no-verify
run side_walk $B/libpn2hip_v_mg0.so --diag-only side --no-verify
run cfg3_box "" --config cfg3
run cfg3_walk $B/libpn2hip_v_mg0.so --config cfg3
run cfg5_box "" --config cfg5
run drv_box "" --steps 20 --warmup 5
run drv_walk $B/libpn2hip_v_mg0.so --steps 20 --warmup 5
run drv_box2 "" --steps 20 --warmup 5
