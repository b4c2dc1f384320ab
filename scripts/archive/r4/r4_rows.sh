#!/bin/bash
# Round 4: the grid three_nn search split by rows over the quad (PN2_NN_ROWSPLIT=1) against
# the round-3 split of each row's points (the nnpts build).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4/rows
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 280 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "fp_grid_fused or three_nn or fp_fused" > $OUT/pytest_parity.log 2>&1 || { tail -30 $OUT/pytest_parity.log; exit 1; }
tail -1 $OUT/pytest_parity.log
B=pointcloud-segmentation-attention_amd/csrc/build
timeout -k 10 120 python3 tools/bench_nn.py > $OUT/nn_rows.json 2> $OUT/nn_rows.err || { tail -20 $OUT/nn_rows.err; exit 1; }
PN2HIP_LIB=$B/libpn2hip_v_nnpts.so timeout -k 10 120 python3 tools/bench_nn.py > $OUT/nn_pts.json 2> $OUT/nn_pts.err || { tail -20 $OUT/nn_pts.err; exit 1; }
for v in rows pts; do python3 -c "import json; d=json.load(open('$OUT/nn_$v.json')); print('$v', {k: d[k] for k in ('grid edge=0.0 sorted', 'grid edge=0.2 sorted', 'fp4 three launches', 'fp4 grid fused', 'fp4 apply only')})"; done
run() {  # name, lib, bench args
  n=$1; l=$2; shift 2
  PN2HIP_LIB=$l timeout -k 10 300 python3 bench.py --no-cpu-baseline --e2e-steps 0 --latency-reps 5 "$@" > $OUT/b_$n.json 2> $OUT/b_$n.err || { tail -20 $OUT/b_$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b_$n.json')); print('$n', round(d['value']), round(d['ms_per_step']*1e3,1), d.get('verified'), round(d.get('latency_ms_per_batch',0),3))"
}
run rows ""
run pts $B/libpn2hip_v_nnpts.so
run side_rows "" --diag-only side --no-verify
run side_pts $B/libpn2hip_v_nnpts.so --diag-only side --no-verify
run cfg3_rows "" --config cfg3
run cfg3_pts $B/libpn2hip_v_nnpts.so --config cfg3
run cfg5_rows "" --config cfg5
run drv_rows "" --steps 20 --warmup 5
run drv_pts $B/libpn2hip_v_nnpts.so --steps 20 --warmup 5
run drv_rows2 "" --steps 20 --warmup 5
