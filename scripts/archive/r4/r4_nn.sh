#!/bin/bash
# Round 4: FP4's neighbour search (the task that sets the pipelined step's period: one more
# copy of FP4 costs +72 us/step, the other side tasks 0-7 us; profiles/r4/dup).
# Variants of three_nn_grid_kernel: K row blocks per workgroup (one LDS staging of the known
# grid serves K), the known grid read from L2 instead of LDS; FP4's search split from its
# interpolation (dup each half); the search on lane 3.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4/nn
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 280 --timeout-method thread -m gpu tests/test_gpu_a_fullsize.py tests/test_gpu_parity.py -k "pipeline or three_nn or fp" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
B=pointcloud-segmentation-attention_amd/csrc/build
run() {  # name, lib ("" = product), dup list, bench args
  n=$1; l=$2; d=$3; shift 3
  PN2HIP_LIB=$l PN2_DUP_TASKS=$d timeout -k 10 300 python3 bench.py --no-cpu-baseline --e2e-steps 0 --latency-reps 0 "$@" > $OUT/b_$n.json 2> $OUT/b_$n.err || { tail -20 $OUT/b_$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b_$n.json')); print('$n', round(d['value']), round(d['ms_per_step']*1e3,1), d['verified'])"
}
for v in "" nnk2 nnk4 nnk8 nnglob nnglobk4; do
  l=""; [ -n "$v" ] && l=$B/libpn2hip_v_$v.so
  PN2HIP_LIB=$l timeout -k 10 120 python3 tools/bench_nn.py > $OUT/nn_${v:-main}.json 2>&1 || { tail -20 $OUT/nn_${v:-main}.json; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/nn_${v:-main}.json')); print('${v:-main}', d['grid edge=0.0 sorted'], d['build known grid'])"
done
run default "" ""
run dup_nn4 "" nn4
run dup_fp4 "" fp4
for v in nnk2 nnk4 nnk8 nnglob nnglobk4; do run $v $B/libpn2hip_v_$v.so ""; done
export PN2_NN4_LANE=3; run nn4lane3 "" ""; unset PN2_NN4_LANE
run default2 "" ""
