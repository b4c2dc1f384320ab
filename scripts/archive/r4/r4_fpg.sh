#!/bin/bash
# Round 4: FP4 as ONE launch (pn2_fp_grid_fused: each workgroup grids the known points in its
# own LDS, searches, writes its rows) against the round-3 three launches (PN2_FP4_SPLIT=1).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4/fpg
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 280 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "fp_grid_fused or three_nn or fp_fused" > $OUT/pytest_parity.log 2>&1 || { tail -30 $OUT/pytest_parity.log; exit 1; }
tail -1 $OUT/pytest_parity.log
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 280 --timeout-method thread -m gpu tests/test_gpu_a_fullsize.py tests/test_gpu_edge.py tests/test_gpu_model.py > $OUT/pytest_stack.log 2>&1 || { tail -30 $OUT/pytest_stack.log; exit 1; }
tail -1 $OUT/pytest_stack.log
timeout -k 10 120 python3 tools/bench_nn.py > $OUT/nn.json 2> $OUT/nn.err || { tail -20 $OUT/nn.err; exit 1; }
cat $OUT/nn.json
run() {  # name, bench args
  n=$1; shift
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --e2e-steps 0 --latency-reps 5 "$@" > $OUT/b_$n.json 2> $OUT/b_$n.err || { tail -20 $OUT/b_$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b_$n.json')); print('$n', round(d['value']), round(d['ms_per_step']*1e3,1), d['verified'], round(d.get('latency_ms_per_batch',0),3))"
}
run fused
export PN2_FP4_SPLIT=1; run split; unset PN2_FP4_SPLIT
export PN2_DUP_TASKS=fp4; run dup_fp4; unset PN2_DUP_TASKS
run drv_fused --steps 20 --warmup 5
export PN2_FP4_SPLIT=1; run drv_split --steps 20 --warmup 5; unset PN2_FP4_SPLIT
run cfg3 --config cfg3
export PN2_FP4_SPLIT=1; run cfg3_split --config cfg3; unset PN2_FP4_SPLIT
run cfg5 --config cfg5
run fused2
