#!/bin/bash
# Round 4: MSG SA1's three radii in ONE grid-query launch (pn2_ball_group_xyz_grid_radii)
# against one launch per radius (PN2_MSG_SA1_SPLIT=1).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4/radii
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 280 --timeout-method thread -m gpu tests/test_gpu_fused_layers.py tests/test_gpu_a_fullsize.py -k "radii or ball_group_xyz or stack_full_size or pipeline" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 200 python3 tools/bench_msg_grid.py > $OUT/msg_grid.json 2> $OUT/msg_grid.err || { tail -20 $OUT/msg_grid.err; exit 1; }
grep -i "three\|build" $OUT/msg_grid.json
run() {  # name, bench args
  n=$1; shift
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --e2e-steps 0 --latency-reps 5 "$@" > $OUT/b_$n.json 2> $OUT/b_$n.err || { tail -20 $OUT/b_$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b_$n.json')); print('$n', round(d['value']), round(d['ms_per_step']*1e3,1), d.get('verified'), round(d.get('latency_ms_per_batch',0),3))"
}
run cfg5 --config cfg5
export PN2_MSG_SA1_SPLIT=1; run cfg5_split --config cfg5; unset PN2_MSG_SA1_SPLIT
run cfg5_b --config cfg5
export PN2_MSG_SA1_SPLIT=1; run cfg5_split_b --config cfg5; unset PN2_MSG_SA1_SPLIT
run cfg5_side --config cfg5 --diag-only side --no-verify
export PN2_MSG_SA1_SPLIT=1; run cfg5_split_side --config cfg5 --diag-only side --no-verify; unset PN2_MSG_SA1_SPLIT
run cfg5_drv --config cfg5 --steps 20 --warmup 5
