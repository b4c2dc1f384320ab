#!/bin/bash
# Round 5: the grid query + grouping with features (pn2_ball_group_grid) and the hit-list
# output phase: parity tests, standalone task costs (cfg2, cfg3), then the chain-stream layouts.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r5/grp
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 280 --timeout-method thread -m gpu tests/test_gpu_fused_layers.py tests/test_gpu_a_fullsize.py -k "ball_group or step or pipeline" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for c in cfg2 cfg3 cfg5; do
timeout -k 10 300 python3 tools/bench_side.py --config $c --json $OUT/side_$c.json > $OUT/side_$c.log 2>&1 || { tail -20 $OUT/side_$c.log; exit 1; }
cat $OUT/side_$c.json | python3 -c "import json,sys; d=json.load(sys.stdin); print(d['config'], d['side_sum_us'], {k: v['us'] for k, v in d.items() if isinstance(v, dict)})"
done
bash scripts/r5_chains.sh
