#!/bin/bash
# Round 5: parity of this round's new launches, A/B of the grid-search prefetch, the pipelined
# configs at 500 steps and the driver's command.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r5/round2
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 280 --timeout-method thread -m gpu tests/test_gpu_fused_layers.py tests/test_gpu_parity.py tests/test_gpu_a_fullsize.py -k "attention or ball_group or fp_ or step or pipeline or three" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
AB_TAG=pf bash scripts/r5_ab.sh main pf1 pf2 main pf1 || exit 1
run() { n=$1; shift; timeout -k 10 300 python3 bench.py --no-cpu-baseline --e2e-steps 0 "$@" > $OUT/b_$n.json 2> $OUT/b_$n.err || { tail -20 $OUT/b_$n.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/b_$n.json')); print('$n', round(d['value']), round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms'],4), d['verified'])"; }
run cfg2_500 --steps 500
run cfg3_500 --config cfg3 --steps 500
run cfg5_500 --config cfg5 --steps 500
run d1 --steps 20 --warmup 5
run d2 --steps 20 --warmup 5
for c in cfg3 cfg5; do
timeout -k 10 300 python3 tools/bench_side.py --config $c --json $OUT/side_$c.json > $OUT/side_$c.log 2>&1 || { tail -20 $OUT/side_$c.log; exit 1; }
cat $OUT/side_$c.json | python3 -c "import json,sys; d=json.load(sys.stdin); print(d['config'], d['side_sum_us'], {k: v['us'] for k, v in d.items() if isinstance(v, dict)})"
done
echo done
