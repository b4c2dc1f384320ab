#!/bin/bash
# Round 5: the split grid build (S workgroups per cloud, tile scan): parity, standalone times,
# bench_side and the pipelined configs.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r5/gb2
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_a_fullsize.py tests/test_gpu_fused_layers.py -x -q --timeout 280 --timeout-method thread \
  -k "grid or ball or fps_chain or fullsize or msg" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 120 python3 tools/bench_gridbuild.py > $OUT/gb.json 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
cat $OUT/gb.json
for c in cfg2 cfg5; do
  timeout -k 10 200 python3 tools/bench_side.py --config $c > $OUT/side_$c.json 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], {k: d[k]['us'] for k in d if isinstance(d[k], dict)}, d['side_sum_us'])" $OUT/side_$c.json $c
done
for c in cfg2 cfg5 cfg3; do
  timeout -k 10 300 python3 bench.py --config $c --steps 500 --warmup 50 --e2e-steps 0 --no-cpu-baseline > $OUT/b_$c.json 2> $OUT/b_$c.err || { tail -20 $OUT/b_$c.err; exit 1; }
  echo "$c $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(round(d['value']), round(d['ms_per_step'],4), d.get('verified'))" $OUT/b_$c.json)"
done
for rep in 1 2 3; do
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --e2e-steps 0 --no-cpu-baseline > $OUT/drv_$rep.json 2> $OUT/drv_$rep.err || { tail -20 $OUT/drv_$rep.err; exit 1; }
  echo "drv20 $rep $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(round(d['value']), round(d['ms_per_step'],4), d.get('verified'))" $OUT/drv_$rep.json)"
done
