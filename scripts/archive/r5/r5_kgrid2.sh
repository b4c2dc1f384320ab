#!/bin/bash
# Round 5: where FP4's known grid is built (stack.FP4_KNOWN_GRID: lane / sampler / off):
# parity tests, bench_side per mode, pipeline A/B cfg2 + cfg3 (2 reps each).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r5/kgrid2
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_a_fullsize.py -x -q --timeout 280 --timeout-method thread \
  -k "fps_chain or fp_grid_fused or three_nn_grid or pipelined or graph_replay or side_stream or fullsize" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 200 python3 tools/bench_fp4.py > $OUT/bench_fp4.json 2> $OUT/bench_fp4.err || { tail -20 $OUT/bench_fp4.err; exit 1; }
cat $OUT/bench_fp4.json
for m in lane sampler off; do
  timeout -k 10 200 python3 tools/bench_side.py --config cfg2 --fp4-known-grid $m > $OUT/side_cfg2_$m.json 2>> $OUT/side.err || { tail -20 $OUT/side.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], {k: d[k]['us'] for k in d if isinstance(d[k], dict)}, d['side_sum_us'])" $OUT/side_cfg2_$m.json $m
done
for rep in 1 2; do
  for c in cfg2 cfg3; do
    for m in lane sampler off; do
      timeout -k 10 300 python3 bench.py --config $c --steps 500 --warmup 50 --e2e-steps 0 --no-cpu-baseline --fp4-known-grid $m > $OUT/bench_${c}_${m}_$rep.json 2> $OUT/bench_${c}_${m}_$rep.err || { tail -20 $OUT/bench_${c}_${m}_$rep.err; exit 1; }
      echo "$c $m $rep $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(round(d['value']), round(d['ms_per_step'],4), d.get('verified'))" $OUT/bench_${c}_${m}_$rep.json)"
    done
  done
done
for rep in 1 2 3; do
  for m in lane off; do
    timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --e2e-steps 0 --no-cpu-baseline --fp4-known-grid $m > $OUT/drv_${m}_$rep.json 2> $OUT/drv_${m}_$rep.err || { tail -20 $OUT/drv_${m}_$rep.err; exit 1; }
    echo "drv20 $m $rep $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(round(d['value']), round(d['ms_per_step'],4), d.get('verified'))" $OUT/drv_${m}_$rep.json)"
  done
done
