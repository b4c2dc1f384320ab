#!/bin/bash
# Round 5: fp32 cube root in grid_dims (cheaper automatic-edge header): parity, grid build /
# FP4 / sampler-built grid times, then cfg2 with FP4's known grid from the sampler vs off.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r5/kg3
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_a_fullsize.py tests/test_gpu_fused_layers.py -x -q --timeout 280 --timeout-method thread \
  -k "grid or fp_ or three_nn or fps_chain or fullsize or ball or msg" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 120 python3 tools/bench_gridbuild.py > $OUT/gb.json 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
cat $OUT/gb.json
timeout -k 10 120 python3 tools/bench_fp4.py > $OUT/fp4.json 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
cat $OUT/fp4.json
for rep in 1 2; do
  for m in sampler off lane; do
    timeout -k 10 300 python3 bench.py --config cfg2 --steps 500 --warmup 50 --e2e-steps 0 --no-cpu-baseline --fp4-known-grid $m > $OUT/b_${m}_$rep.json 2> $OUT/b_${m}_$rep.err || { tail -20 $OUT/b_${m}_$rep.err; exit 1; }
    echo "cfg2 $m $rep $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(round(d['value']), round(d['ms_per_step'],4), d.get('verified'))" $OUT/b_${m}_$rep.json)"
  done
done
for rep in 1 2 3; do
  for m in sampler off; do
    timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --e2e-steps 0 --no-cpu-baseline --fp4-known-grid $m > $OUT/d_${m}_$rep.json 2> $OUT/d_${m}_$rep.err || { tail -20 $OUT/d_${m}_$rep.err; exit 1; }
    echo "drv20 $m $rep $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(round(d['value']), round(d['ms_per_step'],4), d.get('verified'))" $OUT/d_${m}_$rep.json)"
  done
done
