#!/bin/bash
# Round 5: float2 concat columns for even C1 (cfg3's FP4 C1 = 6): parity, FP4 times, cfg3.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r5/fpv2
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_a_fullsize.py tests/test_gpu_fused_layers.py -x -q --timeout 280 --timeout-method thread \
  -k "fp or three_nn or fullsize" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 120 python3 tools/bench_fp4.py > $OUT/fp4.json 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
cat $OUT/fp4.json
timeout -k 10 200 python3 tools/bench_side.py --config cfg3 > $OUT/side_cfg3.json 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print({k: d[k]['us'] for k in d if isinstance(d[k], dict)}, d['side_sum_us'])" $OUT/side_cfg3.json
for rep in 1 2; do
  timeout -k 10 300 python3 bench.py --config cfg3 --steps 500 --warmup 50 --e2e-steps 0 --no-cpu-baseline > $OUT/b_cfg3_$rep.json 2> $OUT/b_cfg3_$rep.err || { tail -20 $OUT/b_cfg3_$rep.err; exit 1; }
  echo "cfg3 $rep $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(round(d['value']), round(d['ms_per_step'],4), d.get('verified'))" $OUT/b_cfg3_$rep.json)"
done
