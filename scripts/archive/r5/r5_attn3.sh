#!/bin/bash
# Round 5: the attention reduction with non-temporal K/V loads, 8 blocks per CU: parity, the
# microbenchmark, and the cfg3 pipeline (2 runs) + bench_side cfg3.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r5/attn3
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fused_layers.py tests/test_gpu_a_fullsize.py -x -q --timeout 250 --timeout-method thread -k "attention or attn or cfg3" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 120 python3 tools/bench_attn.py > $OUT/attn.json 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
cat $OUT/attn.json
timeout -k 10 200 python3 tools/bench_side.py --config cfg3 > $OUT/side_cfg3.json 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print({k: d[k]['us'] for k in d if isinstance(d[k], dict)}, d['side_sum_us'])" $OUT/side_cfg3.json
for rep in 1 2; do
  timeout -k 10 300 python3 bench.py --config cfg3 --steps 500 --warmup 50 --e2e-steps 0 --no-cpu-baseline > $OUT/b_cfg3_$rep.json 2> $OUT/b_cfg3_$rep.err || { tail -20 $OUT/b_cfg3_$rep.err; exit 1; }
  echo "cfg3 $rep $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(round(d['value']), round(d['ms_per_step'],4), d.get('verified'))" $OUT/b_cfg3_$rep.json)"
done
