#!/bin/bash
# Round 5: grid ball query -- next query's centre prefetched, two hits' rows loaded at once:
# parity, standalone, bench_side cfg2/cfg5, the pipelines.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r5/bq
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_a_fullsize.py tests/test_gpu_fused_layers.py -x -q --timeout 280 --timeout-method thread \
  -k "grid or ball or fullsize or msg or group" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for c in cfg2 cfg5 cfg3; do
  timeout -k 10 200 python3 tools/bench_side.py --config $c > $OUT/side_$c.json 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], {k: d[k]['us'] for k in d if isinstance(d[k], dict)}, d['side_sum_us'])" $OUT/side_$c.json $c
done
for c in cfg2 cfg5; do
  timeout -k 10 300 python3 bench.py --config $c --steps 500 --warmup 50 --e2e-steps 0 --no-cpu-baseline > $OUT/b_$c.json 2> $OUT/b_$c.err || { tail -20 $OUT/b_$c.err; exit 1; }
  echo "$c $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(round(d['value']), round(d['ms_per_step'],4), d.get('verified'))" $OUT/b_$c.json)"
done
