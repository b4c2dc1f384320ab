#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r3/grid1b
mkdir -p $OUT
PN2_GRID_SHARED=0 timeout -k 10 400 python3 -u -m pytest -x -q --timeout 280 --timeout-method thread -m gpu tests/test_gpu_a_fullsize.py tests/test_gpu_parity.py -k "pipeline or stack or replay or overlap" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for J in 0 1 0 1; do
  for c in cfg2 cfg3; do
  PN2_GRID_SHARED=$J timeout -k 10 200 python3 bench.py --config $c --no-cpu-baseline --e2e-steps 0 > $OUT/b.json 2> $OUT/err.log || { tail -5 $OUT/err.log; exit 1; }
  PN2_GRID_SHARED=$J timeout -k 10 200 python3 bench.py --config $c --no-cpu-baseline --e2e-steps 0 --steps 20 --warmup 5 > $OUT/d.json 2> $OUT/err.log || { tail -5 $OUT/err.log; exit 1; }
  python3 -c "
import json; a=json.load(open('$OUT/b.json')); b=json.load(open('$OUT/d.json'))
print('$c shared=$J', round(a['value']), round(a['ms_per_step'],4), round(a['roofline']['avg_launch_ms'],3), {k: round(v,4) for k,v in (a.get('host') or {}).items()}, '| 20 steps', round(b['value']))"
  done
done
