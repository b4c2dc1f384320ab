#!/bin/bash
# GPU suite (full-size bit-exact parity first) + smoke + default bench line; logs in gpurun_out/r3/.
set -o pipefail
OUT=gpurun_out/r3
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -60 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python bench.py > $OUT/bench_cfg2.json 2> $OUT/bench_cfg2.err || { tail -20 $OUT/bench_cfg2.err; exit 1; }
cat $OUT/bench_cfg2.json
