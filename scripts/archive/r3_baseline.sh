#!/bin/bash
# Round 3 start: GPU suite + smoke + default bench line on the round-2 code; logs in gpurun_out/r3/.
set -o pipefail
OUT=gpurun_out/r3
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > $OUT/pytest_gpu_base.log 2>&1 || { tail -40 $OUT/pytest_gpu_base.log; exit 1; }
tail -3 $OUT/pytest_gpu_base.log
timeout -k 10 300 python bench.py > $OUT/bench_cfg2_base.json 2> $OUT/bench_cfg2_base.err || exit 1
cat $OUT/bench_cfg2_base.json
