#!/bin/bash
# three side lanes: full-size parity (pipeline included), bench lines, a cfg3 kernel trace
set -o pipefail
OUT=gpurun_out/r3
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_a_fullsize.py -x -q --timeout 300 --timeout-method thread > $OUT/lanes_fullsize.log 2>&1 || { tail -40 $OUT/lanes_fullsize.log; exit 1; }
tail -1 $OUT/lanes_fullsize.log
bash scripts/r3_bench3.sh || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_lanes_cfg3 -o run -- python3 bench.py --config cfg3 --steps 20 --warmup 5 --no-cpu-baseline --e2e-steps 0 > $OUT/prof_lanes_cfg3.log 2>&1 || { tail -20 $OUT/prof_lanes_cfg3.log; exit 1; }
echo prof ok
