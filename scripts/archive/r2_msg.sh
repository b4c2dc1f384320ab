#!/bin/bash
# Round 2: the culled sampler at the MSG SA1 size (cfg5) -- GPU suite, cfg5 bench line and
# kernel stats, cfg2 bench line; logs under gpurun_out/.
set -o pipefail
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit 1
echo "== suite ok"
timeout -k 10 300 python bench.py --config cfg5 > $OUT/bench_cfg5.json 2> $OUT/bench_cfg5.err || exit 1
echo "== cfg5 bench ok"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_cfg5 -o run -- python3 bench.py --config cfg5 --steps 20 --warmup 5 --no-cpu-baseline --e2e-steps 0 > $OUT/prof_cfg5.log 2>&1 || exit 1
echo "== cfg5 stats ok"
timeout -k 10 300 python bench.py > $OUT/bench_cfg2.json 2> $OUT/bench_cfg2.err || exit 1
echo "== done"
