#!/bin/bash
# Round 2 close: cfg5 kernel stats and HBM PMC passes for the culled MSG sampler, the default
# cfg2 bench line and smoke; logs under gpurun_out/.
set -o pipefail
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_cfg5 -o run -- python3 bench.py --config cfg5 --steps 20 --warmup 5 --no-cpu-baseline --e2e-steps 0 > $OUT/prof_cfg5.log 2>&1 || exit 1
echo "== cfg5 stats ok"
TAG=cfg5_B8 BENCH_ARGS="--config cfg5" SKIP_TESTS=1 SKIP_BENCH=1 SKIP_PROF=1 PROF_TIMEOUT=240 bash scripts/gpu_check.sh > $OUT/pmc_cfg5.out 2>&1 || exit 1
echo "== cfg5 pmc ok"
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1
timeout -k 10 300 python bench.py > $OUT/bench_cfg2.json 2> $OUT/bench_cfg2.err || exit 1
echo "== done"
