#!/bin/bash
# Round 2 evidence run: GPU suite, smoke, default bench, rocprofv3 kernel stats, HBM PMC passes
# (one counter per pass), the sampler stamp summary. Stops at the first failing step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out; TAG=${TAG:-r2}; mkdir -p $OUT
step() { echo "== $1"; }
step pytest && timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu_$TAG.log 2>&1 && tail -2 $OUT/pytest_gpu_$TAG.log \
&& step smoke && timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_$TAG.log 2>&1 && tail -1 $OUT/smoke_$TAG.log \
&& step bench && timeout -k 10 400 python -u bench.py > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err && cut -c1-400 $OUT/bench_$TAG.json \
&& step rocprof && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --e2e-steps 0 > $OUT/prof_$TAG.log 2>&1 && tail -2 $OUT/prof_$TAG.log \
&& step pmc_fetch && timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/pmc_FETCH_SIZE_$TAG -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --e2e-steps 0 > $OUT/pmc_FETCH_SIZE_$TAG.log 2>&1 \
&& step pmc_write && timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/pmc_WRITE_SIZE_$TAG -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --e2e-steps 0 > $OUT/pmc_WRITE_SIZE_$TAG.log 2>&1 \
&& python3 tools/pmc_summary.py $OUT/pmc_FETCH_SIZE_$TAG $OUT/pmc_WRITE_SIZE_$TAG > $OUT/pmc_traffic_cfg2_B16.json \
&& step stamps && timeout -k 10 300 make -s -C tools/fps_lab > $OUT/lab_build.log 2>&1 && timeout -k 10 120 python -u tools/stamp_fps_cull.py --json $OUT/sa1_cull_stamps.json > $OUT/stamp_cull_$TAG.log 2>&1 \
&& echo "== done"
