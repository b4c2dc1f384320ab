#!/bin/bash
# HBM PMC passes (one counter per pass) over the default bench, then the summary.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out; TAG=${TAG:-r2}; CFG=${CFG:-cfg2}; B=${B:-16}; mkdir -p $OUT
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/pmc_FETCH_SIZE_$TAG -o run -- python3 bench.py --config $CFG --batch $B --steps 5 --warmup 2 --no-cpu-baseline --e2e-steps 0 > $OUT/pmc_FETCH_SIZE_$TAG.log 2>&1 \
&& timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/pmc_WRITE_SIZE_$TAG -o run -- python3 bench.py --config $CFG --batch $B --steps 5 --warmup 2 --no-cpu-baseline --e2e-steps 0 > $OUT/pmc_WRITE_SIZE_$TAG.log 2>&1 \
&& python3 tools/pmc_summary.py $OUT/pmc_FETCH_SIZE_$TAG $OUT/pmc_WRITE_SIZE_$TAG > $OUT/pmc_traffic_${CFG}_B$B.json && echo "== pmc done"
