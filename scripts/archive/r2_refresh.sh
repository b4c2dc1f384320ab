#!/bin/bash
# Round 2 refresh: cfg3 HBM PMC passes and kernel stats, then the cfg2 / cfg3 / cfg5 bench lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
CFG=cfg3 B=16 TAG=c3 bash scripts/r2_pmc.sh \
&& timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_cfg3 -o run -- python3 bench.py --config cfg3 --steps 20 --warmup 5 --no-cpu-baseline --e2e-steps 0 > $OUT/prof_cfg3.log 2>&1 \
&& bash scripts/r2_benches.sh
