#!/bin/bash
# FP XCD-mapping check: GPU suite, then HBM PMC passes for cfg2 and cfg3 (B = 16).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu_fp.log 2>&1 && tail -1 $OUT/pytest_gpu_fp.log \
&& CFG=cfg2 B=16 TAG=fp2 bash scripts/r2_pmc.sh && CFG=cfg3 B=16 TAG=fp3 bash scripts/r2_pmc.sh \
&& timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_fp3 -o run -- python3 bench.py --config cfg3 --steps 20 --warmup 5 --no-cpu-baseline --e2e-steps 0 > $OUT/prof_fp3.log 2>&1 \
&& timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_fp2 -o run -- python3 bench.py --config cfg2 --steps 20 --warmup 5 --no-cpu-baseline --e2e-steps 0 > $OUT/prof_fp2.log 2>&1 && echo "== done"
