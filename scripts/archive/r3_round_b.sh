#!/bin/bash
# Sampler round-end variants A/B + full-size parity of the product, then kernel stats and HBM
# PMC passes of the cfg2 / cfg3 bench (XCD-aware ball query / grouping); logs in gpurun_out/.
set -o pipefail
bash scripts/r3_ab.sh "$@" || exit 1
TAG=r3_cfg2 SKIP_TESTS=1 SKIP_BENCH=1 BENCH_ARGS="--config cfg2" bash scripts/gpu_check.sh > gpurun_out/r3/check_cfg2.out 2>&1 || { tail -20 gpurun_out/r3/check_cfg2.out; exit 1; }
tail -3 gpurun_out/r3/check_cfg2.out
TAG=r3_cfg3 SKIP_TESTS=1 SKIP_BENCH=1 BENCH_ARGS="--config cfg3" bash scripts/gpu_check.sh > gpurun_out/r3/check_cfg3.out 2>&1 || { tail -20 gpurun_out/r3/check_cfg3.out; exit 1; }
tail -3 gpurun_out/r3/check_cfg3.out
