#!/bin/bash
# Whole-model step: parity + bench (geometric line with its e2e field, and --model).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_mlp.py -x -v --timeout 200 --timeout-method thread > gpurun_out/model_tests.log 2>&1
rc=$?; tail -15 gpurun_out/model_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_e2e.json 2> gpurun_out/bench_e2e.err
rc=$?; cat gpurun_out/bench_e2e.json; tail -3 gpurun_out/bench_e2e.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_model -o run -- python3 bench.py --model --steps 20 --warmup 5 > gpurun_out/prof_model.log 2>&1
rc=$?; tail -2 gpurun_out/prof_model.log; exit $rc
