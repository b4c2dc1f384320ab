#!/bin/bash
# MLP parity, per-layer MLP timings, model bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_mlp.py -x -q --timeout 200 --timeout-method thread > gpurun_out/model_tests.log 2>&1
rc=$?; tail -3 gpurun_out/model_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/bench_mlp.py > gpurun_out/bench_mlp.jsonl 2> gpurun_out/bench_mlp.err; rc=$?; cat gpurun_out/bench_mlp.jsonl; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --model --steps 30 > gpurun_out/bench_model.json 2> gpurun_out/bench_model.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/bench_model.json')); print('model', round(d['value']), round(d['ms_per_step'],3), d['roofline']['avg_launch_ms'])"
