#!/bin/bash
# Per-point MLP outputs staged through LDS (PN2_MLP_STAGE_OUT=1, default) vs stored from the
# registers: parity, per-layer times, whole-model step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_mlp.py tests/test_gpu_model.py -x -q --timeout 300 --timeout-method thread > gpurun_out/so_tests.log 2>&1
rc=$?; tail -3 gpurun_out/so_tests.log; [ $rc -eq 0 ] || exit $rc
for v in 0 1; do
  for cfg in cfg2 cfg3; do
    PN2_MLP_STAGE_OUT=$v timeout -k 10 200 python tools/bench_mlp.py --config $cfg > gpurun_out/so.jsonl || exit 1
    echo "stage_out=$v $cfg $(tail -1 gpurun_out/so.jsonl) $(grep -o '"layer": "FP[0-9]", "us": [0-9.]*' gpurun_out/so.jsonl | tr '\n' ' ')"
  done
  for rep in 1 2; do
    PN2_MLP_STAGE_OUT=$v timeout -k 10 200 python bench.py --model --no-cpu-baseline --steps 40 > gpurun_out/so.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/so.json'));print('stage_out=$v e2e', round(d['value']), round(d['ms_per_step'],3))"
  done
done
