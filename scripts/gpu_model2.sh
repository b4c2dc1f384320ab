#!/bin/bash
# MLP parity + model bench A/B (queues) + profile of the model step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_mlp.py -x -q --timeout 200 --timeout-method thread > gpurun_out/model_tests.log 2>&1
rc=$?; tail -3 gpurun_out/model_tests.log; [ $rc -eq 0 ] || exit $rc
for q in 8 16; do
GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_q$q.json 2> gpurun_out/bench_q$q.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/bench_q$q.json')); print('q=$q geo', round(d['value']), 'e2e', round(d['e2e']['value']), round(d['e2e']['ms_per_step'],3))"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_model -o run -- python3 bench.py --model --steps 20 --warmup 5 > gpurun_out/prof_model.log 2>&1
rc=$?; tail -1 gpurun_out/prof_model.log; exit $rc
