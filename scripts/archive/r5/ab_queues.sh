#!/bin/bash
# A/B of the HIP hardware-queue count (the box exports GPU_MAX_HW_QUEUES=4) for the
# geometric step and the whole-model step, same box, alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/abq
for rep in 1 2; do
for q in 4 8 16; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python bench.py --no-cpu-baseline --e2e-steps 30 > gpurun_out/abq/b_${q}_$rep.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/abq/b_${q}_$rep.json')); print('q=$q rep=$rep geo', round(d['value']), round(d['roofline']['avg_launch_ms'],3), 'e2e', round(d['e2e']['value']), round(d['e2e']['sa1_sampler_ms'],3))"
done; done
