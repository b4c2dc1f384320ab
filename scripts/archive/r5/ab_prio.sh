#!/bin/bash
# A/B: lane-0 stream priority x HW queues, geometric + whole model, same box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/abp
for rep in 1 2; do
for cfg in "4 default" "4 high" "8 high"; do
  set -- $cfg
  GPU_MAX_HW_QUEUES=$1 timeout -k 10 200 python bench.py --no-cpu-baseline --e2e-steps 30 --lane0-priority $2 > gpurun_out/abp/b_$1_$2_$rep.json 2>gpurun_out/abp/b_$1_$2_$rep.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/abp/b_$1_$2_$rep.json')); print('q=$1 prio=$2 rep=$rep geo', round(d['value']), round(d['roofline']['avg_launch_ms'],3), 'e2e', round(d['e2e']['value']), round(d['e2e']['sa1_sampler_ms'],3))"
done; done
