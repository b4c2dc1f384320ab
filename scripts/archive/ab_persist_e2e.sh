#!/bin/bash
# Whole-model step (bench.py --model) with and without persistent MLP workgroups.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
  for ps in 0 1; do
    PN2_MLP_PERSIST=$ps timeout -k 10 200 python bench.py --model --no-cpu-baseline --steps 40 > gpurun_out/e2e_p$ps.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/e2e_p$ps.json'));print('persist=$ps rep=$rep', round(d['value']), round(d['ms_per_step'],3))"
  done
done
