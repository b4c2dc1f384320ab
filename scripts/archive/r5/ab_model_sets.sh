#!/bin/bash
# Whole-model step vs the number of pipelined buffer sets (chains in flight).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
  for n in 2 3 4; do
    for c in cfg2 cfg3; do
      timeout -k 10 200 python bench.py --model --config $c --no-cpu-baseline --steps 40 --sets $n > gpurun_out/ms.json 2>/dev/null || exit 1
      python3 -c "import json;d=json.load(open('gpurun_out/ms.json'));print('$c sets=$n rep=$rep', round(d['value']), round(d['ms_per_step'],3))"
    done
  done
done
