#!/bin/bash
# Geometric step vs how often the SA1 sampler is bracketed by timing events (--time-every)
# and vs the number of buffer sets.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
  for v in "1 3" "10 3" "1000 3" "1 4" "10 4"; do
    set -- $v
    timeout -k 10 200 python bench.py --no-cpu-baseline --e2e-steps 0 --steps 100 --time-every $1 --sets $2 > gpurun_out/te.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/te.json'));print('every=$1 sets=$2 rep=$rep', round(d['value']), round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms'],4))"
  done
done
