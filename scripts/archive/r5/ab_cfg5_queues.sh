#!/bin/bash
# cfg5 (MSG, 16,384 points, B = 8): hardware queues and lane-0 priority.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
  for v in "4 default" "2 default" "3 default" "4 high" "8 default"; do
    set -- $v
    timeout -k 10 200 python bench.py --config cfg5 --no-cpu-baseline --steps 60 --hw-queues $1 --lane0-priority $2 > gpurun_out/c5q.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/c5q.json'));print('q=$1 prio=$2 rep=$rep', round(d['value']), round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms'],4))"
  done
done
