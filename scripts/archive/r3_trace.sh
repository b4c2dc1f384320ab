#!/bin/bash
# kernel traces + per-queue occupancy of chosen pipeline layouts (VARIANTS="cfg lanes queues sets")
set -o pipefail
OUT=gpurun_out/r3/trace
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in ${VARIANTS:-"cfg2 3 6 9" "cfg2 4 7 8" "cfg3 2 5 6" "cfg3 3 6 9"}; do
  set -- $v
  tag=$1_$2_$3_$4
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_$tag -o run -- \
    python3 bench.py --config $1 --steps 100 --warmup 20 --no-cpu-baseline --e2e-steps 0 \
    --sampler-lanes $2 --hw-queues $3 --sets $4 > $OUT/bench_$tag.json 2> $OUT/bench_$tag.err \
    || { tail -20 $OUT/bench_$tag.err; exit 1; }
  f=$(find $OUT/prof_$tag -name '*kernel_trace.csv' | head -1)
  echo "== $tag"
  python3 tools/lane_report.py $f 60 > $OUT/lanes_$tag.txt && cat $OUT/lanes_$tag.txt
done
