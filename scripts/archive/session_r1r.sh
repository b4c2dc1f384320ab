#!/bin/bash
# End-of-milestone GPU session (part 2): the bench lines with the committed PMC traffic:
# cfg2 (default, with the CPU baseline), cfg3, cfg5; and the __graft_entry__ smoke test.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python bench.py > gpurun_out/bench_cfg2_r1r.json 2> gpurun_out/bench_cfg2_r1r.err || exit $?
cut -c1-200 gpurun_out/bench_cfg2_r1r.json
for c in cfg3 cfg5; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > gpurun_out/bench_${c}_r1r.json 2> gpurun_out/bench_${c}_r1r.err || exit $?
  cut -c1-200 gpurun_out/bench_${c}_r1r.json
done
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_r1r.log 2>&1 || exit $?
tail -1 gpurun_out/smoke_r1r.log
