#!/bin/bash
# Round 6, whole-model step: MLP / model parity tests, the model bench (cfg2, cfg3) REP times
# each, and a kernel trace of the cfg2 model step for tools/lane_report.py. Every GPU step has
# its own time limit and the first failure ends the script.
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r6/model}
mkdir -p $OUT
if [ -z "${NOTEST:-}" ]; then
  timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
    tests/test_gpu_model.py tests/test_gpu_mlp.py > $OUT/pytest_model.log 2>&1 || { tail -30 $OUT/pytest_model.log; exit 1; }
  tail -1 $OUT/pytest_model.log
fi
for n in $(seq 1 ${REP:-2}); do
  for c in cfg2 cfg3; do
    timeout -k 10 300 python3 bench.py --model --config $c --no-cpu-baseline ${ARGS:-} > $OUT/model_${c}_$n.json 2> $OUT/model_${c}_$n.err || { tail -20 $OUT/model_${c}_$n.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/model_${c}_$n.json').read().strip().splitlines()[-1]); print('$c', '$n', round(d['value']), round(d['ms_per_step'], 4))"
  done
done
if [ -z "${NOPROF:-}" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --model --steps 100 --warmup 5 --no-cpu-baseline ${ARGS:-} > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
  python3 tools/lane_report.py $(find $OUT/prof -name '*kernel_trace.csv' | head -1) > $OUT/lanes_model_cfg2.txt && head -30 $OUT/lanes_model_cfg2.txt
fi
