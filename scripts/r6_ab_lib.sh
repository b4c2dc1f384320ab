#!/bin/bash
# A/B of two whole-library builds: the GPU suite on the candidate (libpn2hip.so), then the SA1
# sampler alone (tools/bench_sampler.py) and the cfg2 step at 500 steps, interleaved REP times
# against BASE (a copy of the previous build). Every GPU step has its own time limit.
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r6/ab_lib}
BASE=${BASE:-pointcloud-segmentation-attention_amd/csrc/build/libpn2hip_base.so}
mkdir -p $OUT
if [ -z "${NOTEST:-}" ]; then
  timeout -k 10 600 python3 -u -m pytest -x -q --timeout 280 --timeout-method thread -m gpu tests \
    > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
  tail -1 $OUT/pytest_gpu.log
fi
for n in $(seq 1 ${REP:-2}); do
  for v in base cand; do
    if [ $v = base ]; then export PN2HIP_LIB=$BASE; else unset PN2HIP_LIB; fi
    timeout -k 10 200 python3 tools/bench_sampler.py > $OUT/sampler_${v}_$n.json 2> $OUT/sampler_${v}_$n.err || { tail -20 $OUT/sampler_${v}_$n.err; exit 1; }
    echo "sampler $v $n $(tail -1 $OUT/sampler_${v}_$n.json)"
    if [ -z "${NOSTEP:-}" ]; then
      timeout -k 10 300 python3 bench.py --steps 500 --no-cpu-baseline --e2e-steps 0 > $OUT/cfg2_${v}_$n.json 2> $OUT/cfg2_${v}_$n.err || { tail -20 $OUT/cfg2_${v}_$n.err; exit 1; }
      python3 -c "import json; d=json.loads(open('$OUT/cfg2_${v}_$n.json').read().strip().splitlines()[-1]); print('cfg2-500 $v $n', round(d['value']), round(d['roofline']['avg_launch_ms'],4), d.get('verified'))"
    fi
  done
done
unset PN2HIP_LIB
