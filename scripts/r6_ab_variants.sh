#!/bin/bash
# A/B of variant libraries (make variant ... -> csrc/build/libpn2hip_v_<name>.so) against the
# product build: the SA1 sampler alone (tools/bench_sampler.py) and the cfg2 step at 500 steps
# (every timed cloud verified against the oracle), interleaved REP times.
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r6/ab_var}
mkdir -p $OUT
for n in $(seq 1 ${REP:-2}); do
  for v in base ${VARIANTS}; do
    if [ $v = base ]; then unset PN2HIP_LIB; else export PN2HIP_LIB=pointcloud-segmentation-attention_amd/csrc/build/libpn2hip_v_$v.so; fi
    timeout -k 10 200 python3 tools/bench_sampler.py > $OUT/sampler_${v}_$n.json 2> $OUT/sampler_${v}_$n.err || { tail -20 $OUT/sampler_${v}_$n.err; exit 1; }
    echo "sampler $v $n $(tail -1 $OUT/sampler_${v}_$n.json)"
    if [ -z "${NOSTEP:-}" ]; then
      timeout -k 10 300 python3 bench.py --steps 500 --no-cpu-baseline --e2e-steps 0 > $OUT/cfg2_${v}_$n.json 2> $OUT/cfg2_${v}_$n.err || { tail -20 $OUT/cfg2_${v}_$n.err; exit 1; }
      python3 -c "import json; d=json.loads(open('$OUT/cfg2_${v}_$n.json').read().strip().splitlines()[-1]); print('cfg2-500 $v $n', round(d['value']), round(d['roofline']['avg_launch_ms'],4), d.get('verified'), d.get('fault_status'))"
    fi
  done
done
unset PN2HIP_LIB
