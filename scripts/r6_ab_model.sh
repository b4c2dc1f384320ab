#!/bin/bash
# Whole-model step A/B of variant libraries (csrc/build/libpn2hip_v_<name>.so) against the
# product build: bench.py --model, cfg2 and cfg3, interleaved REP times.
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r6/ab_model}
mkdir -p $OUT
for n in $(seq 1 ${REP:-2}); do
  for v in base ${VARIANTS}; do
    if [ $v = base ]; then unset PN2HIP_LIB; else export PN2HIP_LIB=pointcloud-segmentation-attention_amd/csrc/build/libpn2hip_v_$v.so; fi
    for c in ${CFGS:-cfg2 cfg3}; do
      f=$OUT/${c}_${v}_$n.json
      timeout -k 10 300 python3 bench.py --model --config $c --no-cpu-baseline > $f 2> $f.err || { tail -20 $f.err; exit 1; }
      python3 -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$c $v $n', round(d['value']), round(d['ms_per_step'], 4))"
    done
  done
done
unset PN2HIP_LIB
