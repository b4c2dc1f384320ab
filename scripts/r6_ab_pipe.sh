#!/bin/bash
# Pipeline A/B of variant libraries against the product build: the driver's command (20 steps),
# cfg2 at 500 steps and cfg5, interleaved REP times (every timed cloud verified).
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r6/ab_pipe}
mkdir -p $OUT
for n in $(seq 1 ${REP:-3}); do
  for v in base ${VARIANTS}; do
    if [ $v = base ]; then unset PN2HIP_LIB; else export PN2HIP_LIB=pointcloud-segmentation-attention_amd/csrc/build/libpn2hip_v_$v.so; fi
    for run in "drv:--gpus 1 --steps 20 --warmup 5" "c500:--steps 500" "cfg5:--config cfg5"; do
      tag=${run%%:*}; a=${run#*:}
      f=$OUT/${tag}_${v}_$n.json
      timeout -k 10 300 python3 bench.py $a --no-cpu-baseline --e2e-steps 0 > $f 2> $f.err || { tail -20 $f.err; exit 1; }
      python3 -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$tag $v $n', round(d['value']), round(d['roofline']['avg_launch_ms'],4), d.get('verified'), d.get('fault_status'))"
    done
  done
done
unset PN2HIP_LIB
