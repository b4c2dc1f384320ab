#!/bin/bash
# A/B of two library builds on the same box, interleaved: LIBB=<path of build B> (A = the product)
# ARGS = bench arguments; REPS repetitions
set -o pipefail
OUT=gpurun_out/r3/ablib
mkdir -p $OUT
for c in ${CONFIGS:-cfg2}; do
  for r in $(seq ${REPS:-3}); do
    for v in A B; do
      L=""; [ "$v" = "B" ] && L="$LIBB"
      tag=${c}_${v}_$r
      PN2HIP_LIB=$L timeout -k 10 200 python3 bench.py --config $c --steps 400 --warmup 30 --no-cpu-baseline --e2e-steps 0 \
        ${ARGS:-} > $OUT/b_$tag.json 2> $OUT/b_$tag.err || { tail -20 $OUT/b_$tag.err; exit 1; }
      python3 -c "import json; d=json.load(open('$OUT/b_$tag.json')); print('$tag', round(d['value']), round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms'],4))"
    done
  done
done
