#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r3/attn2
mkdir -p $OUT
for f in 0 1 0 1; do
  PN2_ATT_FUSED=$f timeout -k 10 300 python3 bench.py --config cfg3 --no-cpu-baseline --e2e-steps 0 > $OUT/bench_cfg3_$f.json 2> $OUT/e.err || { tail -20 $OUT/e.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_cfg3_$f.json')); print('cfg3 fused=$f', round(d['value']), round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms'],4))"
  PN2_ATT_FUSED=$f timeout -k 10 300 python3 bench.py --config cfg3 --no-cpu-baseline --e2e-steps 0 --diag-only side > $OUT/side_cfg3_$f.json 2> $OUT/e.err || { tail -20 $OUT/e.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/side_cfg3_$f.json')); print('cfg3 fused=$f side-only', round(d['value']), round(d['ms_per_step'],4))"
done
PN2_ATT_FUSED=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_cfg3 -o run -- python3 bench.py --config cfg3 --steps 200 --warmup 20 --no-cpu-baseline --e2e-steps 0 > $OUT/prof_cfg3.json 2> $OUT/prof.err || { tail -20 $OUT/prof.err; exit 1; }
for i in 1 2 3 4 5; do
  timeout -k 10 300 python3 bench.py --config cfg3 --model --steps 20 --warmup 5 > $OUT/model_cfg3_$i.json 2> $OUT/e.err || { tail -20 $OUT/e.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/model_cfg3_$i.json')); print('cfg3 model', round(d['value']), round(d['ms_per_step'],4))"
done
