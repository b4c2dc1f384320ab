#!/bin/bash
# Round 5: the fused MLP kernels alone (tools/bench_mlp.py) and their phase stamps
# (tools/stamp_mlp.py, stamped build), cfg2 and the cfg3 attention layers.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r5/mlp
mkdir -p $OUT
timeout -k 10 200 python3 tools/bench_mlp.py > $OUT/bench_mlp.jsonl 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
cat $OUT/bench_mlp.jsonl
timeout -k 10 200 python3 tools/stamp_mlp.py > $OUT/stamp_mlp.jsonl 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
cut -c1-330 $OUT/stamp_mlp.jsonl
timeout -k 10 200 python3 tools/stamp_mlp.py --attention > $OUT/stamp_mlp_attention.jsonl 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
cut -c1-400 $OUT/stamp_mlp_attention.jsonl
