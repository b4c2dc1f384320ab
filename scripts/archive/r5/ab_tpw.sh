#!/bin/bash
# A/B of tiles per MLP workgroup (PN2_MLP_TPW cap, PN2_MLP_ROUNDS minimum rounds of
# workgroups): isolated layer times (cfg2, cfg3) and the whole-model step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in "1 4" "8 4" "8 2" "8 1"; do
  set -- $v
  for cfg in cfg2 cfg3; do
    PN2_MLP_TPW=$1 PN2_MLP_ROUNDS=$2 timeout -k 10 200 python tools/bench_mlp.py --config $cfg > gpurun_out/tpw.jsonl || exit 1
    echo "tpw<=$1 rounds>=$2 $cfg $(tail -1 gpurun_out/tpw.jsonl) $(grep -o '"layer": "SA1", "us": [0-9.]*' gpurun_out/tpw.jsonl) $(grep -o '"layer": "FP4", "us": [0-9.]*' gpurun_out/tpw.jsonl)"
  done
  for rep in 1 2; do
    PN2_MLP_TPW=$1 PN2_MLP_ROUNDS=$2 timeout -k 10 200 python bench.py --model --no-cpu-baseline --steps 40 > gpurun_out/e2e_tpw.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/e2e_tpw.json'));print('tpw<=$1 rounds>=$2 e2e', round(d['value']), round(d['ms_per_step'],3))"
  done
done
