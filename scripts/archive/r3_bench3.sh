#!/bin/bash
# bench lines for cfg2 (default, with the CPU baseline), cfg3 and cfg5; logs in gpurun_out/r3/
set -o pipefail
OUT=gpurun_out/r3
mkdir -p $OUT
timeout -k 10 400 python bench.py > $OUT/bench_cfg2.json 2> $OUT/bench_cfg2.err || { tail -20 $OUT/bench_cfg2.err; exit 1; }
timeout -k 10 300 python bench.py --config cfg3 --no-cpu-baseline > $OUT/bench_cfg3.json 2> $OUT/bench_cfg3.err || { tail -20 $OUT/bench_cfg3.err; exit 1; }
timeout -k 10 300 python bench.py --config cfg5 --no-cpu-baseline > $OUT/bench_cfg5.json 2> $OUT/bench_cfg5.err || { tail -20 $OUT/bench_cfg5.err; exit 1; }
python - <<'PY'
import json
for c in ("cfg2", "cfg3", "cfg5"):
    d = json.load(open(f"gpurun_out/r3/bench_{c}.json"))
    r = d["roofline"]
    print(c, round(d["value"]), "clouds/s", round(d["ms_per_step"], 4), "ms/step", "sampler", round(r["avg_launch_ms"], 4), "frac", round(r["frac"], 3), "e2e", d.get("e2e", {}).get("value"))
PY
