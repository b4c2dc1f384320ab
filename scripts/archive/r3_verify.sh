#!/bin/bash
# Re-verify a build: GPU suite, smoke, the driver's bench command, a rocprofv3 kernel-stats pass.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r3/${TAG:-verify}
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 280 --timeout-method thread -m gpu tests \
  > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/bench_driver.err || { tail -20 $OUT/bench_driver.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench_driver.json')); print('driver-cmd', round(d['value']), round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms'],4), d.get('e2e',{}).get('value'))"
for c in ${CONFIGS:-cfg2}; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$c -o run -- python3 bench.py --config $c --steps 200 --warmup 20 --no-cpu-baseline --e2e-steps 0 > $OUT/prof_$c.json 2> $OUT/prof_$c.err || { tail -20 $OUT/prof_$c.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/prof_$c.json')); print('$c prof', round(d['value']), round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms'],4))"
done
