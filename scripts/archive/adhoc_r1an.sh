set -u
mkdir -p gpurun_out
for c in cfg2 cfg3; do for s in 2 3 4; do
timeout -k 10 300 python bench.py --config $c --sets $s --no-cpu-baseline > gpurun_out/b_${c}_${s}.json 2>/dev/null || exit 1
echo $c sets=$s $(python -c "import json; d=json.load(open('gpurun_out/b_${c}_${s}.json')); print(round(d['value']), round(d['ms_per_step'],4))")
done; done
timeout -k 10 600 python -m pytest tests -m gpu -q -x -k "pipelined or stack" > gpurun_out/pytest_r1an.log 2>&1; rc=$?; tail -1 gpurun_out/pytest_r1an.log; exit $rc
