set -u
mkdir -p gpurun_out
for te in 1 1000 1; do
timeout -k 10 300 python bench.py --time-every $te --no-cpu-baseline > gpurun_out/b_te$te.json 2>/dev/null || exit 1
echo te=$te $(python -c "import json; d=json.load(open('gpurun_out/b_te$te.json')); print(round(d['value']), round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms'],4))")
done
