set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -x -k "stack or graph or overlap or pipelined or msg or cfg5" > gpurun_out/pytest_r1ak.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_r1ak.log; [ $rc -eq 0 ] || exit $rc
for c in cfg3 cfg5; do
timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > gpurun_out/bench_r1ak_$c.json 2> gpurun_out/bench_r1ak_$c.err; rc=$?; cut -c1-200 gpurun_out/bench_r1ak_$c.json; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_r1ak -o run -- python3 bench.py --config cfg5 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof_r1ak.log 2>&1; rc=$?; [ $rc -eq 0 ] || exit $rc
python tools/timeline.py $(find gpurun_out/prof_r1ak -name "*kernel_trace.csv" | head -1) > gpurun_out/timeline_r1ak.txt; tail -25 gpurun_out/timeline_r1ak.txt
