set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests -m gpu -q -x -k "stack or graph or overlap or golden or pipelined" > gpurun_out/pytest_r1o.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_r1o.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_r1o.json 2> gpurun_out/bench_r1o.err; rc=$?; cut -c1-260 gpurun_out/bench_r1o.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python tools/tune_fps.py > gpurun_out/tune_fps11.jsonl 2> gpurun_out/tune_fps11.err; rc=$?; tail -1 gpurun_out/tune_fps11.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_r1o -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof_r1o.log 2>&1; rc=$?; tail -1 gpurun_out/prof_r1o.log; exit $rc
