set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests -m gpu -q -x -k "stack or graph or overlap or golden or pipelined" > gpurun_out/pytest_r1n.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_r1n.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_r1n.json 2> gpurun_out/bench_r1n.err; rc=$?; cut -c1-330 gpurun_out/bench_r1n.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --eager > gpurun_out/bench_eager_r1n.json 2> gpurun_out/bench_eager_r1n.err; rc=$?; cut -c1-330 gpurun_out/bench_eager_r1n.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_r1n -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof_r1n.log 2>&1; rc=$?; tail -1 gpurun_out/prof_r1n.log; exit $rc
