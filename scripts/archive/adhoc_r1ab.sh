set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python tools/bench_chain.py > gpurun_out/chain_r1ab.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/chain_r1ab.log
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_r1ab.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_r1ab.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_r1ab.json 2> gpurun_out/bench_r1ab.err; rc=$?; cut -c1-200 gpurun_out/bench_r1ab.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_r1ab -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof_r1ab.log 2>&1; rc=$?; [ $rc -eq 0 ] || exit $rc
python tools/timeline.py $(find gpurun_out/prof_r1ab -name "*kernel_trace.csv" | head -1) | tail -1
