set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python tools/bench_chain.py > gpurun_out/chain_r1y.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/chain_r1y.log
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_r1y.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_r1y.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_r1y.json 2> gpurun_out/bench_r1y.err; rc=$?; cut -c1-200 gpurun_out/bench_r1y.json; exit $rc
