set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_gaps -o run -- python3 tools/bench_gaps.py > gpurun_out/prof_gaps.log 2>&1; rc=$?; tail -2 gpurun_out/prof_gaps.log; [ $rc -eq 0 ] || exit $rc
python3 tools/gaps_report.py gpurun_out/prof_gaps/run_kernel_trace.csv
