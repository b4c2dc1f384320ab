set -u
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_r1am.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_r1am.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r1am.log 2>&1; rc=$?; tail -2 gpurun_out/smoke_r1am.log; exit $rc
