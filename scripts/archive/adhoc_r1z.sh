set -u
mkdir -p gpurun_out
timeout -k 10 120 python tools/bench_chain.py > gpurun_out/chain_r1z.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/chain_r1z.log; exit $rc
