set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python tools/bench_chain.py > gpurun_out/chain_ab.log 2>&1 || exit 1
PN2HIP_LIB=$PWD/tools/ab/libpn2hip_chain_nolres.so timeout -k 10 120 python tools/bench_chain.py >> gpurun_out/chain_ab.log 2>&1 || exit 1
timeout -k 10 120 python tools/bench_chain.py >> gpurun_out/chain_ab.log 2>&1
cat gpurun_out/chain_ab.log | grep -v amdgpu.ids
