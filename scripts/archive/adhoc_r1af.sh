set -u
mkdir -p gpurun_out
for i in 1 2; do
timeout -k 10 120 python tools/bench_chain.py > gpurun_out/ab_new_$i.log 2>&1 || exit 1
PN2HIP_LIB=$PWD/tools/ab/libpn2hip_prefill.so timeout -k 10 120 python tools/bench_chain.py > gpurun_out/ab_old_$i.log 2>&1 || exit 1
echo new $(grep chain gpurun_out/ab_new_$i.log); echo old $(grep chain gpurun_out/ab_old_$i.log)
done
