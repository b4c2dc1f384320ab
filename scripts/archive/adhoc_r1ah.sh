set -u
mkdir -p gpurun_out
for i in 1 2; do
for v in cur prefill align64 align128 align256; do
if [ $v = cur ]; then L=""; else L=$PWD/tools/ab/libpn2hip_$v.so; fi
PN2HIP_LIB=$L timeout -k 10 120 python tools/bench_chain.py > gpurun_out/ab_$v.log 2>&1 || exit 1
echo $v $(grep chain gpurun_out/ab_$v.log | cut -c1-120)
done; done
