#!/bin/bash
# sampler A/B against the libs given (+ full-size parity), then the chain-tail A/B (chain1w)
set -o pipefail
bash scripts/r3_ab.sh "$@" || exit 1
timeout -k 10 200 python -u tools/chain_ab.py --lib chain1w=pointcloud-segmentation-attention_amd/csrc/build/libpn2hip_chain1w.so > gpurun_out/r3/chain_ab.log 2>&1 || { tail -20 gpurun_out/r3/chain_ab.log; exit 1; }
tail -1 gpurun_out/r3/chain_ab.log
