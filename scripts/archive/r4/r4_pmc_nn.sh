#!/bin/bash
# Round 4: SQ counters of the FP4 kernels (tools/bench_nn.py): where the grid search's wave
# cycles go (issue vs waiting), LDS bank conflicts. One counter set per pass.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4/pmcnn
mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --kernel-trace --output-format csv -d $OUT/a -o run -- python3 tools/bench_nn.py > $OUT/a.log 2>&1 || { tail -5 $OUT/a.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_LDS --kernel-trace --output-format csv -d $OUT/b -o run -- python3 tools/bench_nn.py > $OUT/b.log 2>&1 || { tail -5 $OUT/b.log; exit 1; }
find $OUT -name "*counter_collection.csv" | head
echo done
