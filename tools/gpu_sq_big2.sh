#!/bin/bash
# SQ / SQC counters of the C5 merge (gpurun): instruction mix and I-cache behaviour of k_merge_big
mkdir -p gpurun_out && R=$PWD && cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/sqb1 $R/gpurun_out/sqb2
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SMEM SQ_INSTS_VMEM --kernel-trace --output-format csv -d $R/gpurun_out/sqb1 -o s1 -- python3 $R/bench.py --big c5 --no-cpu-baseline > $R/gpurun_out/sqb1.log 2>&1 && \
timeout -s KILL 200 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_INSTS_BRANCH SQ_ACTIVE_INST_ANY --kernel-trace --output-format csv -d $R/gpurun_out/sqb2 -o s2 -- python3 $R/bench.py --big c5 --no-cpu-baseline > $R/gpurun_out/sqb2.log 2>&1 && \
python3 $R/tools/sq_summary.py $R/gpurun_out/sqb1 > $R/gpurun_out/sq_big.txt && python3 $R/tools/sq_summary.py $R/gpurun_out/sqb2 >> $R/gpurun_out/sq_big.txt
