#!/bin/bash
# SQ/SQC counter passes over bench.py (gpurun): instruction mix / wait split, issue activity, I-cache.
mkdir -p gpurun_out && R=$PWD && cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --steps 3 --warmup 1 --no-cpu-baseline"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-trace --output-format csv -d $R/gpurun_out/prof_sq -o sq -- python3 $B > $R/gpurun_out/prof_sq.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_BUSY_CU_CYCLES SQ_INST_CYCLES_SALU --kernel-trace --output-format csv -d $R/gpurun_out/prof_sq2 -o sq2 -- python3 $B > $R/gpurun_out/prof_sq2.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_LEVEL_WAVES SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace --output-format csv -d $R/gpurun_out/prof_sq3 -o sq3 -- python3 $B > $R/gpurun_out/prof_sq3.log 2>&1
