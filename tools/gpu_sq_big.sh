#!/bin/bash
# SQ counters of the C5 large-document probe (gpurun): instruction mix, instruction-fetch and issue waits of k_merge_big
mkdir -p gpurun_out && R=$PWD && cd /tmp && export TMPDIR=/tmp && \
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_IFETCH SQ_INSTS_FLAT --kernel-trace --output-format csv -d $R/gpurun_out/prof_sq_c5 -o c5 -- python3 $R/tools/bench_configs.py c5 20 > $R/gpurun_out/prof_sq_c5.log 2>&1
