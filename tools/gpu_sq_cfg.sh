#!/bin/bash
# SQ counters of the C4 probe (gpurun)
mkdir -p gpurun_out && R=$PWD && cd /tmp && export TMPDIR=/tmp && \
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-trace --output-format csv -d $R/gpurun_out/prof_c4 -o c4 -- python3 $R/tools/bench_configs.py c4 100000 > $R/gpurun_out/prof_c4.log 2>&1
