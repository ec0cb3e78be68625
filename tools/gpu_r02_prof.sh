#!/bin/bash
# C4 kernel-trace stats + SQ / LDS counters of the SV / diff walker (separate passes).
mkdir -p gpurun_out && R=$PWD
N=${C4_DOCS:-1000000}
timeout -k 10 300 python -u tools/bench_configs.py c4 $N > gpurun_out/c4.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_c4 -o kt -- python3 $R/tools/bench_configs.py c4 $N > $R/gpurun_out/prof_c4.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-trace --output-format csv -d $R/gpurun_out/prof_c4sq -o sq -- python3 $R/tools/bench_configs.py c4 $N > $R/gpurun_out/prof_c4sq.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_BRANCH --kernel-trace --output-format csv -d $R/gpurun_out/prof_c4sq2 -o sq2 -- python3 $R/tools/bench_configs.py c4 $N > $R/gpurun_out/prof_c4sq2.log 2>&1
