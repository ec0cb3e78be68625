#!/bin/bash
# Round-2 baseline: C4 at 1M documents and C2 at 100k documents with the round-1 kernels, plus a
# rocprofv3 kernel-trace and an SQ pass of the C4 run.
mkdir -p gpurun_out && R=$PWD
timeout -k 10 300 python -u tools/bench_configs.py c4 1000000 > gpurun_out/c4_1m.log 2>&1 && \
timeout -k 10 300 python -u bench.py --docs 100000 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/c2_100k.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_c4 -o kt -- python3 $R/tools/bench_configs.py c4 1000000 > $R/gpurun_out/prof_c4.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-trace --output-format csv -d $R/gpurun_out/prof_c4sq -o sq -- python3 $R/tools/bench_configs.py c4 1000000 > $R/gpurun_out/prof_c4sq.log 2>&1
