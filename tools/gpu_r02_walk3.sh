#!/bin/bash
# Walker iteration: parity tests, C4 at 1M docs, lane census, SQ counters.
mkdir -p gpurun_out && R=$PWD
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 150 --timeout-method thread -k "walker or c4 or sv_diff or golden or fuzz or edge_states or empty" > gpurun_out/t_walk.log 2>&1 && \
timeout -k 10 300 python -u tools/bench_configs.py c4 1000000 > gpurun_out/c4_1m.log 2>&1 && \
timeout -k 10 300 python -u tools/diag_walk.py 1000000 > gpurun_out/diag_walk.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-trace --output-format csv -d $R/gpurun_out/prof_c4sq -o sq -- python3 $R/tools/bench_configs.py c4 1000000 > $R/gpurun_out/prof_c4sq.log 2>&1
