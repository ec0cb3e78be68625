#!/bin/bash
# Round-2 final profile set (gpurun): parity tests, kernel-trace stats of the default bench line, separate
# FETCH_SIZE / WRITE_SIZE passes per workload (lean10k = headline C2, lean100k = C2 at 100k docs, c4 = C4 1M
# docs SV + diff), one SQ pass over C4 (the default bench line with its CPU baselines: a call of its own,
# `python -u bench.py > gpurun_out/f_bench.log`).  Every GPU step has its own limit; the chain stops at the
# first failure.
mkdir -p gpurun_out && R=$PWD
P="python3 $R/bench.py --no-cpu-baseline --no-yjs"
ONLY="--no-v2 --no-c3 --no-mixed --f1-docs 0 --no-host-api"
timeout -k 10 700 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/f_tests.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/f_kt -o kt -- $P > $R/gpurun_out/f_kt.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/f_f_lean10k -o f -- $P $ONLY --steps 3 --warmup 1 --c2big-docs 0 --c4-docs 0 > $R/gpurun_out/f_f1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/f_w_lean10k -o w -- $P $ONLY --steps 3 --warmup 1 --c2big-docs 0 --c4-docs 0 > $R/gpurun_out/f_w1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/f_f_lean100k -o f -- $P $ONLY --steps 3 --warmup 1 --docs 100000 --c2big-docs 0 --c4-docs 0 > $R/gpurun_out/f_f2.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/f_w_lean100k -o w -- $P $ONLY --steps 3 --warmup 1 --docs 100000 --c2big-docs 0 --c4-docs 0 > $R/gpurun_out/f_w2.log 2>&1 && \
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/f_f_c4 -o f -- python3 $R/tools/bench_configs.py c4 1000000 > $R/gpurun_out/f_f3.log 2>&1 && \
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/f_w_c4 -o w -- python3 $R/tools/bench_configs.py c4 1000000 > $R/gpurun_out/f_w3.log 2>&1 && \
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-trace --output-format csv -d $R/gpurun_out/f_sq_c4 -o sq -- python3 $R/tools/bench_configs.py c4 1000000 > $R/gpurun_out/f_sq.log 2>&1
