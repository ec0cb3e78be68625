#!/bin/bash
# Round-2 profile set (gpurun): kernel-trace stats of the default bench line, then separate FETCH_SIZE /
# WRITE_SIZE passes per workload so each kernel's per-launch HBM bytes are isolated:
#   lean10k  = headline C2 (10k docs)      -> k_merge_lean
#   lean100k = C2 at 100k docs             -> k_merge_lean@100k
#   c4       = C4 1M docs SV + diff        -> k_doc_walk<0>, k_doc_walk<1>
# plus one SQ pass over C4.  Every GPU step has its own limit; the chain stops at the first failure.
mkdir -p gpurun_out && R=$PWD
P="python3 $R/bench.py --no-cpu-baseline --no-yjs"
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/p2_kt -o kt -- $P > $R/gpurun_out/p2_kt.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/p2_f_lean10k -o f -- $P --steps 3 --warmup 1 --c2big-docs 0 --c4-docs 0 > $R/gpurun_out/p2_f1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/p2_w_lean10k -o w -- $P --steps 3 --warmup 1 --c2big-docs 0 --c4-docs 0 > $R/gpurun_out/p2_w1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/p2_f_lean100k -o f -- $P --steps 3 --warmup 1 --docs 100000 --c2big-docs 0 --c4-docs 0 > $R/gpurun_out/p2_f2.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/p2_w_lean100k -o w -- $P --steps 3 --warmup 1 --docs 100000 --c2big-docs 0 --c4-docs 0 > $R/gpurun_out/p2_w2.log 2>&1 && \
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/p2_f_c4 -o f -- python3 $R/tools/bench_configs.py c4 1000000 > $R/gpurun_out/p2_f3.log 2>&1 && \
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/p2_w_c4 -o w -- python3 $R/tools/bench_configs.py c4 1000000 > $R/gpurun_out/p2_w3.log 2>&1 && \
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-trace --output-format csv -d $R/gpurun_out/p2_sq_c4 -o sq -- python3 $R/tools/bench_configs.py c4 1000000 > $R/gpurun_out/p2_sq.log 2>&1 && \
cd $R && timeout -k 10 600 python -u bench.py > gpurun_out/p2_bench.log 2>&1
