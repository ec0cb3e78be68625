#!/bin/bash
# Round-2 check of the tree: every -m gpu test, the default bench line, the large-document lines next to
# the CPU port, and rocprofv3 kernel-trace stats of the default bench.  Each GPU step has its own limit.
mkdir -p gpurun_out && R=$PWD
timeout -k 10 700 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 400 python -u bench.py > gpurun_out/bench.log 2>&1 && \
timeout -k 10 150 python -u bench.py --big c3 > gpurun_out/big_c3.log 2>&1 && \
timeout -k 10 150 python -u bench.py --big c5 > gpurun_out/big_c5.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_kt -o kt -- python3 $R/bench.py --no-cpu-baseline --no-yjs > $R/gpurun_out/prof_kt.log 2>&1
