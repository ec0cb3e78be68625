#!/bin/bash
# The c2_mixed block alone (headline kept, other blocks off) and its kernel stats.
mkdir -p gpurun_out && R=$PWD
timeout -k 10 300 python -u bench.py --c2big-docs 0 --c4-docs 0 --f1-docs 0 --no-host-api --no-v2 --no-c3 --no-cpu-baseline > gpurun_out/bench_mixed.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && rm -rf $R/gpurun_out/prof_mixed && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_mixed -o kt -- python3 $R/bench.py --c2big-docs 0 --c4-docs 0 --f1-docs 0 --no-host-api --no-v2 --no-c3 --no-cpu-baseline > $R/gpurun_out/prof_mixed.log 2>&1
