#!/bin/bash
# Kernel-trace stats of the full-size C3 batch (no CPU baselines).
mkdir -p gpurun_out && R=$PWD && cd /tmp && export TMPDIR=/tmp && rm -rf $R/gpurun_out/prof_c3full && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_c3full -o kt -- python3 $R/bench.py --big c3full --no-cpu-baseline > $R/gpurun_out/prof_c3full.log 2>&1
