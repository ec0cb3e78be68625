#!/bin/bash
# Kernel-trace stats of the update-V2 block (headline + v2 blocks of bench.py, no CPU baselines).
mkdir -p gpurun_out && R=$PWD
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_v2 -o kt -- python3 $R/bench.py --c2big-docs 0 --c4-docs 0 --f1-docs 0 --no-host-api --no-cpu-baseline > $R/gpurun_out/prof_v2.log 2>&1
