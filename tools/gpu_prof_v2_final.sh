#!/bin/bash
# Kernel stats of the update-V2 block alone (headline kept, other blocks off).
mkdir -p gpurun_out && R=$PWD && cd /tmp && export TMPDIR=/tmp && rm -rf $R/gpurun_out/prof_v2f && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_v2f -o kt -- python3 $R/bench.py --c2big-docs 0 --c4-docs 0 --f1-docs 0 --no-host-api --no-c3 --no-mixed --no-cpu-baseline --no-yjs > $R/gpurun_out/prof_v2f.log 2>&1
