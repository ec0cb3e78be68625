#!/bin/bash
# kernel trace of bench.py (gpurun): per-kernel durations and the gaps between consecutive dispatches
mkdir -p gpurun_out && R=$PWD && cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_tr -o tr -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline > $R/gpurun_out/prof_tr.log 2>&1
