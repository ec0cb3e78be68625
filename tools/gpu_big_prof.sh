#!/bin/bash
# per-kernel time of the C3 / C5 merges (gpurun): rocprofv3 kernel stats of bench --big
mkdir -p gpurun_out && R=$PWD && cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/bigp3 $R/gpurun_out/bigp5
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/bigp3 -o c3 -- python3 $R/bench.py --big c3 > $R/gpurun_out/bigp3.log 2>&1 && \
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/bigp5 -o c5 -- python3 $R/bench.py --big c5 > $R/gpurun_out/bigp5.log 2>&1
