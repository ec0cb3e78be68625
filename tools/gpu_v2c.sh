#!/bin/bash
# Update-V2 parity tests, then the kernel-trace stats of the headline + v2 bench blocks.
mkdir -p gpurun_out && R=$PWD
timeout -k 10 400 python -u -m pytest tests/test_v2.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/v2_tests.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_v2 -o kt -- python3 $R/bench.py --c2big-docs 0 --c4-docs 0 --f1-docs 0 --no-host-api --no-cpu-baseline > $R/gpurun_out/prof_v2.log 2>&1
