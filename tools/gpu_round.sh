#!/bin/bash
# GPU-box measurement run (gpurun): parity tests, bench line (with CPU baseline), rocprofv3 kernel-trace
# stats and separate FETCH_SIZE / WRITE_SIZE PMC passes of bench.py.  Every GPU step has its own time
# limit and the chain stops at the first failure.  BENCH_ARGS adds bench.py options.
mkdir -p gpurun_out && R=$PWD
B="$R/bench.py ${BENCH_ARGS:-}"
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 300 python -u $B --steps 20 --warmup 3 > gpurun_out/bench.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_kt -o kt -- python3 $B --steps 20 --warmup 3 --no-cpu-baseline > $R/gpurun_out/prof_kt.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/prof_fetch -o f -- python3 $B --steps 3 --warmup 1 --no-cpu-baseline > $R/gpurun_out/prof_fetch.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/prof_write -o w -- python3 $B --steps 3 --warmup 1 --no-cpu-baseline > $R/gpurun_out/prof_write.log 2>&1
