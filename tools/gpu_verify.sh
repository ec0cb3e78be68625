#!/bin/bash
# Full GPU verification of the tree (gpurun): parity tests, bench line, config probes (C2+del, C3, C4, C5),
# C3 / C5 next to the CPU oracle, rocprofv3 kernel-trace stats and FETCH_SIZE / WRITE_SIZE passes.  Each GPU step has its own limit and the
# chain stops at the first failure.
mkdir -p gpurun_out && R=$PWD
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > gpurun_out/bench.log 2>&1 && \
timeout -k 10 300 python -u tools/bench_configs.py c2del 100000 > gpurun_out/cfg_c2del.log 2>&1 && \
timeout -k 10 300 python -u tools/bench_configs.py c4 100000 > gpurun_out/cfg_c4.log 2>&1 && \
timeout -k 10 300 python -u tools/bench_configs.py c3 2000 > gpurun_out/cfg_c3.log 2>&1 && \
timeout -k 10 300 python -u tools/bench_configs.py c5 20 > gpurun_out/cfg_c5.log 2>&1 && \
timeout -k 10 150 python -u bench.py --big c3 > gpurun_out/big_c3.log 2>&1 && \
timeout -k 10 150 python -u bench.py --big c5 > gpurun_out/big_c5.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_kt -o kt -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline > $R/gpurun_out/prof_kt.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/prof_fetch -o f -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $R/gpurun_out/prof_fetch.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/prof_write -o w -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $R/gpurun_out/prof_write.log 2>&1
