#!/bin/bash
# large-document iteration (gpurun): GPU parity tests, tier probe, bench --big c3 / c5
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/t_par.log 2>&1 && \
timeout -k 10 200 python -u tools/probe_big.py > gpurun_out/probe_c3.log 2>&1 && \
timeout -k 10 300 python -u bench.py --big c3 > gpurun_out/big_c3.log 2>&1 && \
timeout -k 10 300 python -u bench.py --big c5 > gpurun_out/big_c5.log 2>&1
