#!/bin/bash
# Large-document tier iteration: its GPU tests, then the C3 / C5 lines without CPU baselines.
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -v -m gpu -k "large_document or golden or fuzz" --timeout 300 --timeout-method thread > gpurun_out/big_tests.log 2>&1 && \
timeout -k 10 150 python -u bench.py --big c3 --no-cpu-baseline > gpurun_out/big_c3.log 2>&1 && \
timeout -k 10 150 python -u bench.py --big c5 --no-cpu-baseline > gpurun_out/big_c5.log 2>&1
