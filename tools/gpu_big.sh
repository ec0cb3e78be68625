#!/bin/bash
# Large-document tier iteration (gpurun): large-document parity tests first, then every GPU parity test,
# k_merge_big phase stamps (C5, C3) and the C3 / C5 probes.  Each step has its own limit; the chain stops
# at the first failure.
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -x -v -m gpu --timeout 240 --timeout-method thread -k "large_document" > gpurun_out/gpu_big_tests.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 120 python -u tools/diag_big.py c5 > gpurun_out/diag_c5.log 2>&1 && \
timeout -k 10 120 python -u tools/diag_big.py > gpurun_out/diag_c3.log 2>&1 && \
timeout -k 10 300 python -u tools/bench_configs.py c3 2000 > gpurun_out/cfg_c3.log 2>&1 && \
timeout -k 10 300 python -u tools/bench_configs.py c5 20 > gpurun_out/cfg_c5.log 2>&1
