#!/bin/bash
# Large-document tier: ContentAny attributes, the 10 MB document, tile edges; then the C3 / C5 lines.
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -v -m gpu -k "large_document" --timeout 300 --timeout-method thread > gpurun_out/big_tests.log 2>&1 && \
timeout -k 10 150 python -u bench.py --big c3 > gpurun_out/big_c3.log 2>&1 && \
timeout -k 10 150 python -u bench.py --big c5 > gpurun_out/big_c5.log 2>&1
