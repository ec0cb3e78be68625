#!/bin/bash
# Jump-table chain follow in k_merge_big: all parity tests, phase stamps, the large-document lines.
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 120 python -u tools/diag_big.py c5 > gpurun_out/diag_big_c5.txt 2>&1 && \
timeout -k 10 120 python -u tools/diag_big.py c3 > gpurun_out/diag_big_c3.txt 2>&1 && \
bash tools/gpu_big_lines.sh
