#!/bin/bash
# large-document probes (gpurun): bench --big c3 / c5 lines, k_merge_big phase stamps
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --big c3 > gpurun_out/big_c3.log 2>&1 && \
timeout -k 10 300 python -u bench.py --big c5 > gpurun_out/big_c5.log 2>&1 && \
timeout -k 10 120 python -u tools/diag_big.py c5 > gpurun_out/diag_c5.log 2>&1 && \
timeout -k 10 120 python -u tools/diag_big.py > gpurun_out/diag_c3.log 2>&1
