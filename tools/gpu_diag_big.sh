#!/bin/bash
# Phase stamps of k_merge_big (diagnostic build) on C5- and C3-shaped documents.
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/diag_big.py c5 > gpurun_out/diag_big_c5.txt 2>&1 && \
timeout -k 10 120 python -u tools/diag_big.py c3 > gpurun_out/diag_big_c3.txt 2>&1
