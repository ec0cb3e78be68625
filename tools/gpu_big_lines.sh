#!/bin/bash
# Large-document lines (GPU beside the C port and yjs): C3 (2 000 docs), C5 (20 XmlFragment docs), C3 at full size.
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --big c3 > gpurun_out/big_c3.log 2>&1 && \
timeout -k 10 300 python -u bench.py --big c5 > gpurun_out/big_c5.log 2>&1 && \
timeout -k 10 600 python -u bench.py --big c3full > gpurun_out/big_c3full.log 2>&1
