#!/bin/bash
# Host-API check: every -m gpu test (the batch API now runs through the pinned two-stream pipeline),
# then the default bench line (host_api block included).
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 600 python -u bench.py --no-yjs > gpurun_out/bench.log 2>&1
