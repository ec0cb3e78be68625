#!/bin/bash
# All -m gpu tests, then the headline + update-V2 bench blocks.
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 400 python -u bench.py --c2big-docs 0 --c4-docs 0 --f1-docs 0 --no-host-api > gpurun_out/bench_v2.log 2>&1
