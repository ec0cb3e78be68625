#!/bin/bash
# Update-V2 codec on the GPU: its parity tests, then the smoke test.
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_v2.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/v2_tests.log 2>&1
