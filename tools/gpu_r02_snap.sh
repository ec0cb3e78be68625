#!/bin/bash
# f-1 check: the Node extension's GPU tests (normalize included), then the snapshot documents-per-wave sweep.
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_node_extension.py tests/test_snapshot.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/t_node.log 2>&1 && \
bash tools/gpu_snap_dpw.sh
