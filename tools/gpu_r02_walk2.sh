#!/bin/bash
# Walker iteration: SV / diff parity tests, C4 at 1M documents, lane census (diag build).
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 150 --timeout-method thread -k "walker or c4 or sv_diff or golden or fuzz or edge_states or empty" > gpurun_out/t_walk.log 2>&1 && \
timeout -k 10 300 python -u tools/bench_configs.py c4 1000000 > gpurun_out/c4_1m.log 2>&1 && \
timeout -k 10 300 python -u tools/diag_walk.py 1000000 > gpurun_out/diag_walk.log 2>&1
