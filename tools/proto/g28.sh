# experiment (tooling): tools/proto/scan_successor_filter.patch as an experiment build -- large-tier tests, C3 full, C5
set -o pipefail
R=$PWD; mkdir -p gpurun_out/g28; export YGM_LIB=$R/hocuspocus_amd/exp/libygm_succ.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "large" --timeout 200 --timeout-method thread > gpurun_out/g28/t_large.log 2>&1 && \
timeout -k 10 300 python -u bench.py --big c3full --no-yjs --no-cpu-baseline > gpurun_out/g28/c3full.log 2>&1 && \
timeout -k 10 300 python -u bench.py --big c5 --big-docs 1000 --no-yjs --no-cpu-baseline > gpurun_out/g28/c5.log 2>&1
