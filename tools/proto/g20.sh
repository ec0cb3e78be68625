set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --big c3full --no-yjs --no-cpu-baseline > gpurun_out/big_c3full.log 2>&1 && \
timeout -k 10 300 python -u bench.py --big c5 --big-docs 1000 --no-yjs --no-cpu-baseline > gpurun_out/big_c5k.log 2>&1 && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "large" --timeout 200 --timeout-method thread > gpurun_out/t_large.log 2>&1
