set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v -m gpu -k "large" --timeout 200 --timeout-method thread > gpurun_out/t_large.log 2>&1 && \
timeout -k 10 300 python -u tools/proto/big_probe.py splice > gpurun_out/big_splice.log 2>&1 && \
timeout -k 10 300 python -u bench.py --big c3full --no-yjs --no-cpu-baseline > gpurun_out/big_c3full.log 2>&1 && \
timeout -k 10 300 python -u bench.py --big c3 --no-yjs > gpurun_out/big_c3.log 2>&1 && \
OCC_DS=1 timeout -k 10 300 python -u tools/proto/big_probe.py occ > gpurun_out/big_occds.log 2>&1
