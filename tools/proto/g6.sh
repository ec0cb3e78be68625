# round-4 probe (tooling): large-document tier with the snapshot scan -- parity, timing
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v -m gpu -k "large" --timeout 200 --timeout-method thread > gpurun_out/t_large.log 2>&1 && \
timeout -k 10 300 python -u tools/proto/big_probe.py > gpurun_out/big_probe.log 2>&1 && \
timeout -k 10 300 python -u tools/proto/big_probe.py diag > gpurun_out/big_probe_diag.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/t_gpu_all.log 2>&1
