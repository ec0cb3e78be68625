# round-4 probe (tooling): delete-set splice in the large-document tier -- parity, coverage, timing
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v -m gpu -k "large" --timeout 200 --timeout-method thread > gpurun_out/t_large.log 2>&1 && \
timeout -k 10 200 python -u tools/proto/big_probe.py splice > gpurun_out/big_splice.log 2>&1 && \
timeout -k 10 300 python -u tools/proto/big_probe.py > gpurun_out/big_probe.log 2>&1 && \
timeout -k 10 300 python -u tools/proto/big_probe.py diagds > gpurun_out/big_probe_ds.log 2>&1
