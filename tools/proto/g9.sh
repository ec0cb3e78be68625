# round-4 probe (tooling): large-document tier after the copy list / scan queue -- parity, C3 blocks, kernel split
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v -m gpu -k "large" --timeout 200 --timeout-method thread > gpurun_out/t_large.log 2>&1 && \
timeout -k 10 300 python -u tools/proto/big_probe.py occ > gpurun_out/big_occ.log 2>&1 && \
timeout -k 10 300 python -u bench.py --big c3 --no-yjs > gpurun_out/big_c3.log 2>&1 && \
(export TMPDIR=/tmp; timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_c3full -o kt -- python3 bench.py --big c3full --no-yjs --no-cpu-baseline > gpurun_out/kt_c3full.log 2>&1) && \
timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/t_gpu_all.log 2>&1
