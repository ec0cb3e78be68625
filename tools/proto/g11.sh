# round-4 probe (tooling): parallel struct emit + register Any/JSON stacks -- all GPU tests, C3 / C5 blocks
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/t_gpu_all.log 2>&1 && \
OCC_DS=1 timeout -k 10 300 python -u tools/proto/big_probe.py occ > gpurun_out/big_occds.log 2>&1 && \
timeout -k 10 300 python -u bench.py --big c3full --no-yjs --no-cpu-baseline > gpurun_out/big_c3full.log 2>&1 && \
timeout -k 10 300 python -u bench.py --big c3 --no-yjs > gpurun_out/big_c3.log 2>&1 && \
timeout -k 10 300 python -u bench.py --big c5 --no-yjs > gpurun_out/big_c5.log 2>&1
