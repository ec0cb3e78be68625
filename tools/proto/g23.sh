# large-document tier check (tooling): parity tests of the tier, C3 full / C5 blocks, a kernel trace of C3 full
set -o pipefail
R=$PWD; mkdir -p gpurun_out/g23; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "large" --timeout 200 --timeout-method thread > gpurun_out/g23/t_large.log 2>&1 && \
timeout -k 10 300 python -u bench.py --big c3full --no-yjs --no-cpu-baseline > gpurun_out/g23/c3full.log 2>&1 && \
timeout -k 10 300 python -u bench.py --big c5 --big-docs 1000 --no-yjs --no-cpu-baseline > gpurun_out/g23/c5.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/g23/kt -o k -- python3 bench.py --big c3full --no-yjs --no-cpu-baseline > $R/gpurun_out/g23/kt.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/g23/kt5 -o k -- python3 bench.py --big c5 --big-docs 1000 --no-yjs --no-cpu-baseline > $R/gpurun_out/g23/kt5.log 2>&1
