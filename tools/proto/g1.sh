set -o pipefail
mkdir -p gpurun_out
(cd tools/proto && for w in 4 8 16; do timeout -k 5 60 ./ldbench 1000000 3328 $w || exit 1; done) > gpurun_out/ldbench.log 2>&1 && \
timeout -k 10 300 python -u -m pytest tests/test_step2.py tests/test_snapshot.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t_step2.log 2>&1
