# round-4 probe (tooling): C3 / C5 / C3 full-size blocks after the snapshot scan + delete-set splice
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --big c3 --no-yjs > gpurun_out/big_c3.log 2>&1 && \
timeout -k 10 300 python -u bench.py --big c5 --no-yjs > gpurun_out/big_c5.log 2>&1 && \
timeout -k 10 600 python -u bench.py --big c3full --no-yjs > gpurun_out/big_c3full.log 2>&1 && \
(export TMPDIR=/tmp; timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kt_c3 -o kt -- python3 bench.py --big c3 --no-yjs --no-cpu-baseline > gpurun_out/kt_c3.log 2>&1)
