set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/proto/big_probe.py occ > gpurun_out/big_occ.log 2>&1 && \
(export TMPDIR=/tmp; timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_c3full -o kt -- python3 bench.py --big c3full --no-yjs --no-cpu-baseline > gpurun_out/kt_c3full.log 2>&1)
