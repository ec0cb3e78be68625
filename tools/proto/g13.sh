set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "large or async or compact" --timeout 200 --timeout-method thread > gpurun_out/t_large.log 2>&1 && \
BIG_MB=0.3,1,3,10 timeout -k 10 300 python -u tools/proto/big_probe.py > gpurun_out/big_probe.log 2>&1 && \
timeout -k 10 300 python -u bench.py --big c3full --no-yjs --no-cpu-baseline > gpurun_out/big_c3full.log 2>&1 && \
(export TMPDIR=/tmp; timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_c3full -o kt -- python3 bench.py --big c3full --no-yjs --no-cpu-baseline > gpurun_out/kt_c3full.log 2>&1) && \
timeout -k 10 300 python -u tools/proto/big_probe.py tiers > gpurun_out/big_tiers.log 2>&1 && \
YGM_LIB=$PWD/hocuspocus_amd/exp/libygm_route1k.so timeout -k 10 300 python -u tools/proto/big_probe.py tiers >> gpurun_out/big_tiers.log 2>&1 && \
YGM_LIB=$PWD/hocuspocus_amd/exp/libygm_route512.so timeout -k 10 300 python -u tools/proto/big_probe.py tiers >> gpurun_out/big_tiers.log 2>&1 && \
YGM_LIB=$PWD/hocuspocus_amd/exp/libygm_noval.so timeout -k 10 300 python -u bench.py --big c3full --no-yjs --no-cpu-baseline > gpurun_out/big_c3full_noval.log 2>&1
