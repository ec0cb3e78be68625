set -o pipefail
mkdir -p gpurun_out
for v in vcap256 vcap64; do
  YGM_LIB=$PWD/hocuspocus_amd/exp/libygm_$v.so timeout -k 10 300 python -u bench.py --big c3full --no-yjs --no-cpu-baseline > gpurun_out/big_c3full_$v.log 2>&1 || exit 1
done
timeout -k 10 300 python -u bench.py --big c3full --no-yjs --no-cpu-baseline > gpurun_out/big_c3full.log 2>&1
