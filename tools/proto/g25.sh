# routing threshold experiments (tooling): C5 (1000 documents) and C3 full with the 16-wave size from 256 / 512 KB
set -o pipefail
R=$PWD; mkdir -p gpurun_out/g25
for v in m256 m512; do
  YGM_LIB=$R/hocuspocus_amd/exp/libygm_$v.so timeout -k 10 300 python -u bench.py --big c5 --big-docs 1000 --no-yjs --no-cpu-baseline > gpurun_out/g25/c5_$v.log 2>&1 || exit 1
  YGM_LIB=$R/hocuspocus_amd/exp/libygm_$v.so timeout -k 10 300 python -u bench.py --big c3full --no-yjs --no-cpu-baseline > gpurun_out/g25/c3_$v.log 2>&1 || exit 1
done
