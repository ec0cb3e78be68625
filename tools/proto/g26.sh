# mid-size register budget experiments (tooling): C5 (1000 documents) and C3 full at 2 / 3 workgroups per CU
set -o pipefail
R=$PWD; mkdir -p gpurun_out/g26
for v in ${EXPS:-occ2 occ3}; do
  YGM_LIB=$R/hocuspocus_amd/exp/libygm_$v.so timeout -k 10 300 python -u bench.py --big c5 --big-docs 1000 --no-yjs --no-cpu-baseline > gpurun_out/g26/c5_$v.log 2>&1 || exit 1
  YGM_LIB=$R/hocuspocus_amd/exp/libygm_$v.so timeout -k 10 300 python -u bench.py --big c3full --no-yjs --no-cpu-baseline > gpurun_out/g26/c3_$v.log 2>&1 || exit 1
done
