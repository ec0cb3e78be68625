# scan experiments (tooling): kernel traces of C3 full with experiment builds of the scan's verdict
set -o pipefail
R=$PWD; mkdir -p gpurun_out/g24; export TMPDIR=/tmp
for v in ${EXPS:-nov ascii}; do
  YGM_LIB=$R/hocuspocus_amd/exp/libygm_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/g24/$v -o k -- python3 bench.py --big c3full --no-yjs --no-cpu-baseline > $R/gpurun_out/g24/$v.log 2>&1 || exit 1
done
