# scan-kernel cost split (tooling): kernel traces of the C3 full block with the product library and two experiment
# builds (no validation in the scan; no parse at all)
set -o pipefail
R=$PWD; mkdir -p gpurun_out/g22; export TMPDIR=/tmp
for v in base noval noparse; do
  L=""; [ $v != base ] && L=$R/hocuspocus_amd/exp/libygm_$v.so
  YGM_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/g22/$v -o k -- python3 bench.py --big c3full --no-yjs --no-cpu-baseline > $R/gpurun_out/g22/$v.log 2>&1 || exit 1
done
