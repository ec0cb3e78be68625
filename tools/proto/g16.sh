# round-4 measurement (tooling): validation-cap A/B; FETCH_SIZE / WRITE_SIZE passes of the C3 full and C5 blocks
set -o pipefail
R=$PWD; mkdir -p gpurun_out
for v in vcap256 vcap64; do
  YGM_LIB=$R/hocuspocus_amd/exp/libygm_$v.so timeout -k 10 300 python -u bench.py --big c3full --no-yjs --no-cpu-baseline > gpurun_out/big_c3full_$v.log 2>&1 || exit 1
done
export TMPDIR=/tmp
for blk in c3full c5; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 400 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $R/gpurun_out/pmc_${blk}_$c -o p -- python3 bench.py --big $blk --no-yjs --no-cpu-baseline > $R/gpurun_out/pmc_${blk}_$c.log 2>&1 || exit 1
  done
done
