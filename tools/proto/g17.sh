set -o pipefail
R=$PWD; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/t_gpu_all.log 2>&1 && \
timeout -k 10 300 python -u bench.py --big c3full --no-yjs --no-cpu-baseline > gpurun_out/big_c3full.log 2>&1 && \
timeout -k 10 300 python -u bench.py --big c3 --no-yjs > gpurun_out/big_c3.log 2>&1 || exit 1
export TMPDIR=/tmp
for blk in c3full c5; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 400 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $R/gpurun_out/pmc_${blk}_$c -o p -- python3 bench.py --big $blk --no-yjs --no-cpu-baseline > $R/gpurun_out/pmc_${blk}_$c.log 2>&1 || exit 1
  done
done
