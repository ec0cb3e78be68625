# round-4 final measurement, part 2 (tooling): FETCH_SIZE / WRITE_SIZE passes of the default bench (lean, walkers) and
# of the C3 full / C5 (1000 documents) blocks
set -o pipefail
R=$PWD; mkdir -p gpurun_out/fin
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 600 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $R/gpurun_out/fin/pmc_bench_$c -o p -- python3 bench.py --no-cpu-baseline --no-c3 --c5-docs 0 > $R/gpurun_out/fin/pmc_bench_$c.log 2>&1 || exit 1
done
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 400 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $R/gpurun_out/fin/pmc_c3full_$c -o p -- python3 bench.py --big c3full --no-yjs --no-cpu-baseline > $R/gpurun_out/fin/pmc_c3full_$c.log 2>&1 || exit 1
  timeout -s KILL 400 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $R/gpurun_out/fin/pmc_c5_$c -o p -- python3 bench.py --big c5 --big-docs 1000 --no-yjs --no-cpu-baseline > $R/gpurun_out/fin/pmc_c5_$c.log 2>&1 || exit 1
done
