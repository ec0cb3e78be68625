# round-6 final measurement, part 2 (tooling): FETCH_SIZE / WRITE_SIZE passes (each its own run) of the default bench
# (lean, walkers), the C3 full / C5 / c5_store blocks and the f1 / c2_mixed / v2 side blocks
set -o pipefail
R=$PWD; mkdir -p gpurun_out/fin6
export TMPDIR=/tmp
p() {   # p TAG COUNTER LIMIT -- bench args
  local tag=$1 c=$2 lim=$3; shift 4
  timeout -s KILL $lim rocprofv3 --pmc $c --kernel-trace --output-format csv -d $R/gpurun_out/fin6/pmc_${tag}_$c -o p -- python3 bench.py "$@" > $R/gpurun_out/fin6/pmc_${tag}_$c.log 2>&1
}
for c in FETCH_SIZE WRITE_SIZE; do
  p bench $c 300 -- --no-cpu-baseline --no-c3 --c5-docs 0 --f1-docs 0 --no-mixed --no-v2 --store-docs 0 || exit 1
  p f1 $c 120 -- --block f1 --no-cpu-baseline || exit 1
  p mixed $c 120 -- --block mixed --no-cpu-baseline || exit 1
  p v2 $c 120 -- --block v2 --no-cpu-baseline || exit 1
  p c3full $c 200 -- --big c3full --no-yjs --no-cpu-baseline || exit 1
  p c5 $c 200 -- --big c5 --big-docs 1000 --no-yjs --no-cpu-baseline || exit 1
  p store $c 200 -- --block store --no-cpu-baseline || exit 1
done
