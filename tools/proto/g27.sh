# large-document tier check + block traffic (tooling): g23, then FETCH_SIZE / WRITE_SIZE passes of C3 full and C5
set -o pipefail
R=$PWD; export TMPDIR=/tmp
bash tools/proto/g23.sh || exit 1
mkdir -p gpurun_out/g27
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 400 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $R/gpurun_out/g27/pmc_c3full_$c -o p -- python3 bench.py --big c3full --no-yjs --no-cpu-baseline > $R/gpurun_out/g27/pmc_c3full_$c.log 2>&1 || exit 1
  timeout -s KILL 400 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $R/gpurun_out/g27/pmc_c5_$c -o p -- python3 bench.py --big c5 --big-docs 1000 --no-yjs --no-cpu-baseline > $R/gpurun_out/g27/pmc_c5_$c.log 2>&1 || exit 1
done
