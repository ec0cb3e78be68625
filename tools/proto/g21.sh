set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u bench.py --no-cpu-baseline --c4-docs 0 > gpurun_out/bench_c3ctx.log 2>&1
