# round-6 final measurement, part 1 (tooling): GPU tests, smoke, the default bench line, its kernel trace
set -o pipefail
R=$PWD; mkdir -p gpurun_out/fin6
timeout -k 10 500 python -u -m pytest tests/ -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/fin6/gpu_tests.log 2>&1 && \
timeout -k 10 120 python -u -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/fin6/smoke.log 2>&1 && \
timeout -k 10 600 python -u bench.py > gpurun_out/fin6/bench.log 2>&1 && \
(export TMPDIR=/tmp; timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/fin6/kt -o kt -- python3 bench.py --no-cpu-baseline > $R/gpurun_out/fin6/kt_bench.log 2>&1)
