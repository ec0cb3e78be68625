# round-5 closing check (tooling): every GPU test, smoke(), the default bench line on the last tree
set -o pipefail
mkdir -p gpurun_out/fin
timeout -k 10 400 python -u -m pytest tests/ -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/fin/gpu_tests_close.log 2>&1 && \
timeout -k 10 120 python -u -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/fin/smoke_close.log 2>&1 && \
timeout -k 10 600 python -u bench.py > gpurun_out/fin/bench_close.log 2>&1
