# closing check (tooling): every GPU test, smoke(), the default bench line
set -o pipefail
mkdir -p gpurun_out/fin3
timeout -k 10 600 python -u -m pytest tests/ -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/fin3/gpu_tests.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/fin3/smoke.log 2>&1 && \
timeout -k 10 900 python -u bench.py > gpurun_out/fin3/bench.log 2>&1
