#!/bin/bash
# Quick GPU iteration (gpurun): GPU parity tests, lean phase diagnostics, bench lines (main build, grid variants, build_exp/*.so).
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 120 python -u tools/diag_phases.py > gpurun_out/diag.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --cpu-seconds 4 > gpurun_out/bench.log 2>&1 || exit $?
for w in ${WPC_LIST:-}; do
  YGM_LEAN_WAVES_PER_CU=$w timeout -k 10 120 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_wpc$w.log 2>&1 || exit $?
done
for so in build_exp/*.so; do
  [ -e "$so" ] || continue
  YGM_LIB=$PWD/$so timeout -k 10 120 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_$(basename $so .so).log 2>&1 || exit $?
done
