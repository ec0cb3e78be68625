#!/bin/bash
# kernel-time probes of the main build and every build_exp/*.so (gpurun); EXP_TESTS=1 also runs the
# lean parity tests against each experiment build
mkdir -p gpurun_out; : > gpurun_out/time.log
timeout -k 10 120 python -u tools/time_lean.py >> gpurun_out/time.log 2>&1 || exit $?
for so in build_exp/*.so; do
  if [ -n "$EXP_TESTS" ]; then
    YGM_LIB=$PWD/$so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "lean or c2" --timeout 200 --timeout-method thread >> gpurun_out/time.log 2>&1 || exit $?
  fi
  YGM_LIB=$PWD/$so timeout -k 10 120 python -u tools/time_lean.py >> gpurun_out/time.log 2>&1 || exit $?
done
