#!/bin/bash
# kernel-time probes of the main build and every build_exp/*.so (gpurun)
mkdir -p gpurun_out; : > gpurun_out/time.log
timeout -k 10 120 python -u tools/time_lean.py >> gpurun_out/time.log 2>&1 || exit $?
for so in build_exp/*.so; do
  YGM_LIB=$PWD/$so timeout -k 10 120 python -u tools/time_lean.py >> gpurun_out/time.log 2>&1 || exit $?
done
