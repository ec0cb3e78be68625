#!/bin/bash
# instruction counters of every build_exp/*.so under tools/time_lean.py (gpurun)
mkdir -p gpurun_out && R=$PWD && cd /tmp && export TMPDIR=/tmp
for so in $R/build_exp/*.so; do
  n=$(basename $so .so)
  YGM_LIB=$so timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-trace --output-format csv -d $R/gpurun_out/prof_$n -o x -- python3 $R/tools/time_lean.py > $R/gpurun_out/prof_$n.log 2>&1 || exit $?
done
