#!/bin/bash
# SQ counter passes over the C2 100k lean merge (gpurun): instruction mix, waits, issue activity.
mkdir -p gpurun_out && R=$PWD && cd /tmp && export TMPDIR=/tmp
B="$R/tools/exp_lean.py --child ${EXP_CORPORA:-c2_100k}"
rm -rf $R/gpurun_out/sql1 $R/gpurun_out/sql2
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-trace --output-format csv -d $R/gpurun_out/sql1 -o sq -- python3 $B > $R/gpurun_out/sql1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH SQ_INSTS_VMEM SQ_BUSY_CU_CYCLES SQ_LDS_BANK_CONFLICT --kernel-trace --output-format csv -d $R/gpurun_out/sql2 -o sq2 -- python3 $B > $R/gpurun_out/sql2.log 2>&1 && \
python3 $R/tools/sq_summary.py $R/gpurun_out/sql1 > $R/gpurun_out/sq_lean.txt && python3 $R/tools/sq_summary.py $R/gpurun_out/sql2 >> $R/gpurun_out/sq_lean.txt
